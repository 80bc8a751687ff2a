"""Split tail A/B in one process: GEMM (14B shapes at SP=1/2/8 rows) and self-attention
(SP=1: 40 heads, SP=8: 5 heads), each timed with and without the split (VS_*_NO_SPLIT)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K


def timed(fn, reps=5):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return sorted(ts)[reps // 2]


def ab(name, fn, env, flops):
    res = {}
    for mode in ("split", "nosplit", "split2"):
        if mode == "nosplit":
            os.environ[env] = "1"
        else:
            os.environ.pop(env, None)
        res[mode] = timed(fn)
    os.environ.pop(env, None)
    s = min(res["split"], res["split2"])
    print(f"{name}: split {s:.3f} ms ({flops / s / 1e9:.0f} TF/s)  nosplit {res['nosplit']:.3f} ms "
          f"({flops / res['nosplit'] / 1e9:.0f} TF/s)  gain {100 * (res['nosplit'] / s - 1):+.1f} %", flush=True)


for M in (59280, 14820, 7410):
    for (N, Kd) in ((5120, 5120), (15360, 5120), (13824, 5120), (5120, 13824)):
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ab(f"gemm M={M} N={N} K={Kd} plan={K.gemm_split_plan(M, N, Kd, 256)}", lambda: K.gemm(a, w, out),
           "VS_GEMM_NO_SPLIT", 2.0 * M * N * Kd)
        del a, w, out
B, S = 2, 29640
for H in (40, 5):
    D = H * 128
    q = torch.randn(B * S, D, device="cuda").to(torch.bfloat16)
    k = torch.randn(B * S, D, device="cuda").to(torch.bfloat16)
    v = torch.randn(B * S, D, device="cuda").to(torch.bfloat16)
    o = torch.empty_like(q)
    ab(f"attn H={H} plan={K.attention_split_plan(B, S, S, H, 256)}", lambda: K.attention(q, k, v, o, H, B),
       "VS_ATTN_NO_SPLIT", 4.0 * S * S * D * B)
    del q, k, v, o
