"""hipBLASLt route per 14B block GEMM (real epilogues) at the SP=1 / SP=8 row counts; run once with
VS_LT_TUNE=0 (heuristic's first algorithm) and once with the default autotune to compare."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K

os.environ["VS_GEMM_BACKEND"] = "lt"


def timed(fn, reps=7):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return sorted(ts)[reps // 2]


tag = "tuned" if os.environ.get("VS_LT_TUNE", "1") != "0" else "heuristic"
for M in (59280, 7410):
    for name, N, Kd, epi in (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_GATE_RES),
                             ("cross-q", 5120, 5120, K.VS_EPI_BIAS), ("cross-o", 5120, 5120, K.VS_EPI_RES),
                             ("ffn-up", 13824, 5120, K.VS_EPI_GELU), ("ffn-down", 5120, 13824, K.VS_EPI_GATE_RES)):
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
        b = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
        gate = (0.1 * torch.randn(2, N, device="cuda")).to(torch.bfloat16)
        x = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        kw = dict(epilogue=epi, bias=b)
        if epi == K.VS_EPI_GATE_RES:
            kw.update(residual=x, gate=gate, gate_bstride=N, rows_per_batch=(M + 1) // 2)
        elif epi == K.VS_EPI_RES:
            kw.update(residual=x, alpha=1.0)
        out = x if epi in (K.VS_EPI_GATE_RES, K.VS_EPI_RES) else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = timed(lambda: K.gemm(a, w, out, **kw))
        fl = 2.0 * M * N * Kd
        print(f"{tag} M={M} {name:8s} N={N} K={Kd}: {t:.3f} ms ({fl/t/1e9:.0f} TF/s)", flush=True)
        del a, w, b, gate, x, out
