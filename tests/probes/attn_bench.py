"""Attention microbenchmark at the 14B 832x480x73 shapes (random data), + spot parity vs fp32.
ATTN_AB="8,4": interleaved rounds of VS_ATTN_IMPL values in one process (8: the 8-wave kernel,
4: attn_fwd_w4)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, H, L = 2, 29640, 40, 512
D = H * 128
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
k = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
v = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty_like(q)
kc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
vc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
impls = os.environ.get("ATTN_AB", "").split(",") if os.environ.get("ATTN_AB") else [None]
cases = [(name, kk, vv, skv, impl) for _ in range(2 if impls[0] is not None else 1) for impl in impls
         for name, kk, vv, skv in (("self", k, v, S), ("cross", kc, vc, L))]
for name, kk, vv, skv, impl in cases:
    if impl is not None:
        K.set_option("attn_impl", int(impl))
    fn = lambda: K.attention(q, kk, vv, o, H, B)
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts)[2]
    fl = 4.0 * S * skv * D * B
    # spot parity: 64 query rows of batch 1, heads 0 and 39
    rows = torch.arange(0, S, S // 64)[:64]
    worst = 0.0
    for hh in (0, 39):
        qs = q.view(B, S, H, 128)[1, rows, hh].float()
        ks = kk.view(B, skv, H, 128)[1, :, hh].float()
        vs = vv.view(B, skv, H, 128)[1, :, hh].float()
        ref = torch.softmax(qs @ ks.t() / 128 ** 0.5, -1) @ vs
        got = o.view(B, S, H, 128)[1, rows, hh].float()
        worst = max(worst, (got - ref).abs().max().item())
    print(f"{name}{'' if impl is None else ' impl ' + impl}: {t:.3f} ms  {fl / t / 1e9:.1f} TF/s  spot max-abs {worst:.3e}", flush=True)
