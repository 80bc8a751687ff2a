"""Cross-attention (14B 832x480x73: 2 x 29640 queries, 512 keys, 40 heads) and self-attention
timing of the library named by VSTYLER_LIB (or the default), for same-box variant A/B runs.
  VSTYLER_LIB=... python tests/probes/cross_ab.py [self]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, H, L = 2, 29640, 40, 512
D = H * 128
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
kc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
vc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty_like(q)
cases = [("cross", kc, vc, L, 30)]
if len(sys.argv) > 1:
    k = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
    cases.append(("self", k, v, S, 3))
tag = os.path.basename(os.path.dirname(os.environ.get("VSTYLER_LIB", "/default/x")))
for name, kk, vv, skv, reps in cases:
    K.attention(q, kk, vv, o, H, B)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            K.attention(q, kk, vv, o, H, B)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    ts.sort()
    fl = 4.0 * S * skv * D * B
    print(f"{tag:>10} {name}: median {ts[2]:.3f} ms min {ts[0]:.3f} ms = {fl / ts[2] / 1e9:.1f} TF/s", flush=True)
