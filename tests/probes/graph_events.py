"""Probe: do external timing events captured inside a hipGraph (torch.cuda.CUDAGraph) record real
per-replay timestamps on ROCm?  Compares with eager event timing of the same kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd")]
import torch  # noqa: E402

from vstyler import kernels as K  # noqa: E402

B, S, H, D = 2, 8192, 8, 128
q = torch.randn(B * S, H * D, device="cuda").to(torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
o = torch.empty_like(q)
for _ in range(3):
    K.attention(q, k, v, o, H, B)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); K.attention(q, k, v, o, H, B); e1.record(); torch.cuda.synchronize()
print("eager ms", e0.elapsed_time(e1))
g = torch.cuda.CUDAGraph()
a0, a1 = torch.cuda.Event(enable_timing=True, external=True), torch.cuda.Event(enable_timing=True, external=True)
with torch.cuda.graph(g):
    K.attention(q, k, v, o, H, B)
    a0.record()
    K.attention(q, k, v, o, H, B)
    a1.record()
    K.attention(q, k, v, o, H, B)
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("graph replay", r, "ms", a0.elapsed_time(a1))
ref = o.clone()
K.attention(q, k, v, o, H, B)
torch.cuda.synchronize()
print("graph output equal eager:", torch.equal(ref, o))
