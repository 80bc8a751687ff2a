"""Self-attention at the 14B 1280x720x121 shape (S = 111600, B = 2, 40 heads) with q/k/v as column
slices of a fused [B*S, 3D] buffer (the model's layout: the K/V slab exceeds 2^31 bytes, so the
rebased-descriptor kernel runs), random data."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, H = 2, 111600, 40
D = H * 128
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(B * S, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty(B * S, D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
fn = lambda: K.attention(q, k, v, o, H, B)
fn(); torch.cuda.synchronize()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
t = sorted(ts)[1]
print(f"self S=111600 (rebased): {t:.2f} ms  {4.0 * S * S * D * B / t / 1e9:.1f} TF/s", flush=True)
