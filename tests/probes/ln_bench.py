"""LayerNorm(+modulate) at the 14B step shape: 2 x 29 640 rows x 5120, HBM rate (read x + write h)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, D = 2, 29640, 5120
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
h = torch.empty_like(x)
mod = (0.1 * torch.randn(B, 6, D, device="cuda", generator=g)).to(torch.bfloat16)
w = torch.ones(D, device="cuda", dtype=torch.bfloat16)
b = torch.zeros(D, device="cuda", dtype=torch.bfloat16)
fns = {"modulate": lambda: K.layernorm_modulate(x, h, 1e-6, shift=mod[:, 0], scale=mod[:, 1], mod_bstride=6 * D,
                                                rows_per_batch=S),
       "affine": lambda: K.layernorm_modulate(x, h, 1e-6, weight=w, bias=b)}
for name, fn in fns.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"layernorm {name}: {ms * 1e3:.1f} us  {2 * x.numel() * 2 / ms / 1e9:.2f} TB/s", flush=True)
