"""Probe: the VAE channel RMS norm + SiLU (vs_vae_rmsnorm) at the tiled 832x480 VAE's shapes -- HBM
rate of read x + write y.  usage: python tests/probes/vae_rmsnorm_bench.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import vae
g = torch.Generator(device="cuda").manual_seed(0)
for npix, c in ((21 * 240 * 416, 96), (21 * 120 * 208, 192), (21 * 60 * 104, 384)):
    x = torch.randn(npix, c, device="cuda", generator=g).to(torch.bfloat16)
    gam = (1 + 0.1 * torch.randn(c, device="cuda", generator=g)).to(torch.bfloat16)
    y = torch.empty_like(x)
    fn = lambda: vae.rmsnorm(x, gam, True, out=y)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"vae_rmsnorm {npix} x {c}: {ms * 1e3:.1f} us  {2 * x.numel() * 2 / ms / 1e9:.2f} TB/s", flush=True)
