"""Generates tests/golden/*.npz from the CPU oracle (oracle/wan_oracle.py).

The reference could not be executed here (denied) and ships no vectors, so these
fixtures are the oracle's own outputs on seeded synthetic inputs: they pin the GPU path (and the
oracle itself) against drift.  bf16 tensors are stored as uint16 bit patterns.
Run:  python tests/golden/make_golden.py [tiny|c1|ops|vae480|all]
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import wan_oracle as O  # noqa: E402

torch.set_num_threads(os.cpu_count())


def u16(t):
    return t.contiguous().view(torch.int16).numpy().view(np.uint16)


def run_denoise(name, cfg, frames, height, width, steps, num_layers=None):
    c = dict(cfg)
    if num_layers is not None:
        c["num_layers"] = num_layers
    W = O.random_weights(c, seed=5)
    lat, cp, cn, vc = O.synthetic_inputs(c, frames, height, width)
    t0 = time.time()
    out = O.denoise(W, c, lat, cp, cn, vc, num_inference_steps=steps)
    dt = time.time() - t0
    t1 = O.set_timesteps(steps)[1][:1].to(torch.bfloat16)
    v1 = O.model_fn(W, c, lat, t1, cp, vc)
    # noise floor: the same computation with fp64 accumulation (a different, equally valid rounding)
    O.ACC_DTYPE = torch.float64
    out64 = O.denoise(W, c, lat, cp, cn, vc, num_inference_steps=steps)
    v1_64 = O.model_fn(W, c, lat, t1, cp, vc)
    O.ACC_DTYPE = torch.float32

    def floor(a, b):
        d = a.float() - b.float()
        return [d.abs().max().item(), (d.norm() / b.float().norm()).item()]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), latents_in=u16(lat), latents_out=u16(out),
                        v_first=u16(v1), steps=steps, frames=frames, height=height, width=width,
                        num_layers=c["num_layers"], noise_latents=np.array(floor(out64, out)),
                        noise_v_first=np.array(floor(v1_64, v1)))
    print(f"{name}: noise floor latents {floor(out64, out)}, v_first {floor(v1_64, v1)}")
    print(f"{name}: denoise {steps} steps in {dt:.1f}s, |out|={out.float().abs().mean():.4f}")


def run_ops():
    g = torch.Generator().manual_seed(11)
    B, S, H, D = 2, 300, 2, 256
    q = torch.randn(B, S, D, generator=g).to(torch.bfloat16)
    k = torch.randn(B, S, D, generator=g).to(torch.bfloat16)
    v = torch.randn(B, S, D, generator=g).to(torch.bfloat16)
    o = O.attention(q, k, v, H)
    x = (3 * torch.randn(B * S, D, generator=g)).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
    freqs = O.rope_freqs(3, 10, 10)
    rn = O.rope_apply(O.rms_norm(x.view(B, S, D), w), freqs, H)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), q=u16(q), k=u16(k), v=u16(v), attn=u16(o), x=u16(x), w=u16(w),
                        rmsnorm_rope=u16(rn))
    print("ops: written")


def run_vae480():
    """The causal VAE's tiled encode + decode at 480x832 (5 frames: two latent frames, the causal cache
    path) with the real 3x3 grid of 30x52-latent tiles (stride 15x26, wan_video_vae.py:1103-1203) at
    the Wan2.1 widths, random weights (seed 31): the oracle's fp32 outputs and their fp32/fp64 noise
    floor, for tests/test_production_c4c5_gpu.py (the host convolutions take minutes, so the GPU tier
    compares against these).  The decode is stored at every 8th output row (all frames, channels,
    columns: every tile row and both vertical seams of each tile column)."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    from oracle import wan_vae_oracle as V
    from vae_util import synthetic_video
    W = V.random_vae_weights(seed=31)
    video = synthetic_video(5, 480, 832)
    ts, st = (30, 52), (15, 26)

    def floor(a, b):
        d = a.float() - b.float()
        return [d.abs().max().item(), (d.norm() / b.float().norm()).item()]

    def both(fn):
        r32 = fn()
        O.ACC_DTYPE = torch.float64
        try:
            r64 = fn()
        finally:
            O.ACC_DTYPE = torch.float32
        return r32, r64
    t0 = time.time()
    enc, enc64 = both(lambda: V.tiled_encode(video, W, ts, st))
    dec, dec64 = both(lambda: V.tiled_decode(enc, W, ts, st))
    rows = slice(0, None, 8)
    np.savez_compressed(os.path.join(HERE, "vae_480x832.npz"), enc=u16(enc), dec_rows8=u16(dec[..., rows, :]),
                        noise_enc=np.array(floor(enc64, enc)),
                        noise_dec_rows8=np.array(floor(dec64[..., rows, :], dec[..., rows, :])),
                        video_sum=np.array(video.float().sum().item()),
                        weight_sum=np.array(sum(v.float().sum().item() for v in W.values())))
    print(f"vae480: enc {tuple(enc.shape)} floor {floor(enc64, enc)}, dec {tuple(dec.shape)} floor "
          f"{floor(dec64, dec)} ({time.time() - t0:.0f} s)")


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("ops", "all"):
        run_ops()
    if which in ("tiny", "all"):
        run_denoise("tiny_2step", O.WAN_CONFIGS["tiny"], 5, 128, 128, 2)
    if which in ("vae480", "all"):
        run_vae480()
    if which in ("c1", "all"):
        # BASELINE config 0 ("C1"): random-init 1.3B-shape DiT+VACE, 2 Euler steps, 5 frames 128x128
        run_denoise("c1_1p3b_2step", O.WAN_CONFIGS["1.3B"], 5, 128, 128, 2)
