"""Probe: the VAE AttentionBlock's flash kernel (vs_vae_attention) vs the fp32-score GEMM route, at the
pipeline's tile shapes (19 latent frames of a 30 x 52 tile, C = 384) and a whole 60 x 104 frame pair.
Times the kernel alone (HIP events) and the whole block, three interleaved rounds; algorithmic flops
4 * frames * pixels^2 * C (QK^T + P.V; the kernel's second QK^T pass not counted).
Usage: python tests/probes/vae_attn_ab.py"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd")]
import torch  # noqa: E402

from vstyler import _lib, vae  # noqa: E402

BF16 = torch.bfloat16


def timed(fn, reps=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    lib = _lib.load()
    c = 384
    g = torch.Generator().manual_seed(3)
    m = vae.WanVideoVAE(device="cuda")
    m.params = {"a.norm.gamma": (1 + 0.1 * torch.randn((c,), generator=g)).to(BF16).cuda()}
    m.cw = {"a.to_qkv.": vae.ConvW((torch.randn((3 * c, c, 1, 1), generator=g) / math.sqrt(c)).to(BF16),
                                   (0.1 * torch.randn((3 * c,), generator=g)).to(BF16), "cuda"),
            "a.proj.": vae.ConvW((torch.randn((c, c, 1, 1), generator=g) / math.sqrt(c)).to(BF16),
                                 (0.1 * torch.randn((c,), generator=g)).to(BF16), "cuda")}
    st = torch.cuda.current_stream().cuda_stream
    for (t, h, w) in ((19, 30, 52), (2, 60, 104), (19, 60, 104)):
        hw = h * w
        x = torch.randn((1, t, h, w, c), generator=g).to(BF16).cuda()
        qkv = torch.randn((t, hw, 3 * c), generator=g).to(BF16).cuda()
        o = torch.empty((t, hw, c), dtype=BF16, device="cuda")
        flops = 4.0 * t * hw * hw * c
        a = m._attn_block(x, "a.", flash=True)
        b = m._attn_block(x, "a.", flash=False)
        d = (a.float() - b.float())
        print(f"[{t}x{h}x{w}] block flash vs gemm route: max-abs {d.abs().max().item():.4g} "
              f"rel-L2 {(d.norm() / b.float().norm()).item():.3g}", flush=True)
        for r in range(3):
            k_ms = timed(lambda: _lib.check(lib.vs_vae_attention(qkv.data_ptr(), hw * 3 * c, 3 * c, o.data_ptr(), hw * c,
                                                                 c, t, hw, c, st)))
            bf = timed(lambda: m._attn_block(x, "a.", flash=True))
            bg = timed(lambda: m._attn_block(x, "a.", flash=False))
            print(f"[{t}x{h}x{w}] round {r}: kernel {k_ms:.3f} ms = {flops / k_ms / 1e9:.0f} TF/s; block flash "
                  f"{bf:.3f} ms, gemm route {bg:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
