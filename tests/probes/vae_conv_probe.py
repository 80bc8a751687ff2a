"""Probe: where the VAE conv's time goes.  The dominant launch of the 832x480x73 VAE (NB = 3: a 3x3x3
CausalConv3d 96 -> 96 channels on a 240x416 tile, 71 % of the VAE kernel time, profiles/r5/
kernel_stats_vae_r5s7.csv) against the same kernel in its plain-GEMM mode at the same K = 27 * 96 and
N = 96 (contiguous A rows, no im2col gather, no padding predicates), and a 1x1x1 conv (the gather
without taps).  Per case: ms per launch (HIP events, median of 5), TF/s, and for each VS_OPT_VAE_PXB
/ VAE_PRE variant; the patch-resident halo kernel (VS_OPT_VAE_HALO) against the per-tap one.  usage: python tests/probes/vae_conv_probe.py   (env: VCP_T frames, default 21)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd")]
import torch  # noqa: E402

from vstyler import kernels as K  # noqa: E402
from vstyler import vae  # noqa: E402

BF16 = torch.bfloat16


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def main():
    T, H, W, C = int(os.environ.get("VCP_T", 21)), 240, 416, 96
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.randn((1, T, H, W, C), generator=g, device="cuda")).to(BF16)
    w3 = (0.03 * torch.randn((C, C, 3, 3, 3), generator=g, device="cuda")).to(BF16)
    b = (0.1 * torch.randn((C,), generator=g, device="cuda")).to(BF16)
    cw3 = vae.ConvW(w3, b, "cuda")
    w1 = (0.1 * torch.randn((C, C, 1, 1, 1), generator=g, device="cuda")).to(BF16)
    cw1 = vae.ConvW(w1, b, "cuda")
    M = T * H * W
    y = torch.empty((1, T, H, W, C), dtype=BF16, device="cuda")
    # plain GEMM at K = 27 * 96 over M / 8 rows (A of M/8 x 2592 = the gathered operand, laid out flat)
    Mg = M // 8
    a = torch.randn((Mg, 27 * C), generator=g, device="cuda").to(BF16)
    wg = cw3.w.reshape(C, -1)
    yg = torch.empty((Mg, C), dtype=BF16, device="cuda")

    def conv3():
        vae.conv(x, cw3, (T, H, W), pad=(2, 1, 1), y=y)

    def conv1():
        vae.conv(x, cw1, (T, H, W), y=y)

    def gemm():
        vae.batched_gemm(a, 0, 27 * C, Mg, 27 * C, wg, 0, wg.shape[1], C, yg, 0, C, 1)

    for halo in (1, 0, 1, 0):
        with K.options(vae_halo=halo):
            ms = timed(conv3)
            print(f"halo {halo}  conv3x3x3 {ms:8.3f} ms  {2.0 * M * C * C * 27 / ms / 1e9:7.1f} TF/s", flush=True)
    if os.environ.get("VCP_HALO_ONLY"):
        return
    for pxb, pre in ((2, 3), (2, 2), (1, 3), (1, 2)):
        with K.options(vae_pxb=pxb, vae_pre=pre, vae_halo=0):
            for name, fn, flop in (("conv3x3x3", conv3, 2.0 * M * C * C * 27), ("gemm K=2592", gemm, 2.0 * Mg * C * C * 27),
                                   ("conv1x1x1", conv1, 2.0 * M * C * C)):
                ms = timed(fn)
                print(f"pxb {pxb} pre {pre}  {name:12s} {ms:8.3f} ms  {flop / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
