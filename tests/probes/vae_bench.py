"""Probe: Wan2.1 VAE tiled encode / decode at 832x480x73 on one MI355X (random weights).
Prints wall time, algorithmic TFLOP and TFLOP/s per call.  Usage: python tests/probes/vae_bench.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd")]
import torch  # noqa: E402

from oracle import wan_vae_oracle as V  # noqa: E402  (weights/shapes only)
from vstyler import vae  # noqa: E402


def main():
    frames, H, W = int(os.environ.get("VAE_T", 73)), int(os.environ.get("VAE_H", 480)), int(os.environ.get("VAE_W", 832))
    reps = int(os.environ.get("VAE_REPS", 2))
    m = vae.WanVideoVAE(device="cuda").load_state_dict(V.random_vae_weights(seed=6))
    g = torch.Generator(device="cuda").manual_seed(1)
    video = (torch.rand((1, 3, frames, H, W), generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    lat = None
    for it in range(reps + 1):
        vae.FLOPS[0] = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lat = m.encode(video, "cuda", tiled=True, tile_size=(30, 52), tile_stride=(15, 26))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"encode[{it}] {tuple(lat.shape)} {dt*1e3:.1f} ms  {vae.FLOPS[0]/1e12:.1f} TFLOP  "
              f"{vae.FLOPS[0]/dt/1e12:.0f} TF/s  peak mem {torch.cuda.max_memory_allocated()/2**30:.1f} GiB", flush=True)
    for it in range(reps + 1):
        vae.FLOPS[0] = 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = m.decode(lat, "cuda", tiled=True, tile_size=(30, 52), tile_stride=(15, 26))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"decode[{it}] {tuple(out.shape)} {dt*1e3:.1f} ms  {vae.FLOPS[0]/1e12:.1f} TFLOP  "
              f"{vae.FLOPS[0]/dt/1e12:.0f} TF/s  peak mem {torch.cuda.max_memory_allocated()/2**30:.1f} GiB", flush=True)
    u8 = vae.vae_output_to_u8(out[0])
    torch.cuda.synchronize()
    print("u8", tuple(u8.shape), u8.float().mean().item())


if __name__ == "__main__":
    main()
