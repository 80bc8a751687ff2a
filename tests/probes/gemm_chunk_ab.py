"""Does splitting a block GEMM into row chunks (each call's A chunk + W resident in the 256 MB
Infinity Cache) change its time on hipBLASLt?  14B shapes at M = 2 x 29640, interleaved rounds.
  python tests/probes/gemm_chunk_ab.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
BF = torch.bfloat16
M = 59280
shapes = {"qkv": (15360, 5120), "o": (5120, 5120), "ffn_up": (13824, 5120), "ffn_down": (5120, 13824)}
g = torch.Generator(device="cuda").manual_seed(0)
res = {}
for name, (N, Kd) in shapes.items():
    a = torch.randn(M, Kd, device="cuda", generator=g, dtype=torch.float32).to(BF)
    w = (0.02 * torch.randn(N, Kd, device="cuda", generator=g)).to(BF)
    b = (0.01 * torch.randn(N, device="cuda", generator=g)).to(BF)
    out = torch.empty(M, N, device="cuda", dtype=BF)
    for chunks in (1, 2, 4, 8):
        rows = M // chunks
        def run():
            for c in range(chunks):
                K.gemm(a[c * rows:(c + 1) * rows], w, out[c * rows:(c + 1) * rows], bias=b)
        run(); torch.cuda.synchronize()         # plan + autotune
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); run(); run(); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 2)
        ts.sort()
        fl = 2.0 * M * N * Kd
        print(f"{name:9s} chunks={chunks}: median {ts[2]:.3f} ms min {ts[0]:.3f} = {fl / ts[2] / 1e9:.0f} TF/s", flush=True)
    del a, w, out
