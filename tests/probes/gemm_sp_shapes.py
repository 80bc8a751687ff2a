"""GEMM at the per-rank Ulysses-SP shapes of the 14B bench (M = 2*29640/p rows) for both tile kernels."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
for M in (7410, 14820, 29640):
    for (N, Kd) in ((5120, 5120), (15360, 5120), (13824, 5120), (5120, 13824)):
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        K.gemm(a, w, out); torch.cuda.synchronize(); ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); K.gemm(a, w, out); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
        t = sorted(ts)[2]
        print(f"M={M} N={N} K={Kd}: {t:.3f} ms {2.0*M*N*Kd/t/1e9:.1f} TF/s", flush=True)
