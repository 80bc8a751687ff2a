"""A/B GEMM microbenchmark at the DiT shapes (random data, interleaved rounds in one process)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
shapes = [(59280, 5120, 5120), (59280, 13824, 5120), (59280, 5120, 13824), (59280, 1536, 1536), (59280, 8960, 1536)]
res = {}
for (M, N, Kd) in shapes:
    a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ref = (a.float() @ w.float().t() + b.float())
    def ours():
        K.gemm(a, w, out, bias=b)
    def blas():
        torch.nn.functional.linear(a, w, b)
    fl = 2.0 * M * N * Kd
    for name, fn in (("vstyler", ours), ("hipblaslt", blas)):
        fn(); torch.cuda.synchronize()
        times = []
        for r in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); e1.record(); torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        t = sorted(times)[len(times) // 2]
        print(f"{name:10s} M={M} N={N} K={Kd}: {t:8.3f} ms  {fl / t / 1e9:7.1f} TF/s", flush=True)
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    print(f"   rel-L2 vs fp32 ref {rel:.2e}", flush=True)
