"""fp8 GEMM microbenchmark at the 14B DiT shapes (random data): quantisation + e4m3 GEMM vs bf16."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch  # noqa: E402

from vstyler import kernels as K  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


for (M, N, Kd) in [(59280, 5120, 5120), (59280, 13824, 5120), (59280, 5120, 13824)]:
    a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
    w8 = w.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    a8 = torch.empty(M, Kd, device="cuda", dtype=torch.uint8)
    sc = torch.empty(M, device="cuda", dtype=torch.float32)
    fl = 2.0 * M * N * Kd
    tq = timeit(lambda: K.quant_fp8_rows(a, a8, sc))
    tg = timeit(lambda: K.gemm_fp8(a8, sc, w8, out))
    tb = timeit(lambda: K.gemm(a, w, out))
    print(f"M={M} N={N} K={Kd}: quant {tq:.3f} ms ({M*Kd*3/tq/1e6:.0f} GB/s)  fp8 gemm {tg:.3f} ms "
          f"{fl/tg/1e9:.0f} TF/s  (+quant {fl/(tg+tq)/1e9:.0f})  bf16 gemm {tb:.3f} ms {fl/tb/1e9:.0f} TF/s", flush=True)
