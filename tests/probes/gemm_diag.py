"""Times the 14B block GEMMs at 59 280 rows on whichever libvstyler.so VSTYLER_LIB names (diagnostic
builds of scripts/build_diag.sh: results are garbage there, only the time counts).
usage: VSTYLER_LIB=... python tests/probes/gemm_diag.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K

M = int(os.environ.get("GD_M", "59280"))
SHAPES = (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("ffn-up", 13824, 5120, K.VS_EPI_GELU),
          ("ffn-down", 5120, 13824, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_BIAS))
only = os.environ.get("GD_SHAPES")
for name, N, Kd, epi in SHAPES:
    if only and name not in only.split(","):
        continue
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = lambda: K.gemm(a, w, out, epilogue=epi, bias=b)
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = min(ts)
    print(f"{os.path.basename(os.path.dirname(os.environ.get('VSTYLER_LIB', 'lib/x')))} {name} {M}x{N}x{Kd}: "
          f"{t:.3f} ms {2 * M * N * Kd / t / 1e9:.0f} TF/s", flush=True)
    del a, w, b, out
