"""fp8_linear's per-row activation quantisation (vs_quant_fp8_rows) at the 14B config-5 shapes: the
q|k|v / o / FFN-up inputs (59 280 x 5120) and the FFN-down input (59 280 x 13 824).  HBM rate =
(bf16 read + fp8 write) / time."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
g = torch.Generator(device="cuda").manual_seed(0)
for M, N in ((59280, 5120), (59280, 13824)):
    x = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    x8 = torch.empty(M, N, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    fn = lambda: K.quant_fp8_rows(x, x8, sc)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"quant {M}x{N}: {ms * 1e3:.1f} us  {3 * x.numel() / ms / 1e9:.2f} TB/s", flush=True)
    del x, x8
