"""Probe: the HBM read+write ceiling at the row kernels' size (59 280 x 5120 bf16 in, same out):
torch copy_, and the library's LayerNorm+modulate for comparison."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "video-styler_amd"))
import torch  # noqa: E402
from vstyler import kernels as K  # noqa: E402

B, S, D = 2, 29640, 5120
x = torch.randn(B * S, D, device="cuda").to(torch.bfloat16)
h = torch.empty_like(x)
big = torch.empty(4 * B * S, D, device="cuda", dtype=torch.bfloat16)
mod = (0.1 * torch.randn(B, 6, D, device="cuda")).to(torch.bfloat16)


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


byt = 2 * x.numel() * 2
for r in range(3):
    c = timed(lambda: h.copy_(x))
    c4 = timed(lambda: big[:2 * B * S].copy_(big[2 * B * S:]))
    ln = timed(lambda: K.layernorm_modulate(x, h, 1e-6, shift=mod[:, 0], scale=mod[:, 1], mod_bstride=6 * D,
                                            rows_per_batch=S))
    print(f"round {r}: copy_ {c:.1f} us {byt / c / 1e6:.2f} TB/s; 2x copy_ {c4:.1f} us {2 * byt / c4 / 1e6:.2f} TB/s; "
          f"LN+modulate {ln:.1f} us {byt / ln / 1e6:.2f} TB/s", flush=True)
