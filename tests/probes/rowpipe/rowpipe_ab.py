"""Probe: persistent software-pipelined LayerNorm+modulate (rowpipe.hip) vs the library's one-block-per-row
kernel at the 14B step shape (2 x 29 640 rows x 5120): bit-identity and HBM rate, interleaved rounds."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "video-styler_amd"))
import torch  # noqa: E402
from vstyler import kernels as K  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "librowpipe.so"))
lib.rowpipe_ln.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong,
                           ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
B, S, D = 2, 29640, 5120
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
h0, h1 = torch.empty_like(x), torch.empty_like(x)
mod = (0.1 * torch.randn(B, 6, D, device="cuda", generator=g)).to(torch.bfloat16)
st = torch.cuda.current_stream().cuda_stream


def ref():
    K.layernorm_modulate(x, h0, 1e-6, shift=mod[:, 0], scale=mod[:, 1], mod_bstride=6 * D, rows_per_batch=S)


def pipe(blocks, wps):
    def f():
        rc = lib.rowpipe_ln(x.data_ptr(), D, h1.data_ptr(), D, B * S, D, S, mod[:, 0].data_ptr(),
                            mod[:, 1].data_ptr(), 6 * D, 1e-6, blocks, wps, st)
        assert rc == 0
    return f


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


ref()
variants = {f"pipe {b}x{w}": pipe(b, w) for b in (1024, 2048, 3072, 4096, 8192) for w in (1, 2, 4)}
for name, fn in variants.items():
    h1.zero_()
    fn()
    torch.cuda.synchronize()
    same = torch.equal(h0, h1)
    print(f"{name}: bit-identical {same}", flush=True)
    if not same:
        sys.exit(1)
byt = 2 * x.numel() * 2
for r in range(3):
    us = timed(ref)
    line = [f"lib {us:.1f} us {byt / us / 1e6:.2f} TB/s"]
    for name, fn in variants.items():
        us = timed(fn)
        line.append(f"{name} {us:.1f}")
    print(f"round {r}: " + ", ".join(line), flush=True)
