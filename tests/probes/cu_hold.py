"""A persistent grid beside a kernel that holds k CUs (VERDICT r4 'Next' 3): under the Ulysses overlap
the all-to-alls run as RCCL kernels on a side stream, and the CUs they occupy are not available to a
persistent compute grid launched meanwhile.  On one GPU: `cu_hold` (tests/probes/fakecomm) keeps k
workgroups of 64 KB LDS resident for D microseconds on a side stream, a short delay on the compute
stream lets them land, then the measured kernel launches.  Per shape, the kernel's duration (HIP
events on its stream) with k = 0, 8, 16, 32 held CUs and D = about half its own time, XCD tile queues
vs the static per-CU lists (option queue), interleaved rounds.  Ideal (perfect balance): the
k = 0 time x 256 / (256 - k) while the hog runs; a static list instead waits for the held CU's
whole list (+ D).
usage: python tests/probes/cu_hold.py   (env: CH_K=0,8,16,32)"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "fakecomm", "libfakecomm.so"))
lib.cu_hold.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
lib.delay_us.argtypes = [ctypes.c_double, ctypes.c_void_p]

side = torch.cuda.Stream()
main = torch.cuda.current_stream()
ks = [int(x) for x in os.environ.get("CH_K", "0,8,16,32").split(",")]


def held(fn, k, d_us):
    """fn's duration (ms) on the main stream with k CUs held for d_us on the side stream."""
    torch.cuda.synchronize()
    if k:
        lib.cu_hold(k, d_us, ctypes.c_void_p(side.cuda_stream))
    lib.delay_us(20.0, ctypes.c_void_p(main.cuda_stream))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def case(name, fn, variants):
    base = {}
    for v, opts in variants.items():
        with K.options(**opts):
            fn()
            torch.cuda.synchronize()
            base[v] = min(held(fn, 0, 0) for _ in range(3))
    d_us = 500.0 * base[list(variants)[0]]         # about half the kernel's own time
    t = {(v, k): [] for v in variants for k in ks}
    for _ in range(3):
        for k in ks:
            for v, opts in variants.items():
                with K.options(**opts):
                    t[(v, k)].append(held(fn, k, d_us))
    for k in ks:
        s = "  ".join(f"{v} {min(t[(v, k)]):.3f} ms ({min(t[(v, k)]) / base[v]:.3f}x)" for v in variants)
        ideal = 1.0 if k == 0 else 256.0 / (256 - k)
        print(f"{name}: {k:2d} CUs held {d_us:.0f} us: {s}   (balanced ideal <= {ideal:.3f}x)", flush=True)


g = torch.Generator(device="cuda").manual_seed(1)
GEMM = {"queue": dict(queue=1), "static": dict(queue=0)}      # (the attention's item queues too)
# r6: split-tail pieces from the queue's piece pool (default) vs as workgroups of their own
GEMM_PIECES = {"queue": dict(queue=1, piece_queue=1), "queue_piece_blocks": dict(queue=1, piece_queue=0),
               "static": dict(queue=0)}
only = os.environ.get("CH_ONLY")          # e.g. "ffn-down" (a substring of the case names)
for M, N, Kd, epi, name in ((59280, 13824, 5120, K.VS_EPI_GELU, "ffn-up 59280"), (7410, 15360, 5120, K.VS_EPI_BIAS,
                            "q|k|v 7410 (SP=8 rows)"), (7410, 5120, 13824, K.VS_EPI_BIAS, "ffn-down 7410"),
                            (59280, 5120, 13824, K.VS_EPI_BIAS, "ffn-down 59280"),
                            (7410, 5120, 5120, K.VS_EPI_BIAS, "o-proj 7410")):
    if only and only not in name:
        continue
    a = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.bfloat16)
    b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    case(name, lambda: K.gemm(a, w, out, epilogue=epi, bias=b), GEMM_PIECES)
    del a, w, b, out
# self-attention at the SP = 8 rank shape (5 heads, full sequence) and at SP = 1
for H, name in ((5, "attention SP=8 (5 heads)"), (40, "attention SP=1 (40 heads)")):
    if only and only not in name:
        continue
    B, S = 2, 29640
    q, k_, v = (torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
    o = torch.empty_like(q)
    case(name, lambda: K.attention(q, k_, v, o, H, B), GEMM)
    del q, k_, v, o
