"""A/B: the hand-written staggered 8-phase GEMM (8p), the 4-wave kernel with the XCD tile queues (w4)
or the static per-CU lists (w4s) and the hipBLASLt route (lt, + its epilogue pass), per 14B block
GEMM with its real epilogue; interleaved rounds, one process (AB_VARIANTS=w4,w4s,lt; lt only with
the A/B build loaded, VSTYLER_LIB=video-styler_amd/vstyler/lib/ab/libvstyler.so).
usage: gemm_ab.py [M ...]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K


# AB_FLUSH=1: overwrite a 1 GiB buffer before each timed launch (evicts L2 and the 256-MB Infinity
# Cache, as the step's other kernels do between one weight's uses), to price a kernel's cache reuse
FLUSH = torch.empty(1 << 29, dtype=torch.float16, device="cuda") if os.environ.get("AB_FLUSH") == "1" else None


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        if FLUSH is not None:
            FLUSH.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return min(ts)


SHAPES_1P3B = (("qkv", 4608, 1536, K.VS_EPI_BIAS), ("o-proj", 1536, 1536, K.VS_EPI_GATE_RES),
               ("ffn-up", 8960, 1536, K.VS_EPI_GELU), ("ffn-down", 1536, 8960, K.VS_EPI_GATE_RES))
SHAPES = (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_GATE_RES),
          ("ffn-up", 13824, 5120, K.VS_EPI_GELU), ("ffn-down", 5120, 13824, K.VS_EPI_GATE_RES),
          ("cross-o", 5120, 5120, K.VS_EPI_RES))
# the per-step context GEMMs (run with M = 1024: the CFG pair's 2 x 512 context rows)
SHAPES_CTX = (("ctx-kv", 10240, 4096, K.VS_EPI_BIAS), ("txt-emb0", 5120, 4096, K.VS_EPI_GELU),
              ("txt-emb2", 5120, 5120, K.VS_EPI_BIAS))
if os.environ.get("AB_MODEL") == "1.3B":     # the 1.3B model's block GEMMs (D 1536, F 8960)
    SHAPES = SHAPES_1P3B
elif os.environ.get("AB_MODEL") == "ctx":
    SHAPES = SHAPES_CTX
SHAPES = tuple(sh for sh in SHAPES if sh[0] in os.environ.get("AB_SHAPES", ",".join(x[0] for x in SHAPES)).split(","))
# lt needs the A/B build (make -C video-styler_amd/csrc ab; VSTYLER_LIB=.../lib/ab/libvstyler.so)
VARIANTS = [v for v in os.environ.get("AB_VARIANTS", "w4,w4s").split(",")]
for M in [int(v) for v in sys.argv[1:]] or (59280, 7410):
    for name, N, Kd, epi in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(1)
        a = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.bfloat16)
        b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
        gate = (0.1 * torch.randn(2, N, device="cuda", generator=g)).to(torch.bfloat16)
        x = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        kw = dict(epilogue=epi, bias=b)
        if epi == K.VS_EPI_GATE_RES:
            kw.update(residual=x, gate=gate, gate_bstride=N, rows_per_batch=(M + 1) // 2)
        if epi == K.VS_EPI_RES:
            kw.update(residual=x)
        out = x if epi in (K.VS_EPI_GATE_RES, K.VS_EPI_RES) else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def setv(v):       # lt (A/B build only) | 8p | w4 (4-wave, XCD tile queues) | w4s (4-wave, static
            # lists) | t128 (the 128x128 kernel) | auto (the product's own choice of schedule)
            os.environ["VS_GEMM_BACKEND"] = "lt" if v == "lt" else "own"     # read by the A/B build only
            K.set_option("gemm_tile", {"auto": 0, "t128": 128}.get(v, 256))
            K.set_option("gemm_kernel", 8 if v == "8p" else 4)
            K.set_option("queue", 0 if v == "w4s" else 1)
        t = {v: [] for v in VARIANTS}
        for v in VARIANTS:             # warm (hipBLASLt autotune happens here)
            setv(v); K.gemm(a, w, out, **kw); torch.cuda.synchronize()
        for r in range(4):
            for v in VARIANTS:
                setv(v); t[v].append(timed(lambda: K.gemm(a, w, out, **kw)))
        fl = 2.0 * M * N * Kd
        s = "  ".join(f"{v} {min(t[v]):.3f} ms ({fl / min(t[v]) / 1e9:.0f} TF/s)" for v in VARIANTS)
        print(f"M={M} {name:8s} N={N} K={Kd}: {s}", flush=True)
        del a, w, b, gate, x, out
os.environ.pop("VS_GEMM_BACKEND", None)
