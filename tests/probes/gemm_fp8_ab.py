"""A/B: the fp8 8-phase MFMA GEMM (VS_FP8_BACKEND=vstyler) vs hipBLASLt fp8 (lt), per 14B block GEMM
with its real epilogue (GELU on the two-pass rounding route); interleaved rounds in one process.
usage: gemm_fp8_ab.py [M ...]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K



def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return min(ts)


SHAPES = (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_GATE_RES),
          ("ffn-up", 13824, 5120, K.VS_EPI_GELU), ("ffn-down", 5120, 13824, K.VS_EPI_GATE_RES))
VARIANTS = os.environ.get("AB_VARIANTS", "w4,w4s").split(",")
for M in [int(v) for v in sys.argv[1:]] or (59280,):
    for name, N, Kd, epi in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(1)
        a = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
        w8 = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.float8_e4m3fn).view(torch.uint8)
        a8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
        sc = torch.empty(M, dtype=torch.float32, device="cuda")
        K.quant_fp8_rows(a, a8, sc)
        b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
        gate = (0.1 * torch.randn(2, N, device="cuda", generator=g)).to(torch.bfloat16)
        x = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        kw = dict(epilogue=epi, bias=b)
        if epi == K.VS_EPI_GATE_RES:
            kw.update(residual=x, gate=gate, gate_bstride=N, rows_per_batch=(M + 1) // 2)
        out = x if epi == K.VS_EPI_GATE_RES else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = {v: [] for v in VARIANTS}
        def setv(v):      # 8p = the 8-phase kernel, w4 / w4s = the 4-wave kernel (tile queues / static lists), lt = hipBLASLt fp8 (A/B build)
            os.environ["VS_GEMM_BACKEND"] = "lt" if v == "lt" else "own"     # read by the A/B build only
            K.set_option("gemm_kernel", 4 if v.startswith("w4") else 8)
            K.set_option("queue", 0 if v == "w4s" else 1)
        for v in VARIANTS:
            setv(v)
            K.gemm_fp8(a8, sc, w8, out, **kw); torch.cuda.synchronize()
        for r in range(4):
            for v in VARIANTS:
                setv(v)
                t[v].append(timed(lambda: K.gemm_fp8(a8, sc, w8, out, **kw)))
        fl = 2.0 * M * N * Kd
        print(f"fp8 M={M} {name:8s} N={N} K={Kd}: " +
              "  ".join(f"{v} {min(t[v]):.3f} ms ({fl / min(t[v]) / 1e9:.0f} TF/s)" for v in VARIANTS), flush=True)
        del a, w8, a8, sc, b, gate, x, out
os.environ.pop("VS_GEMM_BACKEND", None)
