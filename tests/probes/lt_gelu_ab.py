"""A/B: FFN-up GEMM + GELU as hipBLASLt (bias epilogue) + gemm_epi_apply8 GELU pass vs hipBLASLt's
fused GELU_BIAS epilogue (VS_LT_GELU=1).  Interleaved rounds in one process; numerics of both
against an fp64 GELU-tanh of the exact fp32-accumulated product.
  python tests/probes/lt_gelu_ab.py"""
import os, sys
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "video-styler_amd"))
import torch
from vstyler import kernels as K

dev = "cuda"
BF = torch.bfloat16


def gelu64(x):
    return 0.5 * x * (1 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


# numerics at a small shape (hipBLASLt route forced for it)
g = torch.Generator().manual_seed(0)
M, N, Kd = 512, 2048, 1024
a = torch.randn(M, Kd, generator=g).to(BF)
w = (torch.randn(N, Kd, generator=g) * 0.05).to(BF)
b = (torch.randn(N, generator=g) * 0.5).to(BF)
ref_pre = a.double() @ w.double().t() + b.double()
ref = gelu64(ref_pre)
ref_round_first = gelu64(ref_pre.to(BF).double())     # the reference: GELU of the bf16 linear output
os.environ["VS_GEMM_BACKEND"] = "lt"
res = {}
for mode in ("0", "1"):
    os.environ["VS_LT_GELU"] = mode
    out = torch.empty(M, N, dtype=BF, device=dev)
    K.gemm(a.to(dev), w.to(dev), out, epilogue=K.VS_EPI_GELU, bias=b.to(dev))
    torch.cuda.synchronize()
    o = out.cpu().double()
    res[mode] = o
    for name, r in (("fp64 exact", ref), ("reference rounding", ref_round_first)):
        rb = r.to(BF).double()
        ne = (o != rb).float().mean().item()
        rel = ((o - r).norm() / r.norm()).item()
        print(f"VS_LT_GELU={mode} vs {name}: {100 * ne:.2f}% differ from its bf16 rounding, rel-L2 {rel:.3e}, "
              f"max-abs {(o - r).abs().max().item():.3e}")
os.environ.pop("VS_GEMM_BACKEND")

# timing at the 14B FFN-up shape
M, N, Kd = 59280, 13824, 5120
a = torch.randn(M, Kd, device=dev, dtype=BF)
w = torch.randn(N, Kd, device=dev, dtype=BF) * 0.02
b = torch.randn(N, device=dev, dtype=BF) * 0.01
out = torch.empty(M, N, dtype=BF, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for mode in ("0", "1"):          # warm + autotune both plans
    os.environ["VS_LT_GELU"] = mode
    K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
torch.cuda.synchronize()
times = {"0": [], "1": []}
for r in range(6):
    for mode in ("0", "1"):
        os.environ["VS_LT_GELU"] = mode
        ev[0].record()
        for _ in range(5):
            K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
        ev[1].record()
        torch.cuda.synchronize()
        times[mode].append(ev[0].elapsed_time(ev[1]) / 5)
for mode in ("0", "1"):
    t = sorted(times[mode])
    fl = 2.0 * M * N * Kd
    print(f"VS_LT_GELU={mode}: FFN-up + GELU median {t[len(t) // 2]:.3f} ms min {t[0]:.3f} ms "
          f"({fl / t[len(t) // 2] / 1e9:.0f} TF/s incl. GELU)")
