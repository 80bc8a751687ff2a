"""fp8 e4m3 GEMM (fp8_linear semantics) at the 14B block shapes: the fp8 MFMA kernel vs hipBLASLt
(VS_FP8_BACKEND=lt, per-token scale vector), same process, with bit-equality of the two outputs."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K


def timeit(fn, reps=7):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return sorted(ts)[reps // 2]


for M in (59280, 7410):
    for name, N, Kd, epi in (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_GATE_RES),
                             ("ffn-up", 13824, 5120, K.VS_EPI_GELU), ("ffn-down", 5120, 13824, K.VS_EPI_GATE_RES)):
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
        w8 = w.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
        b = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
        gate = (0.1 * torch.randn(2, N, device="cuda")).to(torch.bfloat16)
        x0 = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        a8 = torch.empty(M, Kd, device="cuda", dtype=torch.uint8)
        sc = torch.empty(M, device="cuda", dtype=torch.float32)
        K.quant_fp8_rows(a, a8, sc)
        outs, t = {}, {}
        for be in ("vstyler", "lt"):
            os.environ["VS_FP8_BACKEND"] = be
            x = x0.clone()
            kw = dict(epilogue=epi, bias=b)
            if epi == K.VS_EPI_GATE_RES:
                kw.update(residual=x, gate=gate, gate_bstride=N, rows_per_batch=(M + 1) // 2)
                out = x
            else:
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            fn = lambda: K.gemm_fp8(a8, sc, w8, out, **kw)
            if epi == K.VS_EPI_GATE_RES:
                fn(); torch.cuda.synchronize(); outs[be] = out.clone(); out.copy_(x0)
                t[be] = timeit(fn)
            else:
                t[be] = timeit(fn); outs[be] = out.clone()
        fl = 2.0 * M * N * Kd
        d = (outs["lt"].float() - outs["vstyler"].float()).abs()
        print(f"M={M} {name:8s}: fp8 kernel {t['vstyler']:.3f} ms ({fl/t['vstyler']/1e9:.0f} TF/s)  hipBLASLt "
              f"{t['lt']:.3f} ms ({fl/t['lt']/1e9:.0f} TF/s)  equal {torch.equal(outs['lt'], outs['vstyler'])} "
              f"max-abs {d.max().item():.3g} mismatches {(d > 0).float().mean().item():.2e}", flush=True)
        del a, w, w8, b, gate, x0, a8, sc, outs
