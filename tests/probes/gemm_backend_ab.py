"""vs_gemm MFMA kernels vs the hipBLASLt route, per block GEMM of the 14B model (with its real
epilogue), at the SP=1 and SP=8 row counts; same process, interleaved."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K


def timed(fn, reps=5):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    return sorted(ts)[reps // 2]


# "ctx": the per-step context GEMMs (fused cross k|v over the CFG batch's 2 x 512 context rows)
CTX = sys.argv[1:2] == ["ctx"]
SHAPES = ((("cross-kv", 10240, 5120, K.VS_EPI_BIAS), ("text-1", 5120, 4096, K.VS_EPI_GELU),
           ("text-2", 5120, 5120, K.VS_EPI_BIAS), ("t5-attn", 4096, 4096, K.VS_EPI_BIAS),
           ("t5-ffn", 10240, 4096, K.VS_EPI_BIAS), ("time-proj", 30720, 5120, K.VS_EPI_BIAS),
           ("1.3B-kv", 3072, 1536, K.VS_EPI_BIAS)) if CTX else
          (("qkv", 15360, 5120, K.VS_EPI_BIAS), ("o-proj", 5120, 5120, K.VS_EPI_GATE_RES),
           ("cross-q", 5120, 5120, K.VS_EPI_BIAS), ("cross-o", 5120, 5120, K.VS_EPI_RES),
           ("ffn-up", 13824, 5120, K.VS_EPI_GELU), ("ffn-down", 5120, 13824, K.VS_EPI_GATE_RES)))
for M in (1024, 512, 2) if CTX else ([int(v) for v in sys.argv[1:]] or (59280, 7410)):
    for name, N, Kd, epi in SHAPES:
        a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
        b = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
        gate = (0.1 * torch.randn(2, N, device="cuda")).to(torch.bfloat16)
        x = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        kw = dict(epilogue=epi, bias=b)
        if epi == K.VS_EPI_GATE_RES:
            kw.update(residual=x, gate=gate, gate_bstride=N, rows_per_batch=(M + 1) // 2)
        elif epi == K.VS_EPI_RES:
            kw.update(residual=x, alpha=1.0)
        out = x if epi in (K.VS_EPI_GATE_RES, K.VS_EPI_RES) else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t = {}
        for be in ("vstyler", "lt", "vstyler2", "lt2"):
            os.environ["VS_GEMM_BACKEND"] = be.rstrip("2")
            t[be] = timed(lambda: K.gemm(a, w, out, **kw))
        os.environ.pop("VS_GEMM_BACKEND")
        tv, tl = min(t["vstyler"], t["vstyler2"]), min(t["lt"], t["lt2"])
        fl = 2.0 * M * N * Kd
        print(f"M={M} {name:8s} N={N} K={Kd}: vstyler {tv:.3f} ms ({fl/tv/1e9:.0f} TF/s)  lt {tl:.3f} ms "
              f"({fl/tl/1e9:.0f} TF/s)  lt/vstyler speedup {tv/tl:.3f}", flush=True)
        del a, w, b, gate, x, out
