import os, sys
sys.path.insert(0, "video-styler_amd"); sys.path.insert(0, ".")
import torch
from oracle import wan_oracle as O
from vstyler import kernels as K
BF16 = torch.bfloat16
os.environ["VS_FP8_BACKEND"] = "vstyler"
for (M, N, Kd) in [(520, 300, 5120), (520, 304, 5120), (520, 300, 640), (300, 300, 256)]:
    for kern in ("8p", "4w"):
        os.environ["VS_GEMM_KERNEL"] = kern
        g = torch.Generator().manual_seed(M + N + Kd)
        x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
        x[::5] *= 512
        w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
        w[:, 0] += (torch.arange(N) % 5).to(BF16)
        b = torch.randint(-8, 9, (N,), generator=g).to(BF16)
        ref = O.fp8_linear(x, w, b)
        x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
        sc = torch.empty(M, dtype=torch.float32, device="cuda")
        K.quant_fp8_rows(x.cuda(), x8, sc)
        out = torch.empty(M, N, dtype=BF16, device="cuda")
        K.gemm_fp8(x8, sc, w.to(torch.float8_e4m3fn).view(torch.uint8).cuda(), out, bias=b.cuda())
        o = out.cpu()
        bad = (o != ref)
        print(M, N, Kd, kern, "mismatch", int(bad.sum()), "rows", bad.any(1).nonzero().flatten()[:8].tolist(), "cols", bad.any(0).nonzero().flatten()[:8].tolist(), flush=True)
