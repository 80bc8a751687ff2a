import os, sys
sys.path.insert(0, "video-styler_amd")
import torch
from vstyler import kernels as K
os.environ["VS_GEMM_BACKEND"] = "lt"
for M, N, Kd in ((59280, 5120, 5120), (3705, 5120, 13824)):
    a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
    b = (0.1 * torch.randn(N, device="cuda")).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    K.gemm(a, w, out, bias=b)
    torch.cuda.synchronize()
print("done")
