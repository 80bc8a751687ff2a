"""Probe (needs a library built with -DVS_GEMM_STAMPS, path in VSTYLER_LIB): per-phase cycle
stamps of the 256^2 ping-pong GEMM for wave 0 (group 0) and wave 4 (group 1) of workgroup 0."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch  # noqa: E402

from vstyler import _lib, kernels as K  # noqa: E402

M, N, Kd = int(os.environ.get("GM", 59280)), int(os.environ.get("GN", 5120)), int(os.environ.get("GK", 5120))
a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
w = (0.05 * torch.randn(N, Kd, device="cuda")).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    K.gemm(a, w, out)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (2 * 5 * 32))()
assert lib.vs_debug_gemm_stamps(buf) == 0
st = [[buf[g * 160 + i] for i in range(160)] for g in range(2)]
t0 = min(st[0][0], st[1][0])
names = ["frags+issue", "bar1", "mfma", "bar2"]
for g in range(2):
    print(f"group {g}: per half-step cycles [" + ", ".join(names) + "]  total")
    for h in range(1, 32):
        s = st[g][5 * h:5 * h + 5]
        d = [s[i + 1] - s[i] for i in range(4)]
        nxt = st[g][5 * (h + 1)] - s[4] if h < 31 else 0
        print(f"  h={h:2d} start {s[0]-t0:7d} " + " ".join(f"{x:5d}" for x in d) + f"  | {s[4]-s[0]:5d} (+{nxt})")
