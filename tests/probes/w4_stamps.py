"""Phase timing of attn_fwd_w4's pipelined loop from a -DVS_W4_STAMPS build (diagnostic only):
  VSTYLER_LIB=build/diag/w4st/libvstyler.so python tests/probes/w4_stamps.py
Runs the 14B self-attention once and prints, per wave of block 0, the median cycles (s_memtime
ticks) of phases A, B, C, the barrier wait, D and the whole iteration over iterations 8..39."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import numpy as np
import torch
from vstyler import kernels as K
from vstyler import _lib
B, S, H = 2, 29640, 40
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
o = torch.empty_like(q)
from vstyler import kernels as _K
_K.set_option("attn_impl", 4)
for _ in range(3):
    K.attention(q, k, v, o, H, B)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (4 * 32 * 7))()
assert lib.vs_debug_w4_stamps(buf) == 0
st = np.array(buf, dtype=np.int64).reshape(4, 32, 7)
names = ["A", "B", "C", "bar", "D0-3", "D4-7", "iter"]
for w in range(4):
    nxt = np.append(st[w, 1:, 0], 0)
    d = np.stack([st[w, :, 1] - st[w, :, 0], st[w, :, 2] - st[w, :, 1], st[w, :, 3] - st[w, :, 2],
                  st[w, :, 4] - st[w, :, 3], st[w, :, 6] - st[w, :, 4], st[w, :, 5] - st[w, :, 6], nxt - st[w, :, 0]], 1)
    med = np.median(d[:-1], 0)
    print(f"wave {w}: " + "  ".join(f"{n} {m:.0f}" for n, m in zip(names, med)), flush=True)
print("(s_memtime ticks; MFMA work per phase: 16 x 32 cycles = 512 shader cycles)")
