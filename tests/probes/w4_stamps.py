"""Phase timing of attn_fwd_w4's pipelined loop from a -DVS_W4_STAMPS build (diagnostic only):
  VSTYLER_LIB=build/diag/w4st/libvstyler.so python tests/probes/w4_stamps.py
Runs the 14B self-attention once and prints, per wave of block 0, the median cycles (s_memtime
ticks) of phases A, B, C, the barrier wait, D and the whole iteration over iterations 8..39, then the
item switches of block 0 (first tile, tile loop, last tile + next Q issue, drain, O store, gap to the
next item).  W4S_SKV=512: keys / values of 512 rows (the cross-attention's 8-tile items)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import numpy as np
import torch
from vstyler import kernels as K
from vstyler import _lib
B, S, H = 2, 29640, 40
g = torch.Generator(device="cuda").manual_seed(0)
L = int(os.environ.get("W4S_SKV", S))
q = torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16)
k, v = (torch.randn(B * L, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(2))
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
if L < S:
    # the phases of each item's last tile (T % nkv == nkv - 1) against the median iteration
    nkv0 = (L + 63) // 64
    for w in range(4):
        nxt = np.append(st[w, 1:, 0], 0)
        d = np.stack([st[w, :, 1] - st[w, :, 0], st[w, :, 2] - st[w, :, 1], st[w, :, 3] - st[w, :, 2],
                      st[w, :, 4] - st[w, :, 3], st[w, :, 6] - st[w, :, 4], st[w, :, 5] - st[w, :, 6]], 1)
        last = [i for i in range(31) if (i + 8) % nkv0 == nkv0 - 1]
        if last:
            med = np.median(d[last], 0)
            print(f"wave {w} last tiles: " + "  ".join(f"{n} {m:.0f}" for n, m in zip(names[:6], med)), flush=True)
sw = (ctypes.c_ulonglong * (4 * 16 * 9))()
assert lib.vs_debug_w4_switch(sw) == 0
sw = np.array(sw, dtype=np.int64).reshape(4, 16, 9)
nkv = (L + 63) // 64
for w in range(4):
    a = sw[w]
    ok = a[:, 0] > 0
    a = a[ok]
    nxt0 = np.append(a[1:, 0], 0)
    d = np.stack([a[:, 1] - a[:, 0], (a[:, 2] - a[:, 1]) / max(1, 2 * ((nkv - 1) // 2)), a[:, 3] - a[:, 2],
                  a[:, 4] - a[:, 3], a[:, 5] - a[:, 4], nxt0 - a[:, 5], nxt0 - a[:, 0]], 1)[:-1]
    med = np.median(d, 0)
    q = np.median(np.stack([a[:, 7] - a[:, 6], a[:, 8] - a[:, 7]], 1)[:-1], 0)
    print(f"wave {w} items {len(a)}: first tile {med[0]:.0f}  per loop tile {med[1]:.0f}  last tile + next Q "
          f"{med[2]:.0f} (DMA drain {q[0]:.0f}, Q load {q[1]:.0f})  drain {med[3]:.0f}  O store {med[4]:.0f}  "
          f"gap to next {med[5]:.0f}  item {med[6]:.0f}", flush=True)
