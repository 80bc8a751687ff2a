"""Probe (library built with -DVS_ATTN_STAMPS, path in VSTYLER_LIB): per-phase cycles of the attention
loop for wave 0 (group 0) and wave 4 (group 1) of workgroup 0 at the 14B self-attention shape."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import _lib, kernels as K
B, S, H = 2, 29640, 40
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
o = torch.empty_like(q)
for _ in range(3):
    K.attention(q, k, v, o, H, B)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (2 * 4 * 32))()
assert _lib.load().vs_debug_attn_stamps(buf) == 0
nkv = (S + 63) // 64
names = ["B work", "B->A bar", "A ks0", "A ks1", "A ks2", "A ks3", "A tail", "A->B bar"]
for grp in range(2):
    ring = [buf[grp * 128 + i] for i in range(128)]
    order = [(nkv + k) % 16 for k in range(16)]          # ring slots of tiles nkv-16 .. nkv-1
    st = [ring[8 * s:8 * s + 8] for s in order]
    rows = []
    for t in range(13):
        s = st[t]
        rows.append([s[i + 1] - s[i] for i in range(7)] + [st[t + 1][0] - s[7]])
    avg = [sum(r[i] for r in rows) / len(rows) for i in range(8)]
    print(f"group {grp}: " + "  ".join(f"{n} {a:.0f}" for n, a in zip(names, avg)) + f"  | tile {sum(avg):.0f}")
