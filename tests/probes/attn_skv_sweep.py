"""Attention time vs key count at the 14B query shape (2 x 29 640 rows x 40 heads): T(Skv) = items x
(per-item overhead + tiles x per-tile cost), so the slope and intercept separate the item switch
(Q load, O store, pipeline fill) from the key-tile loop -- the cross-attention has 8 tiles per item.
Both kernels (option attn_impl 8 / 4), interleaved rounds.  usage: python tests/probes/attn_skv_sweep.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, H = 2, 29640, 40
D = H * 128
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty_like(q)
skvs = [int(x) for x in os.environ.get("SKV", "512,1024,2048,4096").split(",")]
kv = {L: [torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16) for _ in range(2)] for L in skvs}
res = {}
for rnd in range(2):
    for impl in (8, 4):
        K.set_option("attn_impl", impl)
        for L in skvs:
            k, v = kv[L]
            fn = lambda: K.attention(q, k, v, o, H, B)
            fn(); torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
            t = sorted(ts)[2]
            res.setdefault((impl, L), []).append(t)
K.set_option("attn_impl", 0)
items = (S + 255) // 256 * H * B
for impl in (8, 4):
    pts = [(L // 64, min(res[(impl, L)])) for L in skvs]
    n = len(pts)
    mx = sum(p[0] for p in pts) / n
    my = sum(p[1] for p in pts) / n
    slope = sum((p[0] - mx) * (p[1] - my) for p in pts) / sum((p[0] - mx) ** 2 for p in pts)
    icpt = my - slope * mx
    per_cu = items / 256
    for L in skvs:
        t = min(res[(impl, L)])
        print(f"impl {impl} Skv {L:5d}: {t:.3f} ms  {4.0 * S * L * D * B / t / 1e9:.0f} TF/s", flush=True)
    print(f"impl {impl}: per key tile {slope * 1e3 / per_cu:.2f} us per CU-item, per item switch "
          f"{icpt * 1e3 / per_cu:.2f} us  (fit over {skvs})", flush=True)
