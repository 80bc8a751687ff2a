"""A/B in one process: persistent attention grid vs one item per block (VS_ATTN_NO_PERSIST=1), at
the 14B 832x480x73 self- and cross-attention shapes, interleaved rounds (random data).
  python tests/probes/attn_persist_ab.py"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
B, S, H, L = 2, 29640, 40, 512
D = H * 128
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
k = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
v = torch.randn(B * S, D, device="cuda", generator=g).to(torch.bfloat16)
kc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
vc = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
o = torch.empty_like(q)
o2 = torch.empty_like(q)
for name, kk, vv, skv, reps in (("cross", kc, vc, L, 20), ("self", k, v, S, 2)):
    fl = 4.0 * S * skv * D * B
    res = {"persist": [], "one-item": []}
    for mode in ("persist", "one-item"):        # warm
        if mode == "persist":
            os.environ.pop("VS_ATTN_NO_PERSIST", None)
        else:
            os.environ["VS_ATTN_NO_PERSIST"] = "1"
        K.attention(q, kk, vv, o if mode == "persist" else o2, H, B)
    torch.cuda.synchronize()
    same = torch.equal(o, o2)
    for rnd in range(5):
        for mode in ("persist", "one-item"):
            if mode == "persist":
                os.environ.pop("VS_ATTN_NO_PERSIST", None)
            else:
                os.environ["VS_ATTN_NO_PERSIST"] = "1"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                K.attention(q, kk, vv, o, H, B)
            e1.record()
            torch.cuda.synchronize()
            res[mode].append(e0.elapsed_time(e1) / reps)
    for mode, ts in res.items():
        ts = sorted(ts)
        print(f"{name} {mode}: median {ts[2]:.3f} ms min {ts[0]:.3f} ms = {fl / ts[2] / 1e9:.1f} TF/s", flush=True)
    print(f"{name}: persistent == one-item-per-block bitwise: {same}", flush=True)
