"""Cross-attention at the 14B 832x480x73 CFG shape (2 x 29640 queries, 2 x 512 context keys, 40
heads): HIP-event time per launch with and without the split tail (VS_ATTN_NO_SPLIT read per call).

usage: python tests/probes/cross_attn_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch  # noqa: E402

from vstyler import kernels as K  # noqa: E402

B, S, L, H = 2, 29640, 512, 40
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16)
kc, vc = (torch.randn(B * L, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(2))
o = torch.empty_like(q)
flops = 4.0 * B * S * L * H * 128
for rep in range(2):
    for mode in ("split", "nosplit"):
        if mode == "nosplit":
            os.environ["VS_ATTN_NO_SPLIT"] = "1"
        else:
            os.environ.pop("VS_ATTN_NO_SPLIT", None)
        K.attention(q, kc, vc, o, H, B)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            K.attention(q, kc, vc, o, H, B)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"cross-attn {mode:8s}: {ms * 1e3:.0f} us/launch = {flops / ms / 1e9:.0f} TF/s", flush=True)
