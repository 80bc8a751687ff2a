"""Runs one kernel a few times for PMC collection: attn (14B self-attention), cross (14B
cross-attention, 512 context keys), vae (one tiled 832x480x73 VAE encode: every vae_conv_kernel
shape of it), vaeconv (its dominant 3x3x3 96 -> 96 conv on the default kernel) or gemm (FFN up)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "video-styler_amd"))
import torch
from vstyler import kernels as K
which = sys.argv[1]
g = torch.Generator(device="cuda").manual_seed(0)
if which == "attn":
    B, S, H = 2, 29640, 40
    q, k, v = (torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(3))
    o = torch.empty_like(q)
    fn = lambda: K.attention(q, k, v, o, H, B)
elif which == "cross":
    B, S, H, L = 2, 29640, 40, 512
    q = torch.randn(B * S, H * 128, device="cuda", generator=g).to(torch.bfloat16)
    k, v = (torch.randn(B * L, H * 128, device="cuda", generator=g).to(torch.bfloat16) for _ in range(2))
    o = torch.empty_like(q)
    fn = lambda: K.attention(q, k, v, o, H, B)
elif which == "vae":
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
    from oracle import wan_vae_oracle as V      # (random weights of the reference layout only)
    from vstyler import vae
    m = vae.WanVideoVAE(device="cuda").load_state_dict(V.random_vae_weights(seed=6))
    video = (torch.rand((1, 3, 73, 480, 832), generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    fn = lambda: m.encode(video, "cuda", tiled=True, tile_size=(30, 52), tile_stride=(15, 26))
elif which == "vaeconv":
    # the dominant VAE conv shape (3x3x3, 96 -> 96 channels, a 240x416 tile, 21 frames) on the default path
    from vstyler import vae
    T, Hh, Ww, C = 21, 240, 416, 96
    x = torch.randn((1, T, Hh, Ww, C), device="cuda", generator=g).to(torch.bfloat16)
    cw = vae.ConvW((0.03 * torch.randn((C, C, 3, 3, 3), device="cuda", generator=g)).to(torch.bfloat16),
                   torch.zeros(C, device="cuda", dtype=torch.bfloat16), "cuda")
    yv = torch.empty_like(x)
    fn = lambda: vae.conv(x, cw, (T, Hh, Ww), pad=(2, 1, 1), y=yv)
else:
    M, N, Kd = int(os.environ.get("KP_M", "59280")), int(os.environ.get("KP_N", "13824")), 5120    # KP_M / KP_N: rows / columns (default the SP = 1 FFN-up)
    a = torch.randn(M, Kd, device="cuda", generator=g).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = lambda: K.gemm(a, w, out)
for _ in range(1 if which == "vae" else 3):
    fn()
torch.cuda.synchronize()
