"""GPU parity of the causal 3-D VAE (vstyler/vae.py + csrc/vae.hip) against the CPU oracle
(oracle/wan_vae_oracle.py, the reference's chunked feature-cache algorithm).

Kernel level: every conv configuration the VAE uses vs a bf16-rounded fp32 torch conv (results may
differ by bf16 rounding of a differently ordered fp32 sum: max-abs <= 1.5 ulp of the output scale,
>= 90 % of elements bit-equal); channel RMS norm+SiLU and the tile gather/blend/u8 kernels
bit-exact.  Model level: encode/decode (tiled) vs the oracle within 1.5x the oracle's own
fp32-vs-fp64 accumulation noise floor (plus 1e-3 rel-L2 slack), computed in the test.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from gpu_util import err
from oracle import wan_oracle as O
from oracle import wan_vae_oracle as V
from vae_util import TINY_VAE, _resample, synthetic_video

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _vae():
    from vstyler import vae
    return vae


def _to_nthwc(x, cpad=None):
    """(B, C, T, H, W) -> (B, T, H, W, Cpad) contiguous on the GPU."""
    y = x.permute(0, 2, 3, 4, 1)
    if cpad is not None and cpad > y.shape[-1]:
        y = F.pad(y, (0, cpad - y.shape[-1]))
    return y.contiguous().cuda()


def _from_nthwc(y, c=None):
    y = y.cpu()
    if c is not None:
        y = y[..., :c]
    return y.permute(0, 4, 1, 2, 3)


def _rand(shape, g, scale=1.0):
    return (scale * torch.randn(shape, generator=g)).to(BF16)


def _close_conv(got, ref):
    got, ref = got.float(), ref.float()
    scale = ref.abs().max().item()
    d = (got - ref).abs()
    assert d.max().item() <= 1.5 * scale * 2.0 ** -8 + 1e-6, (d.max().item(), scale)
    assert (got == ref).float().mean().item() >= 0.9


@pytest.mark.parametrize("cin,cout,res", [(64, 96, True), (96, 192, False), (32, 16, False), (384, 384, True),
                                          (32, 3, False)])
def test_causal_conv3d_k3(cin, cout, res):
    vae = _vae()
    g = torch.Generator().manual_seed(cin + cout)
    x = _rand((2, cin, 5, 12, 20), g)
    w = _rand((cout, cin, 3, 3, 3), g, 1 / math.sqrt(27 * cin))
    b = _rand((cout,), g, 0.1)
    ref = V.causal_conv3d(x, w, b, (1, 1, 1))
    cw = vae.ConvW(w, b, "cuda")
    ldy = (cout + 3) // 4 * 4
    y = torch.zeros((2, 5, 12, 20, ldy), dtype=BF16, device="cuda")
    r = None
    if res:
        r_cpu = _rand((2, cout, 5, 12, 20), g)
        ref = ref + r_cpu
        r = _to_nthwc(r_cpu)
    vae.conv(_to_nthwc(x), cw, (5, 12, 20), pad=(2, 1, 1), y=y, res=r)
    _close_conv(_from_nthwc(y, cout), ref)


@pytest.mark.parametrize("cin,cout,up2", [(96, 96, False), (64, 128, True), (384, 384, False), (32, 16, False),
                                          (192, 64, False)])
def test_conv_pixel_blocks_bit_identical(cin, cout, up2, opt):
    """256-pixel tiles (two 32-pixel blocks per wave, option vae_pxb=2) and the two-stage load pipeline
    (vae_pre=2) == 128-pixel tiles with one stage: the same K order per output, ragged last tile
    (M = 2 * 5 * h * w not a multiple of 256) included."""
    vae = _vae()
    g = torch.Generator().manual_seed(cin * 7 + cout)
    h, w = (6, 10) if up2 else (12, 20)
    x = _to_nthwc(_rand((2, cin, 5, h, w), g))
    cw = vae.ConvW(_rand((cout, cin, 3, 3, 3), g, 1 / math.sqrt(27 * cin)), _rand((cout,), g, 0.1), "cuda")
    outs = []
    for pxb, pre in ((1, 1), (2, 1), (1, 2), (2, 2), (1, 3), (2, 3)):
        opt(vae_pxb=pxb, vae_pre=pre, vae_halo=0)
        outs.append(vae.conv(x, cw, (5, 2 * h if up2 else h, 2 * w if up2 else w), pad=(2, 1, 1), up2=up2).cpu())
    for o in outs[1:]:
        assert torch.equal(outs[0], o)


@pytest.mark.parametrize("cin,cout,kt,t_lo,h,w,up2", [(96, 96, 3, 0, 17, 45, False), (32, 192, 3, 2, 9, 33, False),
                                                      (192, 96, 1, 0, 16, 64, False), (384, 384, 3, 0, 8, 32, False),
                                                      (384, 192, 1, 0, 7, 19, True), (192, 96, 1, 0, 9, 16, True),
                                                      (96, 32, 3, 0, 17, 45, False), (192, 16, 3, 1, 9, 33, False),
                                                      (64, 32, 1, 0, 7, 19, True)])
def test_conv_halo_kernel(cin, cout, kt, t_lo, h, w, up2, opt):
    """The patch-resident 3x3(x3) kernel (option vae_halo, the default for these shapes) vs a
    bf16-rounded fp32 torch conv and vs the per-tap gather kernel: ragged 16 x 32 tiles, the causal
    time pad, frames below t_lo read as zero, a 2-D (kt = 1) conv, the nearest-x2 upsample of the
    Resample convs (up2), 96-channel blocks and the <= 32-channel heads (NB = 1), two batch slices."""
    vae = _vae()
    g = torch.Generator().manual_seed(cin + 3 * cout + kt + up2)
    T = 5
    x = _rand((2, cin, T, h, w), g)
    wt = _rand((cout, cin, kt, 3, 3), g, 1 / math.sqrt(9 * kt * cin))
    b = _rand((cout,), g, 0.1)
    xz = x.clone()
    xz[:, :, :t_lo] = 0
    if up2:
        xz = xz.repeat_interleave(2, dim=3).repeat_interleave(2, dim=4)
    pt = kt - 1
    ref = F.conv3d(F.pad(xz.float(), (1, 1, 1, 1, pt, 0)), wt.float(), b.float()).to(BF16)
    cw = vae.ConvW(wt, b, "cuda")
    xg = _to_nthwc(x)
    ho, wo = (2 * h, 2 * w) if up2 else (h, w)
    outs = []
    for halo in (1, 0):
        opt(vae_halo=halo)
        outs.append(_from_nthwc(vae.conv(xg, cw, (T, ho, wo), pad=(pt, 1, 1), t_lo=t_lo, up2=up2), cout))
    _close_conv(outs[0], ref)
    _close_conv(outs[0], outs[1])


def test_conv_halo_long_sequence(opt):
    """A 121-frame 240 x 416 x 96 slice (2.3 GB: more than 31-bit offsets reach, the C4 tile shape):
    the halo kernel rebases its input resource per frame; vs the per-tap kernel on the GPU."""
    vae = _vae()
    g = torch.Generator(device="cuda").manual_seed(11)
    T, h, w, c = 121, 240, 416, 96
    x = torch.randn((1, T, h, w, c), generator=g, device="cuda").to(BF16)
    wt = (torch.randn((c, c, 3, 3, 3), generator=g, device="cuda") / math.sqrt(27 * c)).to(BF16)
    cw = vae.ConvW(wt, (0.1 * torch.randn((c,), generator=g, device="cuda")).to(BF16), "cuda")
    outs = []
    for halo in (1, 0):
        opt(vae_halo=halo)
        outs.append(vae.conv(x, cw, (T, h, w), pad=(2, 1, 1)))
    del x
    a, b = outs[0].float(), outs[1].float()
    scale = b.abs().max().item()
    assert (a - b).abs().max().item() <= 1.5 * scale * 2.0 ** -8
    assert (outs[0] == outs[1]).float().mean().item() >= 0.9


def test_rgb_input_conv_channel_padding():
    vae = _vae()
    g = torch.Generator().manual_seed(3)
    x = _rand((1, 3, 3, 16, 16), g)
    w = _rand((96, 3, 3, 3, 3), g, 0.2)
    b = _rand((96,), g, 0.1)
    cw = vae.ConvW(w, b, "cuda")
    assert cw.cin == 32
    y = vae.conv(_to_nthwc(x, 32), cw, (3, 16, 16), pad=(2, 1, 1))
    _close_conv(_from_nthwc(y), V.causal_conv3d(x, w, b, (1, 1, 1)))


@pytest.mark.parametrize("mode,c", [("downsample2d", 64), ("downsample3d", 64), ("upsample2d", 128),
                                    ("upsample3d", 128)])
@pytest.mark.parametrize("t", [1, 5])
def test_resample_modes(mode, c, t):
    """Resample (wan_video_vae.py:82-174) incl. stride-2 ZeroPad2d conv, fused nearest-x2 upsample,
    the downsample3d time conv (stride 2, frame 0 passed through) and the upsample3d time conv
    (frames 1.. only, channel halves interleaved into frames)."""
    vae = _vae()
    g = torch.Generator().manual_seed({"downsample2d": 1, "downsample3d": 2, "upsample2d": 3, "upsample3d": 4}[mode] * 10 + t)
    W = {}
    co = c // 2 if mode.startswith("up") else c
    W["r.resample.1.weight"] = _rand((co, c, 3, 3), g, 1 / math.sqrt(9 * c))
    W["r.resample.1.bias"] = _rand((co,), g, 0.1)
    if mode == "upsample3d":
        W["r.time_conv.weight"] = _rand((2 * c, c, 3, 1, 1), g, 1 / math.sqrt(3 * c))
        W["r.time_conv.bias"] = _rand((2 * c,), g, 0.1)
    if mode == "downsample3d":
        W["r.time_conv.weight"] = _rand((c, c, 3, 1, 1), g, 1 / math.sqrt(3 * c))
        W["r.time_conv.bias"] = _rand((c,), g, 0.1)
    x = _rand((2, c, t, 8, 12), g)
    ref = _resample(x, W, "r.", mode)
    m = vae.WanVideoVAE(device="cuda")
    m.cw = {k[:-len("weight")]: vae.ConvW(W[k], W[k[:-len("weight")] + "bias"], "cuda")
            for k in W if k.endswith("weight")}
    got = _from_nthwc(m._resample(_to_nthwc(x), "r.", mode))
    assert got.shape == ref.shape
    _close_conv(got, ref)


def test_rmsnorm_silu_bit_exact():
    vae = _vae()
    g = torch.Generator().manual_seed(5)
    for c in (32, 96, 384):
        x = _rand((3, c, 2, 5, 7), g, 2.0)
        gamma = (1 + 0.1 * torch.randn((c, 1, 1, 1), generator=g)).to(BF16)
        for silu in (False, True):
            ref = V.rms_norm(x, gamma)
            if silu:
                ref = F.silu(ref)
            got = _from_nthwc(vae.rmsnorm(_to_nthwc(x), gamma.reshape(-1).cuda(), silu))
            d = (got.float() - ref.float()).abs()
            ulp = ref.float().abs().clamp_min(1e-30) * 2.0 ** -7
            assert (d <= ulp).all(), (c, silu, d.max().item())
            assert (got == ref).float().mean().item() > 0.995


def test_attention_block():
    vae = _vae()
    g = torch.Generator().manual_seed(9)
    c = 128
    W = {"a.norm.gamma": (1 + 0.1 * torch.randn((c, 1, 1), generator=g)).to(BF16),
         "a.to_qkv.weight": _rand((3 * c, c, 1, 1), g, 1 / math.sqrt(c)),
         "a.to_qkv.bias": _rand((3 * c,), g, 0.1),
         "a.proj.weight": _rand((c, c, 1, 1), g, 1 / math.sqrt(c)),
         "a.proj.bias": _rand((c,), g, 0.1)}
    x = _rand((2, c, 3, 6, 10), g)
    ref = V.attention_block(x, W, "a.")
    m = vae.WanVideoVAE(device="cuda")
    m.params = {"a.norm.gamma": W["a.norm.gamma"].reshape(-1).cuda()}
    m.cw = {"a.to_qkv.": vae.ConvW(W["a.to_qkv.weight"], W["a.to_qkv.bias"], "cuda"),
            "a.proj.": vae.ConvW(W["a.proj.weight"], W["a.proj.bias"], "cuda")}
    got = _from_nthwc(m._attn_block(_to_nthwc(x), "a."))
    mx, rel = err(got, ref)
    assert rel < 4e-3 and mx < 3e-2, (mx, rel)


def _model(cfg, W):
    vae = _vae()
    m = vae.WanVideoVAE(z_dim=cfg["z_dim"], dim=cfg["dim"], dim_mult=cfg["dim_mult"],
                        num_res_blocks=cfg["num_res_blocks"], temperal_downsample=cfg["temperal_downsample"],
                        device="cuda")
    return m.load_state_dict(W)


def _floor(fn):
    old = O.ACC_DTYPE
    try:
        O.ACC_DTYPE = torch.float64
        r64 = fn()
    finally:
        O.ACC_DTYPE = old
    r32 = fn()
    return r32, err(r64, r32)


def _within_floor(got, ref, floor):
    mx, rel = err(got, ref)
    fmx, frel = floor
    assert rel <= 1.5 * frel + 1e-3 and mx <= 1.5 * fmx + 1e-2, dict(gpu=(mx, rel), floor=floor)


@pytest.mark.parametrize("tiled", [False, True])
def test_encode_tiny(tiled):
    W = V.random_vae_weights(TINY_VAE, seed=21)
    video = synthetic_video(9, 64, 96)
    ts, st = (4, 6), (2, 3)
    if tiled:
        ref, floor = _floor(lambda: V.tiled_encode(video, W, ts, st, TINY_VAE))
    else:
        ref, floor = _floor(lambda: V.vae_encode(video, W, TINY_VAE))
    got = _model(TINY_VAE, W).encode(video.cuda(), "cuda", tiled=tiled, tile_size=ts, tile_stride=st)
    assert got.shape == ref.shape == (1, 16, 3, 8, 12)
    _within_floor(got, ref, floor)


@pytest.mark.parametrize("tiled", [False, True])
def test_decode_tiny(tiled):
    W = V.random_vae_weights(TINY_VAE, seed=22)
    g = torch.Generator().manual_seed(4)
    z = torch.randn((1, 16, 3, 8, 12), generator=g).to(BF16)
    ts, st = (4, 6), (2, 3)
    if tiled:
        ref, floor = _floor(lambda: V.tiled_decode(z, W, ts, st, TINY_VAE))
    else:
        ref, floor = _floor(lambda: V.single_decode(z, W, TINY_VAE))
    got = _model(TINY_VAE, W).decode(z.cuda(), "cuda", tiled=tiled, tile_size=ts, tile_stride=st)
    assert got.shape == ref.shape == (1, 3, 9, 64, 96)
    _within_floor(got, ref, floor)


def test_encode_decode_wan21_dims():
    """The real Wan2.1 VAE widths (dim 96, 384-wide middle with attention) on a small video."""
    W = V.random_vae_weights(seed=23)
    video = synthetic_video(5, 32, 48)
    ref, floor = _floor(lambda: V.vae_encode(video, W))
    m = _model(V.VAE_CONFIG, W)
    got = m.encode(video.cuda(), "cuda", tiled=False)
    _within_floor(got, ref, floor)
    zref, zfloor = _floor(lambda: V.single_decode(ref, W))
    zgot = m.decode(ref.cuda(), "cuda", tiled=False)
    assert zgot.shape == (1, 3, 5, 32, 48)
    _within_floor(zgot, zref, zfloor)


def test_output_to_u8_bit_exact():
    vae = _vae()
    g = torch.Generator().manual_seed(6)
    v = (torch.rand((1, 3, 2, 5, 9), generator=g) * 2.2 - 1.1).clamp(-1, 1).to(BF16)
    ref = V.vae_output_to_u8(v)
    got = vae.vae_output_to_u8(v[0].cuda()).cpu()
    assert torch.equal(got, ref)
