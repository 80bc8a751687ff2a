"""TEST INFRASTRUCTURE ONLY -- from-scratch PyTorch-CPU restatement of the Wan2.1 causal 3-D VAE
(reference `diffsynth/models/wan_video_vae.py`, the Wan2.1 part) and of the VACE conditioning unit
that calls it (`diffsynth/pipelines/wan_video_new.py:861-920`).

Faithful to the reference's *chunked* execution: the encoder runs on chunks of [1, 4, 4, ...]
frames and the decoder on one latent frame at a time, each causal conv carrying the 2-frame
feature cache of `:44-52,283-301` (incl. the 'Rep' sentinel of upsample3d `:122-156` and the
skip-first-chunk rule of downsample3d `:162-173`).  The product (`vstyler/vae.py`) runs the
mathematically equivalent whole-sequence form, so the tests check that equivalence too.

Convolutions accumulate in `wan_oracle.ACC_DTYPE` (fp32; fp64 only to measure the noise floor) on
bf16-valued inputs with one bf16 rounding of (acc + bias), as a bf16 conv does; elementwise ops
(F.normalize, scale, gamma, SiLU, residual add, latent (de)normalisation, tile blending) run as
torch bf16 ops, exactly the tensors the reference materialises.  Parity status: numerics
"parity unpinned" (no reference vectors exist); structure pinned by the registry md5 key hash
`ccc42284ea13e1ad04693284c7a09be6` (configs/model_config.py:164) and the latent mean/std.
"""
import math

import torch
import torch.nn.functional as F

from . import wan_oracle as _wo

BF16 = torch.bfloat16
CACHE_T = 2  # wan_video_vae.py:8

# wan_video_vae.py:1063-1070
VAE_MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
            0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
VAE_STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
           3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]

# VideoVAE_ defaults (wan_video_vae.py:953-960) and WanVideoVAE (:1060-1078)
VAE_CONFIG = dict(dim=96, z_dim=16, dim_mult=(1, 2, 4, 4), num_res_blocks=2,
                  temperal_downsample=(False, True, True))


# ------------------------------------------------------------------------------------------
# parameter layout (module tree of Encoder3d :517-567, Decoder3d :736-787, VideoVAE_ :951-976)
# ------------------------------------------------------------------------------------------
def _res_shapes(p, i, o, d):
    d[p + "residual.0.gamma"] = (i, 1, 1, 1)
    d[p + "residual.2.weight"] = (o, i, 3, 3, 3)
    d[p + "residual.2.bias"] = (o,)
    d[p + "residual.3.gamma"] = (o, 1, 1, 1)
    d[p + "residual.6.weight"] = (o, o, 3, 3, 3)
    d[p + "residual.6.bias"] = (o,)
    if i != o:
        d[p + "shortcut.weight"] = (o, i, 1, 1, 1)
        d[p + "shortcut.bias"] = (o,)


def _attn_shapes(p, c, d):
    d[p + "norm.gamma"] = (c, 1, 1)
    d[p + "to_qkv.weight"] = (3 * c, c, 1, 1)
    d[p + "to_qkv.bias"] = (3 * c,)
    d[p + "proj.weight"] = (c, c, 1, 1)
    d[p + "proj.bias"] = (c,)


def _resample_shapes(p, c, mode, d):
    co = c // 2 if mode.startswith("up") else c
    d[p + "resample.1.weight"] = (co, c, 3, 3)
    d[p + "resample.1.bias"] = (co,)
    if mode == "upsample3d":
        d[p + "time_conv.weight"] = (2 * c, c, 3, 1, 1)
        d[p + "time_conv.bias"] = (2 * c,)
    elif mode == "downsample3d":
        d[p + "time_conv.weight"] = (c, c, 3, 1, 1)
        d[p + "time_conv.bias"] = (c,)


def encoder_layers(cfg):
    """Ordered (kind, prefix, args) of Encoder3d.downsamples (:543-558)."""
    dim, mult, nrb = cfg["dim"], cfg["dim_mult"], cfg["num_res_blocks"]
    dims = [dim * u for u in (1,) + tuple(mult)]
    out, k = [], 0
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(nrb):
            out.append(("res", f"encoder.downsamples.{k}.", (a, b)))
            k += 1
            a = b
        if i != len(mult) - 1:
            mode = "downsample3d" if cfg["temperal_downsample"][i] else "downsample2d"
            out.append(("resample", f"encoder.downsamples.{k}.", (b, mode)))
            k += 1
    return out, dims


def decoder_layers(cfg):
    """Ordered (kind, prefix, args) of Decoder3d.upsamples (:767-783)."""
    dim, mult, nrb = cfg["dim"], cfg["dim_mult"], cfg["num_res_blocks"]
    dims = [dim * u for u in (mult[-1],) + tuple(mult[::-1])]
    tu = tuple(cfg["temperal_downsample"][::-1])
    out, k = [], 0
    for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
        if i in (1, 2, 3):
            a = a // 2
        for _ in range(nrb + 1):
            out.append(("res", f"decoder.upsamples.{k}.", (a, b)))
            k += 1
            a = b
        if i != len(mult) - 1:
            mode = "upsample3d" if tu[i] else "upsample2d"
            out.append(("resample", f"decoder.upsamples.{k}.", (b, mode)))
            k += 1
    return out, dims


def vae_param_shapes(cfg=VAE_CONFIG):
    """State-dict layout of the civitai Wan2.1 VAE file (keys without the 'model.' prefix that
    WanVideoVAEStateDictConverter.from_civitai adds, :1260-1266)."""
    z = cfg["z_dim"]
    d = {}
    layers, dims = encoder_layers(cfg)
    d["encoder.conv1.weight"] = (dims[0], 3, 3, 3, 3)
    d["encoder.conv1.bias"] = (dims[0],)
    for kind, p, args in layers:
        (_res_shapes if kind == "res" else _resample_shapes)(p, *args, d)
    top = dims[-1]
    _res_shapes("encoder.middle.0.", top, top, d)
    _attn_shapes("encoder.middle.1.", top, d)
    _res_shapes("encoder.middle.2.", top, top, d)
    d["encoder.head.0.gamma"] = (top, 1, 1, 1)
    d["encoder.head.2.weight"] = (2 * z, top, 3, 3, 3)
    d["encoder.head.2.bias"] = (2 * z,)
    d["conv1.weight"] = (2 * z, 2 * z, 1, 1, 1)
    d["conv1.bias"] = (2 * z,)
    d["conv2.weight"] = (z, z, 1, 1, 1)
    d["conv2.bias"] = (z,)
    layers, dd = decoder_layers(cfg)
    d["decoder.conv1.weight"] = (dd[0], z, 3, 3, 3)
    d["decoder.conv1.bias"] = (dd[0],)
    _res_shapes("decoder.middle.0.", dd[0], dd[0], d)
    _attn_shapes("decoder.middle.1.", dd[0], d)
    _res_shapes("decoder.middle.2.", dd[0], dd[0], d)
    for kind, p, args in layers:
        (_res_shapes if kind == "res" else _resample_shapes)(p, *args, d)
    d["decoder.head.0.gamma"] = (dd[-1], 1, 1, 1)
    d["decoder.head.2.weight"] = (3, dd[-1], 3, 3, 3)
    d["decoder.head.2.bias"] = (3,)
    return d


def random_vae_weights(cfg=VAE_CONFIG, seed=6):
    """Synthetic weights: conv weights N(0, 1/fan_in) (keeps activations O(1) through ~40 convs),
    biases 0.01*N, gammas 1 + 0.1*N; all bf16."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in vae_param_shapes(cfg).items():
        if name.endswith("gamma"):
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif name.endswith("bias"):
            t = 0.01 * torch.randn(shape, generator=g)
        else:
            fan_in = math.prod(shape[1:])
            t = torch.randn(shape, generator=g) / math.sqrt(fan_in)
        out[name] = t.to(BF16)
    return out


# ------------------------------------------------------------------------------------------
# operators
# ------------------------------------------------------------------------------------------
def _acc():
    return _wo.ACC_DTYPE


def causal_conv3d(x, w, b, padding, cache_x=None, stride=1):
    """CausalConv3d.forward (:38-52): time padded only at the front by 2*pad_t, reduced by the
    cached frames concatenated in front."""
    pt, ph, pw = padding
    pad = [pw, pw, ph, ph, 2 * pt, 0]
    if cache_x is not None and pad[4] > 0:
        x = torch.cat([cache_x, x], dim=2)
        pad[4] -= cache_x.shape[2]
    x = F.pad(x, pad)
    acc = _acc()
    y = F.conv3d(x.to(acc), w.to(acc), b.to(acc), stride=stride)
    return y.to(BF16)


def conv2d(x, w, b, stride=1, padding=0):
    acc = _acc()
    return F.conv2d(x.to(acc), w.to(acc), b.to(acc), stride=stride, padding=padding).to(BF16)


def rms_norm(x, gamma):
    """RMS_norm.forward (:67-70): bf16 F.normalize over channels, * sqrt(C), * gamma (+ 0.)."""
    return F.normalize(x, dim=1) * (x.shape[1] ** 0.5) * gamma


def upsample_nearest2x(x):
    """Upsample.forward (:75-79): nearest-exact x2 in fp32, back to bf16."""
    return F.interpolate(x.float(), scale_factor=(2.0, 2.0), mode="nearest-exact").type_as(x)


def _cached_conv(x, W, p, padding, feat_cache, feat_idx):
    """The cache protocol wrapped around every causal conv (:286-298, :570-582)."""
    idx = feat_idx[0]
    cache_x = x[:, :, -CACHE_T:].clone()
    if cache_x.shape[2] < 2 and feat_cache[idx] is not None:
        cache_x = torch.cat([feat_cache[idx][:, :, -1:], cache_x], dim=2)
    y = causal_conv3d(x, W[p + "weight"], W[p + "bias"], padding, feat_cache[idx])
    feat_cache[idx] = cache_x
    feat_idx[0] += 1
    return y


def residual_block(x, W, p, feat_cache, feat_idx):
    """ResidualBlock.forward (:283-301)."""
    if p + "shortcut.weight" in W:
        h = causal_conv3d(x, W[p + "shortcut.weight"], W[p + "shortcut.bias"], (0, 0, 0))
    else:
        h = x
    x = F.silu(rms_norm(x, W[p + "residual.0.gamma"]))
    x = _cached_conv(x, W, p + "residual.2.", (1, 1, 1), feat_cache, feat_idx)
    x = F.silu(rms_norm(x, W[p + "residual.3.gamma"]))
    x = _cached_conv(x, W, p + "residual.6.", (1, 1, 1), feat_cache, feat_idx)
    return x + h


def attention_block(x, W, p):
    """AttentionBlock.forward (:321-342): per frame single-head attention over H*W tokens."""
    identity = x
    b, c, t, h, w = x.shape
    x = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    x = rms_norm(x, W[p + "norm.gamma"])
    qkv = conv2d(x, W[p + "to_qkv.weight"], W[p + "to_qkv.bias"])
    qkv = qkv.reshape(b * t, 1, c * 3, h * w).permute(0, 1, 3, 2)
    q, k, v = qkv.chunk(3, dim=-1)
    acc = _acc()
    s = (q.to(acc) @ k.to(acc).transpose(-1, -2)) / math.sqrt(c)
    o = (torch.softmax(s, dim=-1) @ v.to(acc)).to(BF16)
    o = o.squeeze(1).permute(0, 2, 1).reshape(b * t, c, h, w)
    o = conv2d(o, W[p + "proj.weight"], W[p + "proj.bias"])
    o = o.reshape(b, t, c, h, w).permute(0, 2, 1, 3, 4)
    return o + identity


def resample(x, W, p, mode, feat_cache, feat_idx):
    """Resample.forward (:120-174) with its feature-cache protocol."""
    b, c, t, h, w = x.shape
    if mode == "upsample3d":
        idx = feat_idx[0]
        if feat_cache[idx] is None:
            feat_cache[idx] = "Rep"
            feat_idx[0] += 1
        else:
            cache_x = x[:, :, -CACHE_T:].clone()
            if cache_x.shape[2] < 2 and not isinstance(feat_cache[idx], str):
                cache_x = torch.cat([feat_cache[idx][:, :, -1:], cache_x], dim=2)
            if cache_x.shape[2] < 2 and isinstance(feat_cache[idx], str):
                cache_x = torch.cat([torch.zeros_like(cache_x), cache_x], dim=2)
            prev = None if isinstance(feat_cache[idx], str) else feat_cache[idx]
            x = causal_conv3d(x, W[p + "time_conv.weight"], W[p + "time_conv.bias"], (1, 0, 0), prev)
            feat_cache[idx] = cache_x
            feat_idx[0] += 1
            x = x.reshape(b, 2, c, t, h, w)
            x = torch.stack((x[:, 0], x[:, 1]), 3).reshape(b, c, t * 2, h, w)
    t = x.shape[2]
    x2 = x.permute(0, 2, 1, 3, 4).reshape(b * t, x.shape[1], x.shape[3], x.shape[4])
    if mode.startswith("upsample"):
        x2 = conv2d(upsample_nearest2x(x2), W[p + "resample.1.weight"], W[p + "resample.1.bias"], padding=1)
    else:
        x2 = conv2d(F.pad(x2, (0, 1, 0, 1)), W[p + "resample.1.weight"], W[p + "resample.1.bias"], stride=2)
    x = x2.reshape(b, t, x2.shape[1], x2.shape[2], x2.shape[3]).permute(0, 2, 1, 3, 4)
    if mode == "downsample3d":
        idx = feat_idx[0]
        if feat_cache[idx] is None:
            feat_cache[idx] = x.clone()
            feat_idx[0] += 1
        else:
            cache_x = x[:, :, -1:].clone()
            x = causal_conv3d(torch.cat([feat_cache[idx][:, :, -1:], x], 2), W[p + "time_conv.weight"],
                              W[p + "time_conv.bias"], (0, 0, 0), stride=(2, 1, 1))
            feat_cache[idx] = cache_x
            feat_idx[0] += 1
    return x


def encoder3d(x, W, cfg, feat_cache, feat_idx):
    """Encoder3d.forward (:569-617)."""
    x = _cached_conv(x, W, "encoder.conv1.", (1, 1, 1), feat_cache, feat_idx)
    layers, _ = encoder_layers(cfg)
    for kind, p, args in layers:
        if kind == "res":
            x = residual_block(x, W, p, feat_cache, feat_idx)
        else:
            x = resample(x, W, p, args[1], feat_cache, feat_idx)
    x = residual_block(x, W, "encoder.middle.0.", feat_cache, feat_idx)
    x = attention_block(x, W, "encoder.middle.1.")
    x = residual_block(x, W, "encoder.middle.2.", feat_cache, feat_idx)
    x = F.silu(rms_norm(x, W["encoder.head.0.gamma"]))
    return _cached_conv(x, W, "encoder.head.2.", (1, 1, 1), feat_cache, feat_idx)


def decoder3d(x, W, cfg, feat_cache, feat_idx):
    """Decoder3d.forward (:789-838)."""
    x = _cached_conv(x, W, "decoder.conv1.", (1, 1, 1), feat_cache, feat_idx)
    x = residual_block(x, W, "decoder.middle.0.", feat_cache, feat_idx)
    x = attention_block(x, W, "decoder.middle.1.")
    x = residual_block(x, W, "decoder.middle.2.", feat_cache, feat_idx)
    layers, _ = decoder_layers(cfg)
    for kind, p, args in layers:
        if kind == "res":
            x = residual_block(x, W, p, feat_cache, feat_idx)
        else:
            x = resample(x, W, p, args[1], feat_cache, feat_idx)
    x = F.silu(rms_norm(x, W["decoder.head.0.gamma"]))
    return _cached_conv(x, W, "decoder.head.2.", (1, 1, 1), feat_cache, feat_idx)


def _n_cache(W, part):
    """count_conv3d (:943-948) == number of feature-cache slots the forward pass consumes."""
    n = sum(1 for k in W if k.startswith(part) and k.endswith(".weight") and W[k].dim() == 5
            and ".shortcut." not in k)
    return n


def _scale(z_dim):
    mean = torch.tensor(VAE_MEAN[:z_dim]).to(BF16).view(1, z_dim, 1, 1, 1)
    inv_std = (1.0 / torch.tensor(VAE_STD[:z_dim])).to(BF16).view(1, z_dim, 1, 1, 1)
    return mean, inv_std


def vae_encode(x, W, cfg=VAE_CONFIG):
    """VideoVAE_.encode (:984-1009): chunks of [1, 4, 4, ...] frames; returns normalised mu."""
    z_dim = cfg["z_dim"]
    cache = [None] * (_n_cache(W, "encoder.") + 8)
    t = x.shape[2]
    outs = []
    for i in range(1 + (t - 1) // 4):
        idx = [0]
        chunk = x[:, :, :1] if i == 0 else x[:, :, 1 + 4 * (i - 1):1 + 4 * i]
        outs.append(encoder3d(chunk, W, cfg, cache, idx))
    out = torch.cat(outs, 2)
    mu = causal_conv3d(out, W["conv1.weight"], W["conv1.bias"], (0, 0, 0))[:, :z_dim]
    mean, inv_std = _scale(z_dim)
    return (mu - mean) * inv_std


def vae_decode(z, W, cfg=VAE_CONFIG):
    """VideoVAE_.decode (:1011-1034): one latent frame per chunk."""
    mean, inv_std = _scale(cfg["z_dim"])
    z = z / inv_std + mean
    x = causal_conv3d(z, W["conv2.weight"], W["conv2.bias"], (0, 0, 0))
    cache = [None] * (_n_cache(W, "decoder.") + 8)
    outs = []
    for i in range(z.shape[2]):
        idx = [0]
        outs.append(decoder3d(x[:, :, i:i + 1], W, cfg, cache, idx))
    return torch.cat(outs, 2)


# ------------------------------------------------------------------------------------------
# tiling (WanVideoVAE :1081-1247)
# ------------------------------------------------------------------------------------------
def tile_tasks(H, W, size, stride):
    """Task list of tiled_encode/tiled_decode (:1108-1115)."""
    tasks = []
    for h in range(0, H, stride[0]):
        if h - stride[0] >= 0 and h - stride[0] + size[0] >= H:
            continue
        for w in range(0, W, stride[1]):
            if w - stride[1] >= 0 and w - stride[1] + size[1] >= W:
                continue
            tasks.append((h, h + size[0], w, w + size[1]))
    return tasks


def _mask_1d(length, left_bound, right_bound, bw):
    x = torch.ones((length,))
    if not left_bound:
        x[:bw] = (torch.arange(bw) + 1) / bw
    if not right_bound:
        x[-bw:] = torch.flip((torch.arange(bw) + 1) / bw, dims=(0,))
    return x


def build_mask(H, W, is_bound, border):
    """build_mask (:1090-1100)."""
    h = _mask_1d(H, is_bound[0], is_bound[1], border[0])
    w = _mask_1d(W, is_bound[2], is_bound[3], border[1])
    m = torch.minimum(h[:, None].expand(H, W), w[None, :].expand(H, W))
    return m.view(1, 1, 1, H, W)


def tiled_encode(video, W, tile_size=(30, 52), tile_stride=(15, 26), cfg=VAE_CONFIG):
    """WanVideoVAE.encode(tiled=True) for one video (1, 3, T, H, W) bf16 (:1155-1203,1218-1232)."""
    f = 8
    size = (tile_size[0] * f, tile_size[1] * f)
    stride = (tile_stride[0] * f, tile_stride[1] * f)
    _, _, T, H, Wd = video.shape
    out_t = (T + 3) // 4
    weight = torch.zeros((1, 1, out_t, H // f, Wd // f), dtype=video.dtype)
    values = torch.zeros((1, cfg["z_dim"], out_t, H // f, Wd // f), dtype=video.dtype)
    for h, h_, w, w_ in tile_tasks(H, Wd, size, stride):
        hs = vae_encode(video[:, :, :, h:h_, w:w_], W, cfg)
        mask = build_mask(hs.shape[3], hs.shape[4], (h == 0, h_ >= H, w == 0, w_ >= Wd),
                          ((size[0] - stride[0]) // f, (size[1] - stride[1]) // f)).to(video.dtype)
        th, tw = h // f, w // f
        values[:, :, :, th:th + hs.shape[3], tw:tw + hs.shape[4]] += hs * mask
        weight[:, :, :, th:th + hs.shape[3], tw:tw + hs.shape[4]] += mask
    return values / weight


def tiled_decode(z, W, tile_size=(30, 52), tile_stride=(15, 26), cfg=VAE_CONFIG):
    """WanVideoVAE.decode(tiled=True) for one latent (1, 16, T, H, W) bf16 (:1103-1152)."""
    f = 8
    _, _, T, H, Wd = z.shape
    out_t = T * 4 - 3
    weight = torch.zeros((1, 1, out_t, H * f, Wd * f), dtype=z.dtype)
    values = torch.zeros((1, 3, out_t, H * f, Wd * f), dtype=z.dtype)
    for h, h_, w, w_ in tile_tasks(H, Wd, tile_size, tile_stride):
        v = vae_decode(z[:, :, :, h:h_, w:w_], W, cfg)
        mask = build_mask(v.shape[3], v.shape[4], (h == 0, h_ >= H, w == 0, w_ >= Wd),
                          ((tile_size[0] - tile_stride[0]) * f, (tile_size[1] - tile_stride[1]) * f)).to(z.dtype)
        values[:, :, :, h * f:h * f + v.shape[3], w * f:w * f + v.shape[4]] += v * mask
        weight[:, :, :, h * f:h * f + v.shape[3], w * f:w * f + v.shape[4]] += mask
    return (values / weight).clamp_(-1, 1)


def single_decode(z, W, cfg=VAE_CONFIG):
    """WanVideoVAE.single_decode (:1212-1215)."""
    return vae_decode(z, W, cfg).clamp_(-1, 1)


# ------------------------------------------------------------------------------------------
# VACE conditioning (WanVideoUnit_VACE.process, wan_video_new.py:861-920) and pixel I/O
# ------------------------------------------------------------------------------------------
def preprocess_video(frames_u8, min_value=-1.0, max_value=1.0):
    """BasePipeline.preprocess_video/preprocess_image (utils/__init__.py:60-73): uint8 (T, H, W, 3)
    -> bf16 (1, 3, T, H, W) computed as bf16(bf16(x) * bf16-op scale) + min."""
    x = frames_u8.to(torch.float32).to(BF16)
    x = x * ((max_value - min_value) / 255) + min_value
    return x.permute(3, 0, 1, 2).unsqueeze(0)


def encode_list(videos, W, tiled=False, tile_size=(34, 34), tile_stride=(18, 16), cfg=VAE_CONFIG):
    """WanVideoVAE.encode over a list of (3, T, H, W) videos (wan_video_vae.py:1218-1232) -> stacked
    latents.  Reproduces the reference's in-loop `tile_size = tile_size * upsampling_factor`
    (:1224-1225): the j-th video of the list is tiled with tile_size/stride x 8^j (latent units)."""
    outs = []
    ts, st = tuple(tile_size), tuple(tile_stride)
    for v in videos:
        v = v.unsqueeze(0)
        if tiled:
            outs.append(tiled_encode(v, W, ts, st, cfg)[0])
            ts, st = (ts[0] * 8, ts[1] * 8), (st[0] * 8, st[1] * 8)
        else:
            outs.append(vae_encode(v, W, cfg)[0])
    return torch.stack(outs)


def vace_context(W, vace_video=None, vace_video_mask=None, num_frames=None, height=None, width=None,
                 tiled=True, tile_size=(30, 52), tile_stride=(15, 26), cfg=VAE_CONFIG, vace_reference_image=None):
    """WanVideoUnit_VACE.process (wan_video_new.py:875-920): returns (1, 96, f + T', H/8, W/8), f = the
    number of reference images (preprocessed bf16 (1, 3, f, H, W) or None).  Reference images:
    each frame is encoded as its own video (:903-909), concatenated with 16 zero channels, and
    prepended along time to the video latents; the mask latents get f zero frames (:911-912)."""
    if vace_video is None:
        vace_video = torch.zeros((1, 3, num_frames, height, width), dtype=BF16)
    if vace_video_mask is None:
        vace_video_mask = torch.ones_like(vace_video)
    inactive = vace_video * (1 - vace_video_mask) + 0 * vace_video_mask
    reactive = vace_video * vace_video_mask + 0 * (1 - vace_video_mask)
    enc = (lambda v: tiled_encode(v, W, tile_size, tile_stride, cfg)) if tiled else \
        (lambda v: vae_encode(v, W, cfg))
    lat = torch.cat((enc(inactive), enc(reactive)), dim=1)
    m = vace_video_mask[0, 0]
    T, H, Wd = m.shape
    m = m.reshape(T, H // 8, 8, Wd // 8, 8).permute(2, 4, 0, 1, 3).reshape(1, 64, T, H // 8, Wd // 8)
    m = F.interpolate(m, size=((T + 3) // 4, H // 8, Wd // 8), mode="nearest-exact")
    if vace_reference_image is not None:
        f = vace_reference_image.shape[2]
        refs = [vace_reference_image[0, :, j:j + 1] for j in range(f)]
        rl = encode_list(refs, W, tiled, tile_size, tile_stride, cfg)              # (f, 16, 1, h, w)
        rl = torch.cat((rl, torch.zeros_like(rl)), dim=1)
        lat = torch.cat((*[u.unsqueeze(0) for u in rl], lat), dim=2)
        m = torch.cat((torch.zeros_like(m[:, :, :f]), m), dim=2)
    return torch.cat((lat, m), dim=1)


def vae_output_to_u8(video):
    """vae_output_to_video (utils/__init__.py:76-91) for B=1: (1,3,T,H,W) bf16 -> (T,H,W,3) uint8:
    mean over B, (x - (-1)) * (255/2) in bf16, clip, truncating cast."""
    x = video.float().mean(0).to(video.dtype).permute(1, 2, 3, 0)
    x = ((x - (-1)) * (255 / 2)).clip(0, 255)
    return x.to(torch.uint8)
