"""Test helpers for the VAE: a torch-CPU *whole-sequence* restatement (the formulation the product
`vstyler/vae.py` runs) built from the oracle's primitives, used to prove on the CPU that it equals
the reference's chunked feature-cache algorithm (oracle/wan_vae_oracle.py)."""
import torch
import torch.nn.functional as F

from oracle import wan_vae_oracle as V

TINY_VAE = dict(dim=32, z_dim=16, dim_mult=(1, 2, 4, 4), num_res_blocks=2, temperal_downsample=(False, True, True))


def _conv3(x, W, p):
    return V.causal_conv3d(x, W[p + "weight"], W[p + "bias"], (1, 1, 1))


def _res(x, W, p):
    h = V.causal_conv3d(x, W[p + "shortcut.weight"], W[p + "shortcut.bias"], (0, 0, 0)) \
        if p + "shortcut.weight" in W else x
    x = F.silu(V.rms_norm(x, W[p + "residual.0.gamma"]))
    x = _conv3(x, W, p + "residual.2.")
    x = F.silu(V.rms_norm(x, W[p + "residual.3.gamma"]))
    return _conv3(x, W, p + "residual.6.") + h


def _spatial(x, W, p, mode):
    b, c, t, h, w = x.shape
    x2 = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    if mode.startswith("up"):
        x2 = V.conv2d(V.upsample_nearest2x(x2), W[p + "resample.1.weight"], W[p + "resample.1.bias"], padding=1)
    else:
        x2 = V.conv2d(F.pad(x2, (0, 1, 0, 1)), W[p + "resample.1.weight"], W[p + "resample.1.bias"], stride=2)
    return x2.reshape(b, t, *x2.shape[1:]).permute(0, 2, 1, 3, 4)


def _resample(x, W, p, mode):
    b, c, t, h, w = x.shape
    if mode == "upsample3d":
        if t > 1:
            y = V.causal_conv3d(x[:, :, 1:], W[p + "time_conv.weight"], W[p + "time_conv.bias"], (1, 0, 0))
            y = y.reshape(b, 2, c, t - 1, h, w)
            y = torch.stack((y[:, 0], y[:, 1]), 3).reshape(b, c, 2 * (t - 1), h, w)
            x = torch.cat([x[:, :, :1], y], 2)
    x = _spatial(x, W, p, mode)
    if mode == "downsample3d" and x.shape[2] > 1:
        y = V.causal_conv3d(x, W[p + "time_conv.weight"], W[p + "time_conv.bias"], (0, 0, 0), stride=(2, 1, 1))
        x = torch.cat([x[:, :, :1], y], 2)
    return x


def encode_whole(x, W, cfg):
    t = 1 + 4 * ((x.shape[2] - 1) // 4)
    x = _conv3(x[:, :, :t], W, "encoder.conv1.")
    layers, _ = V.encoder_layers(cfg)
    for kind, p, args in layers:
        x = _res(x, W, p) if kind == "res" else _resample(x, W, p, args[1])
    x = _res(x, W, "encoder.middle.0.")
    x = V.attention_block(x, W, "encoder.middle.1.")
    x = _res(x, W, "encoder.middle.2.")
    x = _conv3(F.silu(V.rms_norm(x, W["encoder.head.0.gamma"])), W, "encoder.head.2.")
    mu = V.causal_conv3d(x, W["conv1.weight"], W["conv1.bias"], (0, 0, 0))[:, :cfg["z_dim"]]
    mean, inv_std = V._scale(cfg["z_dim"])
    return (mu - mean) * inv_std


def decode_whole(z, W, cfg):
    mean, inv_std = V._scale(cfg["z_dim"])
    x = V.causal_conv3d(z / inv_std + mean, W["conv2.weight"], W["conv2.bias"], (0, 0, 0))
    x = _conv3(x, W, "decoder.conv1.")
    x = _res(x, W, "decoder.middle.0.")
    x = V.attention_block(x, W, "decoder.middle.1.")
    x = _res(x, W, "decoder.middle.2.")
    layers, _ = V.decoder_layers(cfg)
    for kind, p, args in layers:
        x = _res(x, W, p) if kind == "res" else _resample(x, W, p, args[1])
    return _conv3(F.silu(V.rms_norm(x, W["decoder.head.0.gamma"])), W, "decoder.head.2.")


def synthetic_video(frames, height, width, seed=7):
    """bf16 (1, 3, T, H, W) in [-1, 1]: smooth gradients + noise (a natural-ish video)."""
    g = torch.Generator().manual_seed(seed)
    t = torch.linspace(0, 1, frames).view(1, 1, frames, 1, 1)
    yy = torch.linspace(-1, 1, height).view(1, 1, 1, height, 1)
    xx = torch.linspace(-1, 1, width).view(1, 1, 1, 1, width)
    base = torch.cat([torch.sin(3 * xx + 2 * t) * torch.cos(2 * yy), yy * xx + t - 0.5,
                      torch.cos(4 * yy - t) * 0.8 + 0 * xx], dim=1)
    v = base + 0.15 * torch.randn((1, 3, frames, height, width), generator=g)
    return v.clamp(-1, 1).to(torch.bfloat16)
