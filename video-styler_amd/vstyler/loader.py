"""Checkpoint loading with the reference's model detection (md5 of sorted 'key:shape' strings).

Reference: diffsynth/models/utils.py:65-88 (readers), :148-182 (hash), diffsynth/models/
model_manager.py:162-196 (detector), configs/model_config.py:142-179 (hash table),
wan_video_dit.py:506-536 / wan_video_vace.py:98-113 (hash -> config).  Serialized files are read
with safetensors or torch.load(weights_only=True) only.
"""
import hashlib
import os

import torch

from .models import VaceWanModel, WanModel

WAN_DIT_CONFIGS = {
    "9269f8db9040a9d860eaca435be61814": dict(dim=1536, ffn_dim=8960, num_heads=12, num_layers=30),   # 1.3B
    "aafcfd9672c3a2456dc46e1cb6e52c70": dict(dim=5120, ffn_dim=13824, num_heads=40, num_layers=40),  # 14B
}
WAN_COMMON = dict(in_dim=16, out_dim=16, text_dim=4096, freq_dim=256, eps=1e-6, patch_size=(1, 2, 2))
VACE_14B_HASH = "3b2726384e4f64837bdf216eea3f310d"
VACE_14B = dict(vace_layers=(0, 5, 10, 15, 20, 25, 30, 35), vace_in_dim=96, patch_size=(1, 2, 2),
                dim=5120, num_heads=40, ffn_dim=13824, eps=1e-6)
VACE_DEFAULT = dict(vace_layers=tuple(range(0, 30, 2)), vace_in_dim=96, patch_size=(1, 2, 2),
                    dim=1536, num_heads=12, ffn_dim=8960, eps=1e-6)   # VaceWanModel() defaults


def hash_state_dict_keys(state_dict, with_shape=True):
    """models/utils.py:148-182."""
    keys = []
    for key, value in state_dict.items():
        if isinstance(key, str) and isinstance(value, torch.Tensor):
            if with_shape:
                keys.append(key + ":" + "_".join(map(str, list(value.shape))))
            keys.append(key)
    keys.sort()
    return hashlib.md5(",".join(keys).encode("UTF-8")).hexdigest()


def load_state_dict(path, device="cpu", torch_dtype=None):
    if isinstance(path, (list, tuple)):
        sd = {}
        for p in path:
            sd.update(load_state_dict(p, device, torch_dtype))
        return sd
    if os.path.isdir(path):
        sd = {}
        for name in sorted(os.listdir(path)):
            if name.split(".")[-1] in ("safetensors", "bin", "ckpt", "pth", "pt"):
                sd.update(load_state_dict(os.path.join(path, name), device, torch_dtype))
        return sd
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path, device=str(device))
    else:
        sd = torch.load(path, map_location=device, weights_only=True)
    if torch_dtype is not None:
        sd = {k: (v.to(torch_dtype) if isinstance(v, torch.Tensor) and v.is_floating_point() else v)
              for k, v in sd.items()}
    return sd


_PREFIXES = ("model.diffusion_model.", "diffusion_model.")


def normalize_keys(state_dict):
    """ComfyUI / Kijai WanVideo checkpoints (the config-5 workflow's model files) carry the Wan key
    layout under a 'model.diffusion_model.' or 'diffusion_model.' prefix, fp8 e4m3fn linear weights
    and, in their '_scaled' variants, per-tensor '<name>.scale_weight' factors.  Strip the prefix and
    fold scale_weight into its weight (exact fp8 -> bf16 upcast, then the scale) so the reference's
    md5 key-layout detection applies unchanged.  Other layouts pass through."""
    sd = {}
    for k, v in state_dict.items():
        for pre in _PREFIXES:
            if k.startswith(pre):
                k = k[len(pre):]
                break
        sd[k] = v
    for k in [k for k in sd if k.endswith(".scale_weight")]:
        base = k[: -len(".scale_weight")] + ".weight"
        s = sd.pop(k)
        if base in sd:
            sd[base] = (sd[base].to(torch.float32) * s.to(torch.float32)).to(torch.bfloat16)
    sd.pop("scaled_fp8", None)
    return sd


def build_dit(state_dict, device):
    sd = {k: v for k, v in state_dict.items() if not k.startswith("vace")}
    h = hash_state_dict_keys(sd)
    if h not in WAN_DIT_CONFIGS:
        return None
    cfg = dict(WAN_COMMON, **WAN_DIT_CONFIGS[h])
    model = WanModel(device=device, **cfg)
    model.load_state_dict({k: v.to(torch.bfloat16) for k, v in sd.items()}, strict=True)
    return model


def build_vace(state_dict, device):
    sd = {k: v for k, v in state_dict.items() if k.startswith("vace")}
    if not sd:
        return None
    cfg = VACE_14B if hash_state_dict_keys(sd) == VACE_14B_HASH else VACE_DEFAULT
    model = VaceWanModel(device=device, **cfg)
    model.load_state_dict({k: v.to(torch.bfloat16) for k, v in sd.items()}, strict=True)
    return model


# configs/model_config.py:163-164 -- the two Wan2.1 VAE file layouts (WanVideoVAE, z_dim 16)
WAN_VAE_HASHES = ("1378ea763357eea97acdef78e65d6d96", "ccc42284ea13e1ad04693284c7a09be6")


def build_vae(state_dict, device):
    """WanVideoVAE (wan_video_vae.py:1058) from the civitai layout (optionally under 'model_state')."""
    sd = state_dict.get("model_state", state_dict)
    if hash_state_dict_keys(sd) not in WAN_VAE_HASHES and \
            not ("encoder.conv1.weight" in sd and "decoder.head.2.weight" in sd and "conv2.weight" in sd):
        return None
    from .vae import WanVideoVAE
    z_dim = sd["conv2.weight"].shape[0]
    if z_dim != 16:
        return None  # the 48-channel Wan2.2 VAE (WanVideoVAE38) is out of scope
    return WanVideoVAE(z_dim=z_dim, dim=sd["encoder.conv1.weight"].shape[0], device=device).load_state_dict(sd)


T5_HASH = "9c8818c2cbea55eca56c7b447df170da"   # configs/model_config.py:161 (WanTextEncoder)


def build_text_encoder(state_dict, device):
    if hash_state_dict_keys(state_dict) != T5_HASH:
        return None
    from .t5 import WanTextEncoder
    return WanTextEncoder(device=device).load_state_dict(state_dict)


def load_models(paths, device="cuda"):
    """Returns {'wan_video_dit': WanModel, 'wan_video_vace': VaceWanModel, ...} for the files given."""
    out = {}
    for path in paths:
        sd = normalize_keys(load_state_dict(path, device="cpu"))
        vae = build_vae(sd, device)
        if vae is not None:
            out["wan_video_vae"] = vae
            continue
        te = build_text_encoder(sd, device)
        if te is not None:
            out["wan_video_text_encoder"] = te
            continue
        if sd and all(k.startswith("vace") for k in sd):
            # a VACE-module-only file (the ComfyUI workflow's WanVideoVACEModelSelect input)
            out["wan_video_vace"] = build_vace(sd, device)
            continue
        dit = build_dit(sd, device)
        if dit is not None:
            out["wan_video_dit"] = dit
            vace = build_vace(sd, device)
            if vace is not None:
                out["wan_video_vace"] = vace
            continue
        raise NotImplementedError(f"unrecognised checkpoint {path} (hash {hash_state_dict_keys(sd)})")
    return out
