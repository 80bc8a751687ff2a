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
MAIN_LAYERS_BY_DIM = {1536: 30, 5120: 40}
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


def _n_blocks(sd, prefix):
    ids = {int(k.split(".")[1]) for k in sd if k.startswith(prefix + ".") and k.split(".")[1].isdigit()}
    return len(ids)


def dit_config_from_shapes(sd):
    """Extension for checkpoints whose key hash the reference's table does not list (fine-tunes of
    another width, the tiny test checkpoints): the WanModel config read off the tensor shapes of the
    Wan key layout (wan_video_dit.py:272-308; head_dim 128 as every Wan2.1 model, patch 1x2x2).
    None when the layout is not a Wan DiT."""
    need = ("patch_embedding.weight", "blocks.0.ffn.0.weight", "text_embedding.0.weight",
            "time_embedding.0.weight", "head.head.weight")
    if not all(k in sd for k in need):
        return None
    pe = sd["patch_embedding.weight"]
    if tuple(pe.shape[2:]) != (1, 2, 2):
        return None
    dim = pe.shape[0]
    return dict(WAN_COMMON, dim=dim, in_dim=pe.shape[1], ffn_dim=sd["blocks.0.ffn.0.weight"].shape[0],
                num_heads=dim // 128, num_layers=_n_blocks(sd, "blocks"),
                text_dim=sd["text_embedding.0.weight"].shape[1], freq_dim=sd["time_embedding.0.weight"].shape[1],
                out_dim=sd["head.head.weight"].shape[0] // 4)


def vace_config_from_shapes(sd, num_layers):
    """The VaceWanModel config of a VACE key set outside the hash table: widths off the shapes, the
    n VACE blocks spread evenly over the main blocks (range(0, L, L // n): (0,2,..,28) for 1.3B,
    (0,5,..,35) for 14B, the two published layouts, wan_video_vace.py:98-113)."""
    pe = sd["vace_patch_embedding.weight"]
    dim, n = pe.shape[0], _n_blocks(sd, "vace_blocks")
    step = max(1, num_layers // n) if num_layers else 2
    return dict(vace_layers=tuple(range(0, n * step, step)), vace_in_dim=pe.shape[1], patch_size=(1, 2, 2),
                dim=dim, num_heads=dim // 128, ffn_dim=sd["vace_blocks.0.ffn.0.weight"].shape[0], eps=1e-6)


def build_dit(state_dict, device):
    sd = {k: v for k, v in state_dict.items() if not k.startswith("vace")}
    h = hash_state_dict_keys(sd)
    if h in WAN_DIT_CONFIGS:
        cfg = dict(WAN_COMMON, **WAN_DIT_CONFIGS[h])
    else:
        cfg = dit_config_from_shapes(sd)
        if cfg is None:
            return None
    model = WanModel(device=device, **cfg)
    model.load_state_dict({k: v.to(torch.bfloat16) for k, v in sd.items()}, strict=True)
    return model


def build_vace(state_dict, device, num_layers=None):
    sd = {k: v for k, v in state_dict.items() if k.startswith("vace")}
    if not sd:
        return None
    h = hash_state_dict_keys(sd)
    if h == VACE_14B_HASH:
        cfg = VACE_14B
    elif sd["vace_patch_embedding.weight"].shape[0] == VACE_DEFAULT["dim"] and \
            _n_blocks(sd, "vace_blocks") == len(VACE_DEFAULT["vace_layers"]):
        cfg = VACE_DEFAULT
    else:
        if not num_layers:
            # the main-block count fixes the injection spacing; without the DiT it is known only for
            # the two published widths (wan_video_dit.py:509-536: 1536 -> 30 blocks, 5120 -> 40)
            num_layers = MAIN_LAYERS_BY_DIM.get(sd["vace_patch_embedding.weight"].shape[0])
            if not num_layers:
                raise ValueError("VACE module of an unlisted layout and width: load it together with its DiT "
                                 "so the injection layers follow the DiT's block count")
        cfg = vace_config_from_shapes(sd, num_layers)
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


def t5_config_from_shapes(sd):
    """The WanTextEncoder config of a UMT5 key set the hash table does not list (other widths, the
    tiny test checkpoints), read off the shapes of wan_video_text_encoder.py:209-252's layout
    (shared_pos=False, head_dim 64).  None when the layout is not that encoder's."""
    need = ("token_embedding.weight", "norm.weight", "blocks.0.attn.q.weight", "blocks.0.ffn.fc1.weight",
            "blocks.0.pos_embedding.embedding.weight")
    if not all(k in sd for k in need):
        return None
    vocab, dim = sd["token_embedding.weight"].shape
    dim_attn = sd["blocks.0.attn.q.weight"].shape[0]
    num_buckets, num_heads = sd["blocks.0.pos_embedding.embedding.weight"].shape
    if dim_attn != 64 * num_heads:
        return None
    return dict(vocab=vocab, dim=dim, dim_attn=dim_attn, dim_ffn=sd["blocks.0.ffn.fc1.weight"].shape[0],
                num_heads=num_heads, num_layers=_n_blocks(sd, "blocks"), num_buckets=num_buckets)


def build_text_encoder(state_dict, device):
    if hash_state_dict_keys(state_dict) == T5_HASH:
        cfg = {}
    else:
        cfg = t5_config_from_shapes(state_dict)
        if cfg is None:
            return None
    from .t5 import WanTextEncoder
    return WanTextEncoder(device=device, **cfg).load_state_dict(state_dict)


def load_models(paths, device="cuda"):
    """Returns {'wan_video_dit': WanModel, 'wan_video_vace': VaceWanModel, ...} for the files given."""
    out = {}
    vace_only = []
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
            # a VACE-module-only file (the ComfyUI workflow's WanVideoVACEModelSelect input): built
            # once every file is read, with the DiT's block count when a DiT came with it
            vace_only.append(sd)
            continue
        dit = build_dit(sd, device)
        if dit is not None:
            out["wan_video_dit"] = dit
            vace = build_vace(sd, device, num_layers=len(dit.blocks))
            if vace is not None:
                out["wan_video_vace"] = vace
            continue
        raise NotImplementedError(f"unrecognised checkpoint {path} (hash {hash_state_dict_keys(sd)})")
    dit = out.get("wan_video_dit")
    for sd in vace_only:
        out["wan_video_vace"] = build_vace(sd, device, num_layers=len(dit.blocks) if dit is not None else None)
    return out
