"""LoRA for the VACE/DiT linears.

merge_lora   : GeneralLoRALoader.load (diffsynth/lora/__init__.py:11-45): W <- W + alpha*(B@A),
               computed by the MFMA GEMM with the VS_EPI_RES epilogue (bf16 mm, *alpha, + W).
hotload_lora : AutoWrappedLinear hot-load (vram_management/layers.py:180-182, pipeline
               wan_video_new.py:96-103): y = W x + b + sum_i B_i (alpha_i A_i x), fused into the main
               GEMM as a second K phase (the "LoRA-fused linear" of BASELINE config 3).  Like the
               reference's lora_A_weights / lora_B_weights lists, hot-loads accumulate: the padded
               A_i are stacked along the rank rows and the B_i along the rank columns, so several
               adapters stay ONE K phase (sum_i (x A_i^T) B_i^T = (x [A_1; A_2]^T) [B_1 B_2]^T).
"""
import torch

from . import kernels as K
from .models import Linear

BF16 = torch.bfloat16


def load_lora_state_dict(lora_config, device):
    from .loader import load_state_dict
    if isinstance(lora_config, str):
        path = lora_config
    else:
        lora_config.download_if_necessary()
        path = lora_config.path
    return normalize_lora_keys(load_state_dict(path, device=device, torch_dtype=BF16))


def normalize_lora_keys(sd):
    """Map the kohya/ComfyUI layout used by CausVid-style Wan LoRAs ('<name>.lora_down.weight' = A,
    '<name>.lora_up.weight' = B, optional '<name>.alpha' scalar, scale alpha / rank) onto the
    reference's lora_A/lora_B layout (the alpha/rank scale folded into B); other keys pass through."""
    out = {}
    for key, val in sd.items():
        if key.endswith(".lora_down.weight"):
            base = key[: -len(".lora_down.weight")]
            up = sd[base + ".lora_up.weight"]
            scale = 1.0
            if base + ".alpha" in sd:
                scale = float(sd[base + ".alpha"]) / val.shape[0]
            out[base + ".lora_A.weight"] = val
            out[base + ".lora_B.weight"] = up if scale == 1.0 else (up.float() * scale).to(up.dtype)
        elif key.endswith(".lora_up.weight") or key.endswith(".alpha"):
            continue
        else:
            out[key] = val
    return out


def get_name_dict(lora_state_dict):
    """lora/__init__.py:11-25: '<prefix>.<name>.lora_B[.default].weight' -> module name."""
    names = {}
    for key in lora_state_dict:
        if ".lora_B." not in key:
            continue
        keys = key.split(".")
        if len(keys) > keys.index("lora_B") + 2:
            keys.pop(keys.index("lora_B") + 1)
        keys.pop(keys.index("lora_B"))
        if keys[0] == "diffusion_model":
            keys.pop(0)
        keys.pop(-1)
        names[".".join(keys)] = (key, key.replace(".lora_B.", ".lora_A."))
    return names


def _padded(t, rows=None, cols=None):
    """zero-pad a 2-D bf16 matrix so its K dim is a multiple of 64 (exact for a low-rank product)."""
    r, c = t.shape
    rr = rows or r
    cc = cols or c
    if (rr, cc) == (r, c) and t.is_contiguous():
        return t
    out = torch.zeros((rr, cc), dtype=t.dtype, device=t.device)
    out[:r, :c] = t
    return out


def merge_lora(model, lora, alpha=1.0):
    updated = 0
    names = get_name_dict(lora)
    for name, module in model.named_modules():
        if name in names and isinstance(module, Linear):
            up = lora[names[name][0]].to(device=module.weight.device, dtype=BF16)     # B: [out, r]
            down = lora[names[name][1]].to(device=module.weight.device, dtype=BF16)   # A: [r, in]
            if up.dim() == 4:
                up, down = up[:, :, 0, 0], down[:, :, 0, 0]
            r = up.shape[1]
            rp = (r + 63) // 64 * 64
            b_mat = _padded(up, cols=rp)                          # [out, rp]
            a_t = _padded(down.t().contiguous(), cols=rp)         # [in, rp]
            w = module.weight
            K.gemm(b_mat, a_t, w, epilogue=K.VS_EPI_RES, residual=w, alpha=float(alpha))
            w8 = getattr(module, "weight_fp8", None)
            if w8 is not None:
                # quantize_fp8_ ran first (config-5 order): refresh the e4m3 copy linear() reads, in
                # place so the fused q|k|v / k|v e4m3 buffer it may be a view of sees it too
                w8.copy_(w.detach().to(torch.float8_e4m3fn).view(torch.uint8))
            updated += 1
    print(f"{updated} tensors are updated by LoRA.")
    return updated


def hotload_lora(model, lora, alpha=1.0):
    """Attach (alpha*A, B) to each matching Linear (layers.py:180-182 appends to the layer's lists);
    an adapter already attached stays and the new one is stacked onto it.  The GEMM adds them all as
    one fused K phase.  fp8 layers take no hot-loaded LoRA (gap vs the reference's AutoWrappedLinear,
    layers.py:168-180, which adds the unmerged term after fp8_linear): merge instead.  Every matching
    module is checked before any is touched, so a refused call leaves the model unchanged."""
    targets = []
    for name, module in model.named_modules():
        if not isinstance(module, Linear):
            continue
        ka, kb = f"{name}.lora_A.default.weight", f"{name}.lora_B.default.weight"
        if ka in lora and kb in lora:
            targets.append((name, module, ka, kb))
    fp8 = [name for name, module, _, _ in targets if getattr(module, "weight_fp8", None) is not None]
    if fp8:
        raise NotImplementedError(f"hot-loaded LoRA on fp8 layers ({', '.join(fp8[:3])}"
                                  f"{', ...' if len(fp8) > 3 else ''}): merge the LoRA instead")
    updated = 0
    for name, module, ka, kb in targets:
        a = (lora[ka].to(device=module.weight.device, dtype=BF16) * alpha).to(BF16)   # [r, in]
        b = lora[kb].to(device=module.weight.device, dtype=BF16)                       # [out, r]
        rp = (a.shape[0] + 63) // 64 * 64
        a, b = _padded(a, rows=rp), _padded(b, cols=rp)   # [rp, in], [out, rp]
        if getattr(module, "lora_A", None) is not None:
            a = torch.cat([module.lora_A, a], dim=0)
            b = torch.cat([module.lora_B, b], dim=1).contiguous()
        module.lora_A, module.lora_B = a, b
        updated += 1
    return updated
