"""Model-level parity at the BASELINE production shapes ('a parity check at any BASELINE
production shape').  The oracle restatement (oracle/wan_oracle.py) runs through torch's GPU ops here
-- the same functions the CPU tests use, device-agnostic, attention chunked per (batch, head) -- once
with fp32 and once with fp64 accumulation; the product forward (libvstyler kernels) must stay within
NOISE_X times that fp32/fp64 noise floor of the fp32 oracle (max-abs and rel-L2 on the velocity, the
SURVEY §8d metric).  The product path never imports the oracle.

  * C3 shape: Wan2.1-VACE-14B dims (D 5120, F 13 824, 40 heads) at 832x480x73 (S = 29 640) as a
    CFG batch-2 forward of ONE main DiT block and ONE VACE block (wan_video_dit.py:196-230,
    wan_video_vace.py:5-87, model_fn_wan_video wan_video_new.py:1338-1468), with a Ditto-format
    rank-128 LoRA on the VACE block (self/cross q,k,v,o, ffn.0, ffn.2; lora/__init__.py:28-45)
    merged, and hot-loaded (AutoWrappedLinear's unmerged term, layers.py:180-182);
  * C2: Wan2.1-VACE-1.3B (30 + 15 blocks) single forward at 832x480x73.
"""
import pytest
import torch

from oracle import wan_oracle as O
from gpu_util import BF16

pytestmark = pytest.mark.gpu
NOISE_X = 1.5


def floor_check(out, ref32, ref64, tag):
    o, r, r64 = out.float(), ref32.float(), ref64.float()
    mx, rl = (o - r).abs().max().item(), ((o - r).norm() / r.norm()).item()
    fmx, frl = (r - r64).abs().max().item(), ((r - r64).norm() / r64.norm()).item()
    print(f"{tag}: max-abs {mx:.4g} rel-L2 {rl:.4g} (noise floor {fmx:.4g} / {frl:.4g})")
    assert mx <= NOISE_X * fmx + 1e-3 and rl <= NOISE_X * frl + 1e-4, (tag, mx, rl, fmx, frl)


def oracle_both(fn):
    """fn() under fp32 and fp64 accumulation (the oracle's two valid rounding orders)."""
    out32 = fn()
    O.ACC_DTYPE = torch.float64
    try:
        out64 = fn()
    finally:
        O.ACC_DTYPE = torch.float32
    return out32, out64


def build(cfg, W):
    from vstyler.models import VaceWanModel, WanModel
    dit = WanModel(dim=cfg["dim"], in_dim=16, ffn_dim=cfg["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256,
                   eps=1e-6, patch_size=(1, 2, 2), num_heads=cfg["num_heads"], num_layers=cfg["num_layers"],
                   device="cuda")
    dit.load_state_dict({k: v for k, v in W.items() if not k.startswith("vace")})
    vace = VaceWanModel(vace_layers=cfg["vace_layers"], dim=cfg["dim"], num_heads=cfg["num_heads"],
                        ffn_dim=cfg["ffn_dim"], device="cuda")
    vace.load_state_dict({k: v for k, v in W.items() if k.startswith("vace")})
    return dit, vace


def gpu_weights(cfg, seed):
    """O.random_weights' layout and init rules, drawn on the GPU (a 14B-dim block is too slow to draw
    on the host): same names, shapes and distributions; any seeded draw is a valid test input."""
    shapes = O.dit_param_shapes(cfg)
    shapes.update(O.vace_param_shapes(cfg))
    g = torch.Generator(device="cuda").manual_seed(seed)
    W = {}
    for name, shape in shapes.items():
        x = torch.randn(shape, generator=g, device="cuda")
        if name.endswith("modulation"):
            x = x / cfg["dim"] ** 0.5
        elif "norm" in name and name.endswith("weight"):
            x = 1 + 0.1 * x
        elif name.endswith("bias"):
            x = 0.01 * x
        else:
            x = 0.02 * x
        W[name] = x.to(BF16)
    return W


def inputs(cfg, batch_ctx):
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 73, 480, 832)
    ctx = torch.cat([cp, cn])[:batch_ctx]
    return lat.cuda(), ctx.cuda(), vc.cuda()


DITTO_TARGETS = [f"{a}.{l}" for a in ("self_attn", "cross_attn") for l in "qkvo"] + ["ffn.0", "ffn.2"]


@pytest.mark.parametrize("lora", ["merge", "hotload"])
def test_c3_14b_block_pair_ditto_lora_832x480x73(lora):
    from vstyler import model_fn_wan_video
    from vstyler.lora import hotload_lora, merge_lora
    cfg = dict(O.WAN_CONFIGS["14B"], num_layers=1, vace_layers=(0,))
    W = gpu_weights(cfg, seed=7)
    dit, vace = build(cfg, W)
    # Ditto LoRA (train.sh: rank 128 on the VACE blocks), keys in the reference's peft layout
    g = torch.Generator(device="cuda").manual_seed(8)
    r, D, F = 128, cfg["dim"], cfg["ffn_dim"]
    lora_sd = {}
    for t in DITTO_TARGETS:
        out_f, in_f = {"ffn.0": (F, D), "ffn.2": (D, F)}.get(t, (D, D))
        lora_sd[f"vace_blocks.0.{t}.lora_A.default.weight"] = (0.02 * torch.randn(r, in_f, generator=g, device="cuda")).to(BF16)
        lora_sd[f"vace_blocks.0.{t}.lora_B.default.weight"] = (0.02 * torch.randn(out_f, r, generator=g, device="cuda")).to(BF16)
    alpha = 1.0
    if lora == "merge":
        assert merge_lora(vace, lora_sd, alpha=alpha) == len(DITTO_TARGETS)
    else:
        assert hotload_lora(vace, lora_sd, alpha=alpha) == len(DITTO_TARGETS)
    # oracle: GeneralLoRALoader's bf16 merge, or the hot-loaded term per linear (lora_linear)
    Wm = dict(W)
    for t in DITTO_TARGETS:
        key = f"vace_blocks.0.{t}.weight"
        la, lb = (lora_sd[f"vace_blocks.0.{t}.lora_{x}.default.weight"] for x in "AB")
        if lora == "merge":
            Wm[key] = O.lora_merge(W[key], lb, la, alpha)
        else:
            O.HOTLOAD[id(W[key])] = (O.bf(la.float() * alpha), lb)
    lat, ctx, vc = inputs(cfg, 2)
    t = torch.tensor([937.5], device="cuda").to(BF16)
    out = model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc)
    torch.cuda.synchronize()
    try:
        ref32, ref64 = oracle_both(lambda: O.model_fn(Wm, cfg, torch.cat([lat, lat]), t.expand(2), ctx,
                                                      torch.cat([vc, vc])))
    finally:
        O.HOTLOAD.clear()
    floor_check(out, ref32, ref64, f"C3 14B 1+1 blocks 832x480x73 CFG2, Ditto LoRA {lora}")


def test_c2_1p3b_forward_832x480x73():
    from vstyler import model_fn_wan_video
    cfg = O.WAN_CONFIGS["1.3B"]
    W = gpu_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    lat, ctx, vc = inputs(cfg, 1)
    t = torch.tensor([1000.0], device="cuda").to(BF16)
    out = model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc)
    torch.cuda.synchronize()
    ref32, ref64 = oracle_both(lambda: O.model_fn(W, cfg, lat, t, ctx, vc))
    floor_check(out, ref32, ref64, "C2 1.3B 30+15 blocks 832x480x73 forward")
