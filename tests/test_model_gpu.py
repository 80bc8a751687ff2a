"""Model-level parity on the GPU: model_fn / 2-step denoise vs the oracle and the golden fixtures.

Tolerance (max-abs and rel-L2 on latents, the metric of SURVEY.md §8d): at most NOISE_X times the
intrinsic bf16 noise floor of the same computation, measured by running the oracle once with fp32
and once with fp64 accumulation (two equally valid rounding orders; stored in the golden file by
tests/golden/make_golden.py).  Measured floor for C1 (1.3B shape, 45 blocks, 2 steps, CFG 5):
max-abs 0.180 / rel-L2 0.0381; tiny: 0.039 / 0.0067."""
import os

import numpy as np
import pytest
import torch

from oracle import wan_oracle as O
from gpu_util import BF16, err

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOISE_X = 1.5


def within_floor(out, ref, floor, tag):
    mx, rl = err(out, ref)
    fmx, frl = float(floor[0]), float(floor[1])
    print(f"{tag}: max-abs {mx:.4g} rel-L2 {rl:.4g} (noise floor {fmx:.4g} / {frl:.4g})")
    assert mx <= NOISE_X * fmx + 1e-3 and rl <= NOISE_X * frl + 1e-4, (mx, rl, fmx, frl)


def bfarr(a):
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


def build(cfg, W, device="cuda"):
    from vstyler.models import VaceWanModel, WanModel
    dit = WanModel(dim=cfg["dim"], in_dim=16, ffn_dim=cfg["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256,
                   eps=1e-6, patch_size=(1, 2, 2), num_heads=cfg["num_heads"], num_layers=cfg["num_layers"],
                   device=device)
    dit.load_state_dict({k: v for k, v in W.items() if not k.startswith("vace")})
    vace = VaceWanModel(vace_layers=cfg["vace_layers"], dim=cfg["dim"], num_heads=cfg["num_heads"],
                        ffn_dim=cfg["ffn_dim"], device=device)
    vace.load_state_dict({k: v for k, v in W.items() if k.startswith("vace")})
    return dit, vace


@pytest.fixture(scope="module")
def tiny():
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    return cfg, W, dit, vace


def test_model_fn_tiny_matches_oracle(tiny):
    from vstyler import model_fn_wan_video
    cfg, W, dit, vace = tiny
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([1000.0]).to(BF16)
    ref = O.model_fn(W, cfg, lat, t, cp, vc)
    out = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t.cuda(), context=cp.cuda(),
                             vace_context=vc.cuda())
    mx, rl = err(out, ref)
    assert rl < 2e-2 and mx < 0.1, (mx, rl)


def test_model_fn_batched_cfg_equals_two_calls(tiny):
    from vstyler import model_fn_wan_video
    cfg, W, dit, vace = tiny
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([833.3333]).to(BF16).cuda()
    both = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=torch.cat([cp, cn]).cuda(),
                              vace_context=vc.cuda())
    p = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=cp.cuda(), vace_context=vc.cuda())
    n = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=cn.cuda(), vace_context=vc.cuda())
    assert torch.equal(both[0:1], p) and torch.equal(both[1:2], n)


def test_cfg_shared_prefix_bit_identical(tiny):
    """The first DiT / VACE block's phases 1-3 computed once for both CFG samples (host option
    cfg_prefix, default on) give the batch-2 forward of the option off bit for bit, and the forward of
    per-sample latents (no shared prefix possible) agrees with both."""
    from vstyler import model_fn_wan_video
    from vstyler.options import host_options
    cfg, W, dit, vace = tiny
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([777.0]).to(BF16).cuda()
    ctx = torch.cat([cp, cn]).cuda()
    outs = []
    for on in (1, 0):
        with host_options(cfg_prefix=on):
            outs.append(model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=ctx,
                                           vace_context=vc.cuda()).clone())
    lat2 = torch.cat([lat, lat]).cuda()          # batch-2 latents: the shared-prefix test cannot apply
    outs.append(model_fn_wan_video(dit, vace=vace, latents=lat2, timestep=t, context=ctx,
                                   vace_context=torch.cat([vc, vc]).cuda()))
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_denoise_tiny_vs_golden(tiny):
    from vstyler import WanVideoPipeline
    cfg, W, dit, vace = tiny
    z = np.load(os.path.join(GOLD, "tiny_2step.npz"))
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    out = pipe.denoise(lat, cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=2)
    within_floor(out, bfarr(z["latents_out"]).view(out.shape), z["noise_latents"], "tiny 2-step")


def test_pipeline_call_surface_tiny(tiny):
    """WanVideoPipeline.__call__ with seed noise (utils/__init__.py:117-122) and precomputed embeddings."""
    from vstyler import WanVideoPipeline
    cfg, W, dit, vace = tiny
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    out = pipe(prompt_emb=cp, negative_prompt_emb=cn, vace_context=vc, seed=1, height=128, width=128, num_frames=5,
               num_inference_steps=2, output_type="latents")
    z = np.load(os.path.join(GOLD, "tiny_2step.npz"))
    assert err(out, bfarr(z["latents_out"]).view(out.shape))[0] < 0.1


def test_c1_1p3b_shape_2step_vs_golden():
    """BASELINE config 0 (C1): random-init 1.3B-shape DiT+VACE (30+15 blocks), 2 steps, 128x128x5."""
    from vstyler import WanVideoPipeline
    cfg = O.WAN_CONFIGS["1.3B"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    z = np.load(os.path.join(GOLD, "c1_1p3b_2step.npz"))
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    out = pipe.denoise(lat, cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=2)
    within_floor(out, bfarr(z["latents_out"]).view(out.shape), z["noise_latents"], "C1 2-step latents")
    from vstyler import model_fn_wan_video
    t = torch.tensor([1000.0]).to(BF16).cuda()
    v = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=cp.cuda(), vace_context=vc.cuda())
    within_floor(v, bfarr(z["v_first"]).view(v.shape), z["noise_v_first"], "C1 single forward")


def test_lora_merge_and_hotload():
    from vstyler.lora import hotload_lora, merge_lora
    from vstyler.models import Linear
    import torch.nn as nn
    g = torch.Generator().manual_seed(90)
    D, r = 256, 32
    m = nn.Module()
    m.add_module("q", Linear(D, D, device="cuda"))
    w = (0.05 * torch.randn(D, D, generator=g)).to(BF16)
    b = (0.01 * torch.randn(D, generator=g)).to(BF16)
    m.q.weight.data.copy_(w)
    m.q.bias.data.copy_(b)
    up = (0.05 * torch.randn(D, r, generator=g)).to(BF16)
    down = (0.05 * torch.randn(r, D, generator=g)).to(BF16)
    lora = {"diffusion_model.q.lora_B.default.weight": up, "diffusion_model.q.lora_A.default.weight": down}
    merge_lora(m, lora, alpha=0.7)
    ref = O.lora_merge(w, up, down, 0.7)
    mx, _ = err(m.q.weight, ref)
    assert mx <= 2 ** -8, mx
    # hot-load: fused second K phase
    m.q.weight.data.copy_(w)
    hotload_lora(m, {"q.lora_A.default.weight": down, "q.lora_B.default.weight": up}, alpha=0.7)
    from vstyler.models import Workspace, linear
    x = (torch.randn(100, D, generator=g)).to(BF16)
    out = torch.empty(100, D, dtype=BF16, device="cuda")
    linear(m.q, x.cuda(), out, Workspace("cuda"))
    ref = O.lora_linear(x, w, b, O.bf(down.float() * 0.7), up)
    assert err(out, ref)[1] < 1e-2


def test_two_hotloaded_loras_add_up():
    """Two hot-loads on one Linear accumulate like the reference's lora_A_weights / lora_B_weights
    lists (layers.py:180-182, forward :183-185: out + x A1^T B1^T + x A2^T B2^T); ranks 32 and 96
    (padded to 64 and 128, stacked into one K phase)."""
    from vstyler.lora import hotload_lora
    from vstyler.models import Linear, Workspace, linear
    import torch.nn as nn
    g = torch.Generator().manual_seed(92)
    D = 256
    m = nn.Module()
    m.add_module("q", Linear(D, D, device="cuda"))
    w = (0.05 * torch.randn(D, D, generator=g)).to(BF16)
    b = (0.01 * torch.randn(D, generator=g)).to(BF16)
    m.q.weight.data.copy_(w)
    m.q.bias.data.copy_(b)
    adapters = []
    for r, alpha in ((32, 0.7), (96, 1.3)):
        up = (0.05 * torch.randn(D, r, generator=g)).to(BF16)
        down = (0.05 * torch.randn(r, D, generator=g)).to(BF16)
        assert hotload_lora(m, {"q.lora_A.default.weight": down, "q.lora_B.default.weight": up}, alpha=alpha) == 1
        adapters.append((O.bf(down.float() * alpha), up))
    assert m.q.lora_A.shape == (64 + 128, D) and m.q.lora_B.shape == (D, 64 + 128)
    x = torch.randn(100, D, generator=g).to(BF16)
    out = torch.empty(100, D, dtype=BF16, device="cuda")
    linear(m.q, x.cuda(), out, Workspace("cuda"))
    ref = O.linear(x, w, b)
    for a_s, up in adapters:                     # the reference's loop: one bf16 add per adapter
        t = O.bf(x.float() @ a_s.float().t())
        ref = O.bf(ref.float() + O.bf(t.float() @ up.float().t()).float())
    one = O.lora_linear(x, w, b, *adapters[0])
    assert err(one, ref)[1] > 1e-2               # the second adapter is not negligible
    assert err(out, ref)[1] < 1e-2


def test_merge_lora_after_fp8_quantisation_refreshes_e4m3_copy():
    """merge_lora on a layer quantize_fp8_ already converted rewrites its e4m3 copy (which
    linear() reads instead of the bf16 weight), including the fused q|k|v e4m3 buffer views."""
    from vstyler.lora import merge_lora
    from vstyler.models import quantize_fp8_, _fused_views
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    quantize_fp8_(vace)
    g = torch.Generator().manual_seed(93)
    D, r = cfg["dim"], 32
    lora = {}
    for n in ("vace_blocks.0.self_attn.k", "vace_blocks.0.ffn.0"):
        lin_out = cfg["ffn_dim"] if n.endswith("ffn.0") else D
        lora[n + ".lora_A.default.weight"] = (0.05 * torch.randn(r, D, generator=g)).to(BF16)
        lora[n + ".lora_B.default.weight"] = (0.05 * torch.randn(lin_out, r, generator=g)).to(BF16)
    assert merge_lora(vace, lora, alpha=1.0) == 2
    blk = vace.vace_blocks[0]
    for lin in (blk.self_attn.k, blk.ffn[0]):
        want = lin.weight.detach().to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(lin.weight_fp8, want)
    assert _fused_views(blk.self_attn) is not None
    fw8 = blk.self_attn._fw8
    assert torch.equal(fw8[D:2 * D], blk.self_attn.k.weight.detach().to(torch.float8_e4m3fn).view(torch.uint8))


def test_denoise_graph_replay_bit_identical_to_eager(tiny):
    """The hipGraph-captured step (captured once, replayed with per-step timestep/dsigma slots)
    gives exactly the eager loop's latents (same kernels, same order)."""
    from vstyler import WanVideoPipeline
    cfg, W, dit, vace = tiny
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    eager = pipe.denoise(lat, cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=4, use_graph=False)
    assert pipe.last_graph is None
    graph = pipe.denoise(lat, cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=4, use_graph=True)
    assert pipe.last_graph is not None
    assert torch.equal(eager, graph)


def test_hotloaded_lora_on_fused_projections_matches_merged():
    """A LoRA hot-loaded on Linears that normally run fused (self-attention q|k|v, cross-attention
    k|v of the VACE blocks) makes those blocks fall back to per-Linear GEMMs with the fused second K
    phase; the forward must match the same LoRA merged into the weights (which keeps the fusion)."""
    from vstyler import model_fn_wan_video
    from vstyler.lora import hotload_lora, merge_lora
    from vstyler.models import _fused_views
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    g = torch.Generator().manual_seed(91)
    D, r = cfg["dim"], 32
    lora = {}
    for n in ("vace_blocks.0.self_attn.q", "vace_blocks.0.self_attn.v", "vace_blocks.1.cross_attn.k"):
        lora[n + ".lora_A.default.weight"] = (0.05 * torch.randn(r, D, generator=g)).to(BF16)
        lora[n + ".lora_B.default.weight"] = (0.05 * torch.randn(D, r, generator=g)).to(BF16)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([700.0]).to(BF16).cuda()
    outs = []
    for mode in ("merge", "hotload"):
        dit, vace = build(cfg, W)
        (merge_lora if mode == "merge" else hotload_lora)(vace, lora, alpha=0.8)
        fused = _fused_views(vace.vace_blocks[0].self_attn) is not None
        assert fused == (mode == "merge")
        outs.append(model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=cp.cuda(),
                                       vace_context=vc.cuda()))
    mx, rl = err(outs[1], outs[0].cpu())
    assert rl < 1e-2, (mx, rl)
