"""GPU parity of the UniPC sampler (vstyler/unipc.py) against the oracle restatement of
FlowUniPCMultistepScheduler (denoising_enhancing/wan/utils/fm_solvers_unipc.py): the update is a
fixed sequence of fp32 ops, so the trajectories must agree bit for bit."""
import pytest
import torch

from oracle.unipc_oracle import UniPCOracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("steps,shift", [(4, 2.0), (6, 5.0), (1, 2.0)])
def test_unipc_trajectory_bit_exact(steps, shift):
    from vstyler.unipc import FlowUniPCMultistepScheduler
    g = torch.Generator().manual_seed(steps)
    x = torch.randn(2, 16, 3, 8, 12, generator=g)
    w = torch.randn(16, 16, generator=g) * 0.3

    def model(s):  # a deterministic stand-in velocity field
        return torch.einsum("bc...,cd->bd...", s, w) + 0.1 * torch.sin(3 * s)

    ref = UniPCOracle(shift=1.0)
    ref.set_timesteps(steps, shift=shift)
    sched = FlowUniPCMultistepScheduler(shift=1.0)
    sched.set_timesteps(steps, shift=shift)
    assert torch.equal(sched.timesteps, ref.timesteps) and torch.equal(sched.sigmas, ref.sigmas)
    xr, xg = x.clone(), x.cuda()
    for t in ref.timesteps:
        v = model(xr)
        xr = ref.step(v, t, xr)
        xg = sched.step(v.cuda(), t, xg)[0]
        assert torch.equal(xg.cpu(), xr), (t, (xg.cpu() - xr).abs().max().item())


def test_slg_skips_uncond_block_only():
    """model_fn(slg_blocks) == the oracle with those blocks skipped on sample 1; sample 0 untouched."""
    from oracle import wan_oracle as O
    from test_model_gpu import build
    from vstyler import model_fn_wan_video
    from gpu_util import err
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([700.0]).to(torch.bfloat16)
    ctx = torch.cat([cp, cn]).cuda()
    full = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t.cuda(), context=ctx, vace_context=vc.cuda())
    slg = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t.cuda(), context=ctx,
                             vace_context=vc.cuda(), slg_blocks=(2,))
    assert torch.equal(full[0:1], slg[0:1])
    ref = O.model_fn(W, cfg, lat, t, cn, vc, skip_blocks=(2,))
    mx, rl = err(slg[1:2], ref)
    assert rl < 2e-2 and mx < 0.1, (mx, rl)
    assert not torch.equal(full[1:2], slg[1:2])


def test_config5_sampler_tiny_vs_oracle():
    """fp8 block linears + UniPC 4 steps + CFG 1.2 + SLG, tiny model, vs the oracle chain within
    1.5x the oracle's own fp32-vs-fp64 floor."""
    from oracle import wan_oracle as O
    from test_model_gpu import build
    from gpu_util import err
    from vstyler import WanVideoPipeline
    from vstyler.models import quantize_fp8_
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    quantize_fp8_(dit)
    quantize_fp8_(vace)
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    kw = dict(vace_scale=0.975, cfg_scale=1.2, num_inference_steps=4, sigma_shift=2.0, slg_blocks=(2,))
    got = pipe.denoise_unipc(lat, cp.cuda(), cn.cuda(), vc.cuda(), **kw)
    old, olda = O.FP8_BLOCK_LINEARS, O.ACC_DTYPE
    try:
        O.FP8_BLOCK_LINEARS = True
        ref = O.denoise_unipc(W, cfg, lat, cp, cn, vc, **kw)
        O.ACC_DTYPE = torch.float64
        ref64 = O.denoise_unipc(W, cfg, lat, cp, cn, vc, **kw)
    finally:
        O.FP8_BLOCK_LINEARS, O.ACC_DTYPE = old, olda
    fmx, frl = err(ref64, ref)
    mx, rl = err(got, ref)
    print(f"config-5 tiny sampler: max-abs {mx:.4g} rel-L2 {rl:.4g} (floor {fmx:.4g} / {frl:.4g})")
    assert rl <= 1.5 * frl + 2e-3 and mx <= 1.5 * fmx + 2e-2
