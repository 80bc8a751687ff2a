"""Localise the 14B-dim block-pair mismatch: product B=2 vs two B=1 calls, and B=1 vs the oracle
(run on the GPU), at a short (5-frame) and the full 73-frame 832x480 latent."""
import os, sys
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd"), os.path.join(ROOT, "tests")]
import torch
from oracle import wan_oracle as O
from test_production_model_gpu import build, gpu_weights
from vstyler import model_fn_wan_video

BF16 = torch.bfloat16
for dims, frames in (("14B", 5), ("1.3B", 5), ("14B", 73)):
    cfg = dict(O.WAN_CONFIGS[dims], num_layers=1, vace_layers=(0,))
    W = gpu_weights(cfg, seed=7)
    dit, vace = build(cfg, W)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, frames, 480, 832)
    lat, vc = lat.cuda(), vc.cuda()
    ctx = torch.cat([cp, cn]).cuda()
    t = torch.tensor([937.5], device="cuda").to(BF16)
    for use_vace in (True, False):
        v = vace if use_vace else None
        both = model_fn_wan_video(dit, vace=v, latents=lat, timestep=t, context=ctx, vace_context=vc)
        p = model_fn_wan_video(dit, vace=v, latents=lat, timestep=t, context=ctx[0:1], vace_context=vc)
        ref = O.model_fn(W if use_vace else {k: x for k, x in W.items()}, cfg, lat, t, ctx[0:1],
                         vc if use_vace else None)
        d = (p.float() - ref.float())
        print(f"{dims} frames {frames} vace {use_vace}: B2[0]==B1 {torch.equal(both[0:1], p)}; "
              f"B1 vs oracle max-abs {d.abs().max().item():.4g} rel {(d.norm() / ref.float().norm()).item():.4g}; "
              f"B2[0] vs oracle rel {((both[0:1].float() - ref.float()).norm() / ref.float().norm()).item():.4g}",
              flush=True)
    del dit, vace, W
    torch.cuda.empty_cache()
