"""14B-dim block pair, CFG batch 2 at 832x480x73: run the product forward twice (fresh Workspace
buffers NaN-poisoned with VSTYLER_OPTS=ws_poison=1) and compare with each other and the oracle."""
import os, sys
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "video-styler_amd"), os.path.join(ROOT, "tests")]
import torch
from oracle import wan_oracle as O
from test_production_model_gpu import build, gpu_weights
from vstyler import model_fn_wan_video

BF16 = torch.bfloat16
cfg = dict(O.WAN_CONFIGS["14B"], num_layers=1, vace_layers=(0,))
W = gpu_weights(cfg, seed=7)
dit, vace = build(cfg, W)
lat, cp, cn, vc = O.synthetic_inputs(cfg, 73, 480, 832)
lat, vc = lat.cuda(), vc.cuda()
ctx = torch.cat([cp, cn]).cuda()
t = torch.tensor([937.5], device="cuda").to(BF16)
first = os.environ.get("C3_ORDER", "oracle")
outs = []
if first == "product":
    outs.append(model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc).clone())
ref = O.model_fn(W, cfg, torch.cat([lat, lat]), t.expand(2), ctx, torch.cat([vc, vc]))
for _ in range(2):
    outs.append(model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc).clone())
torch.cuda.synchronize()
from vstyler.options import host_option
tag = f"poison={host_option('ws_poison')} order={first}"
for i, o in enumerate(outs):
    d = o.float() - ref.float()
    print(f"[{tag}] run {i}: finite {bool(torch.isfinite(o.float()).all())} rel vs oracle "
          f"{(d.norm() / ref.float().norm()).item():.4g}  equal-to-run0 {torch.equal(o, outs[0])}", flush=True)
