"""14B-dim 1-block forward, CFG batch 2 at 832x480x73: B=2 vs the oracle under the current env
(run once per GEMM-route variant in separate processes)."""
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
use_vace = os.environ.get("C3_VACE", "1") == "1"
ref = O.model_fn(W, cfg, torch.cat([lat, lat]), t.expand(2), ctx, torch.cat([vc, vc]) if use_vace else None)
both = model_fn_wan_video(dit, vace=vace if use_vace else None, latents=lat, timestep=t, context=ctx, vace_context=vc)
d = both.float() - ref.float()
tag = " ".join(f"{k}={os.environ[k]}" for k in ("VS_GEMM_BACKEND", "VS_LT_SWEPT", "VS_LT_TUNE", "VS_LT_GELU",
                                                  "VSTYLER_FUSE_RES_LN", "VSTYLER_FUSE_FFN_LN", "C3_VACE", "VS_ATTN_NC", "VS_ATTN_NO_SPLIT", "VS_ATTN_NO_PERSIST") if k in os.environ)
print(f"[{tag or 'default'}] B2 vs oracle: rel {(d.norm() / ref.float().norm()).item():.4g} "
      f"(sample0 {(d[0].norm() / ref[0].float().norm()).item():.4g}, sample1 {(d[1].norm() / ref[1].float().norm()).item():.4g})",
      flush=True)
