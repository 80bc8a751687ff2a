"""Config 5: the 14B DiT + VACE forward (fp8 block linears, CFG batch 2, 832x480x73) with the
LayerNorms writing fp8_linear's quantised activations directly (models.ln_into) vs bf16 rows + a
separate quantisation pass; interleaved rounds in one process (eager forwards, ms each)."""
import os, sys, time
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "video-styler_amd"))
sys.path.insert(0, ROOT)
import torch
from bench import MODELS
from vstyler import model_fn_wan_video, models
from vstyler.models import VaceWanModel, WanModel, init_random_, quantize_fp8_

dev = torch.device("cuda:0")
m = MODELS["14B"]
T, Hl, Wl = 19, 60, 104
dit = WanModel(dim=m["dim"], in_dim=16, ffn_dim=m["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256, eps=1e-6,
               patch_size=(1, 2, 2), num_heads=m["num_heads"], num_layers=m["num_layers"], device=dev)
vace = VaceWanModel(vace_layers=m["vace_layers"], dim=m["dim"], num_heads=m["num_heads"], ffn_dim=m["ffn_dim"],
                    device=dev)
init_random_(dit, seed=5)
init_random_(vace, seed=6)
quantize_fp8_(dit)
quantize_fp8_(vace)
g = torch.Generator().manual_seed(1)
lat = torch.randn(1, 16, T, Hl, Wl, generator=g).to(torch.bfloat16).to(dev)
ctx = (0.1 * torch.randn(2, 512, 4096, generator=g)).to(torch.bfloat16).to(dev)
vc = torch.ones(1, 96, T, Hl, Wl).to(torch.bfloat16).to(dev)
t = torch.tensor([999.0], device=dev).to(torch.bfloat16)
real = models._fp8_consumer
fn = lambda: model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc)
res = {"fused": [], "separate": []}
for rnd in range(3):
    for name in res:
        models._fp8_consumer = real if name == "fused" else (lambda target: False)
        fn(); torch.cuda.synchronize()
        ts = []
        for _ in range(2):
            t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
        res[name].append(1000 * min(ts))
    print(f"round {rnd}: " + "  ".join(f"{k} {v[-1]:.1f} ms" for k, v in res.items()), flush=True)
