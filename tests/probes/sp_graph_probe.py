"""Probe (diagnostic, one GPU): the Ulysses SP denoising step captured into a hipGraph with the
RCCL collectives inside, at world size 1 over 'nccl' with force_collectives -- which stage stalls?
Prints a line before and after every eager run, capture and replay; run under `timeout`.
  python tests/probes/sp_graph_probe.py [torch|native] [steps]"""
import os, sys, time
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
for p in (ROOT, os.path.join(ROOT, "video-styler_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29611"), RANK="0",
                  WORLD_SIZE="1", LOCAL_RANK="0")
import torch
from oracle import wan_oracle as O
from vstyler import WanVideoPipeline
from vstyler.usp import UlyssesGroup, init_distributed
from test_model_gpu import build

t0 = time.time()


def say(msg):
    print(f"[{time.time() - t0:7.1f} s] {msg}", flush=True)


init_distributed()
say(f"process group up: {torch.distributed.get_backend()}")
comm = sys.argv[1] if len(sys.argv) > 1 else "torch"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg = O.WAN_CONFIGS["tiny"]
W = O.random_weights(cfg, seed=5)
dit, vace = build(cfg, W, "cuda:0")
lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
from vstyler.options import set_host_option
set_host_option("sp_graph", 1)
for graph in (False, True):
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = dit, vace
    sp = UlyssesGroup(force_collectives=True, comm=comm)
    pipe.use_unified_sequence_parallel, pipe.sp_group = True, sp
    say(f"comm={comm} graph={graph}: denoise {steps} steps ...")
    out = pipe.denoise(lat.cuda(), cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=steps, use_graph=graph)
    torch.cuda.synchronize()
    say(f"comm={comm} graph={graph}: done, captured={pipe.last_graph is not None}, "
        f"collectives={sp.collective_calls}, sum={out.float().sum().item():.6f}")
    del pipe
    if getattr(sp, "native", None) is not None:
        sp.native.close()
torch.distributed.destroy_process_group()
say("clean exit")
