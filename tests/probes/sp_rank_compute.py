"""Per-rank compute of one 14B 832x480x73 CFG step under Ulysses SP=P, measured on ONE GPU: the
product UlyssesGroup with its RCCL collectives replaced by same-size device copies (rank 0's
data stands in for every peer, so the numbers are garbage; the work and the bytes moved per rank
are the real ones).  Bounds the SP speedup the 8-GPU run can reach: t(SP=1) / t(rank, SP=P).
  python tests/probes/sp_rank_compute.py [P ...]
SPC_SIZE=720p: BASELINE C4's 1280x720x121 (latent 31 x 90 x 160, S = 111 600) instead of 832x480x73;
SPC_REPS: timed repetitions (default 3); SPC_GRAPH=1: eager vs hipGraph replay of the per-rank step."""
import os, sys, time
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "video-styler_amd"))
sys.path.insert(0, ROOT)
import torch
from bench import MODELS
from vstyler import model_fn_wan_video
from vstyler import kernels as K
from vstyler.models import VaceWanModel, WanModel, init_random_
from vstyler.usp import UlyssesGroup, _Done


class LocalUlysses(UlyssesGroup):
    def __init__(self, world, overlap=True):
        self.group, self.world_size, self.rank, self.overlap = None, world, 0, overlap

    def _all_to_all(self, recv, send):
        recv.copy_(send)
        return _Done()

    def _all_gather(self, recv, send):
        recv.view(self.world_size, -1).copy_(send.reshape(1, -1).expand(self.world_size, -1))


dev = torch.device("cuda:0")
m = MODELS["14B"]
T, Hl, Wl = (31, 90, 160) if os.environ.get("SPC_SIZE") == "720p" else (19, 60, 104)
REPS = int(os.environ.get("SPC_REPS", "3"))
dit = WanModel(dim=m["dim"], in_dim=16, ffn_dim=m["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256, eps=1e-6,
               patch_size=(1, 2, 2), num_heads=m["num_heads"], num_layers=m["num_layers"], device=dev)
vace = VaceWanModel(vace_layers=m["vace_layers"], dim=m["dim"], num_heads=m["num_heads"], ffn_dim=m["ffn_dim"],
                    device=dev)
init_random_(dit, seed=5)
init_random_(vace, seed=6)
g = torch.Generator().manual_seed(1)
lat = torch.randn(1, 16, T, Hl, Wl, generator=g).to(torch.bfloat16).to(dev)
ctx = (0.1 * torch.randn(2, 512, 4096, generator=g)).to(torch.bfloat16).to(dev)
vc = torch.ones(1, 96, T, Hl, Wl).to(torch.bfloat16).to(dev)
t = torch.tensor([999.0], device=dev).to(torch.bfloat16)
from vstyler.options import HOST_DEFAULTS, host_option, set_host_option
OVL = bool(host_option("sp_overlap"))      # VSTYLER_OPTS=sp_overlap=0 turns it off
AB = os.environ.get("SPC_AB")        # "OPT=a,b": interleaved rounds of a host option's values, one process
if AB:
    var, vals = AB.split("=")
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    sp = LocalUlysses(P, overlap=OVL)
    fn = lambda: model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc,
                                    use_unified_sequence_parallel=True, sp_group=sp)
    res = {v: [] for v in vals.split(",")}
    for rnd in range(4):
        for v in res:
            if var in HOST_DEFAULTS:
                set_host_option(var, v)
            else:                       # a libvstyler option (e.g. piece_queue)
                K.set_option(var, int(v))
            fn(); torch.cuda.synchronize()
            ts = []
            for _ in range(2):
                t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
            res[v].append(1000 * min(ts))
    for v, ms in res.items():
        print(f"SP={P} {var}={v}: per-rank CFG step " + " ".join(f"{x:.1f}" for x in ms) + " ms", flush=True)
    sys.exit(0)
if os.environ.get("SPC_GRAPH") == "1":
    # the per-rank step eager vs hipGraph-replayed (the exchanges are device copies on the caller's
    # stream, so the step is capturable as with vs_sp_* under host option sp_graph=1): the launch cost
    # the SP graph removes, interleaved rounds on one stream
    for a in sys.argv[1:] or ["8"]:
        P = int(a)
        sp = LocalUlysses(P, overlap=OVL) if P > 1 else None
        fn = lambda: model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc,
                                        use_unified_sequence_parallel=sp is not None, sp_group=sp)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn(); fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                fn()
            torch.cuda.synchronize()
            res = {"eager": [], "graph": []}
            for rnd in range(REPS):
                for mode in res:
                    t0 = time.perf_counter()
                    (g.replay() if mode == "graph" else fn())
                    torch.cuda.synchronize()
                    res[mode].append(1000 * (time.perf_counter() - t0))
        print(f"SP={P} overlap={OVL}: per-rank CFG step eager " + " ".join(f"{x:.1f}" for x in res["eager"]) +
              " ms | graph " + " ".join(f"{x:.1f}" for x in res["graph"]) + " ms", flush=True)
        del g
    sys.exit(0)
# args: P = Ulysses over P ranks (both CFG samples per rank); cU = CFG parallelism x Ulysses over u
# ranks (world 2u): a rank's work is its CFG sample's batch-1 forward sharded over u (+ one velocity
# exchange per step, not modelled)
for a in sys.argv[1:] or ["1", "8"]:
    cfgp = a.startswith("c")
    P = int(a[1:] if cfgp else a)
    sp = LocalUlysses(P, overlap=OVL) if P > 1 else None
    c = ctx[0:1] if cfgp else ctx
    fn = lambda: model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=c, vace_context=vc,
                                    use_unified_sequence_parallel=sp is not None, sp_group=sp)
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    label = f"CFG2 x SP={P} (world {2 * P})" if cfgp else f"SP={P} overlap={OVL}"
    print(f"{label} S={T * Hl * Wl // 4}: per-rank CFG step (eager) {1000 * min(ts):.1f} ms", flush=True)
