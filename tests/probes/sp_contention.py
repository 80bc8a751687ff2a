"""How the SP=8 per-rank step behaves when the exchanges are kernels on a side stream that compete
for CUs (as RCCL's all-to-all does on a real node), on ONE GPU: the product UlyssesGroup with each
collective replaced by a G-workgroup copy kernel (tests/probes/fakecomm) launched on a side stream
after an event, and waited on by event -- RCCL's async pattern.  Interleaved rounds in one process:
  python tests/probes/sp_contention.py   (env: SPC_G=16,64  SPC_PERSIST=0,1  SPC_QUEUE=1,0 -- the r5 XCD
  tile / item queues of the persistent GEMM and attention grids vs the static per-CU lists)"""
import ctypes, os, sys, time
ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "video-styler_amd"))
sys.path.insert(0, ROOT)
import torch
from bench import MODELS
from vstyler import model_fn_wan_video
from vstyler.models import VaceWanModel, WanModel, init_random_
from vstyler.usp import UlyssesGroup, _Done
from vstyler import kernels as K
from vstyler import _lib
from vstyler.options import HOST_DEFAULTS, set_host_option

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "fakecomm", "libfakecomm.so"))
lib.fake_comm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]


class _Ev:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class FakeCommUlysses(UlyssesGroup):
    def __init__(self, world, overlap=True, nblocks=16):
        self.group, self.world_size, self.rank, self.overlap = None, world, 0, overlap
        self.force_collectives, self.collective_calls = False, 0
        self.nblocks = nblocks
        self.side = torch.cuda.Stream()

    def _all_to_all(self, recv, send):
        if self.nblocks <= 0:
            recv.copy_(send)
            return _Done()
        ev = torch.cuda.Event()
        ev.record()
        self.side.wait_event(ev)
        lib.fake_comm(send.data_ptr(), recv.data_ptr(), send.numel() * send.element_size(), self.nblocks,
                      ctypes.c_void_p(self.side.cuda_stream))
        done = torch.cuda.Event()
        done.record(self.side)
        return _Ev(done)

    def _all_gather(self, recv, send):
        recv.view(self.world_size, -1).copy_(send.reshape(1, -1).expand(self.world_size, -1))


dev = torch.device("cuda:0")
m = MODELS["14B"]
T, Hl, Wl = 19, 60, 104
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
P = 8
Gs = [int(x) for x in os.environ.get("SPC_G", "0,16,64").split(",")]
pers = os.environ.get("SPC_PERSIST", "1,0").split(",")
queues = os.environ.get("SPC_QUEUE", "1").split(",")
ovs = [o == "1" for o in os.environ.get("SPC_OVERLAP", "1,0").split(",")]
ev = os.environ.get("SPC_ENV", "")          # "OPT=a,b": one more interleaved dimension (an option or env var)
evar, evals = ev.split("=") if ev else ("", "-")
cases = [(G, pz, ov, e, qu) for G in Gs for pz in pers for ov in ovs for e in evals.split(",") for qu in queues]
res = {c: [] for c in cases}
for rnd in range(3):
    for c in cases:
        G, pz, ov, e, qu = c
        if evar in _lib.OPTIONS:          # a libvstyler option (e.g. piece_queue)
            K.set_option(evar, int(e))
        elif evar in HOST_DEFAULTS:
            set_host_option(evar, e)
        elif evar:
            os.environ[evar] = e
        K.set_option("attn_persist", 1 if pz == "1" else 0)
        K.set_option("queue", int(qu))
        sp = FakeCommUlysses(P, overlap=ov, nblocks=G)
        fn = lambda: model_fn_wan_video(dit, vace=vace, latents=lat, timestep=t, context=ctx, vace_context=vc,
                                        use_unified_sequence_parallel=True, sp_group=sp)
        fn(); torch.cuda.synchronize()
        ts = []
        for _ in range(2):
            t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
        res[c].append(1000 * min(ts))
    print(f"round {rnd} done", flush=True)
for (G, pz, ov, e, qu), ms in res.items():
    print(f"SP=8 comm-G={G:3d} persist={pz} overlap={int(ov)} queue={qu}" + (f" {evar}={e}" if evar else "") + ": "
          + " ".join(f"{x:.1f}" for x in ms) + " ms", flush=True)
