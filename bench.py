"""Headline benchmark: denoising steps/s of Wan2.1-VACE-14B at 832x480x73 on MI355X.

One step = the reference's CFG denoising step (wan_video_new.py:518-542): DiT(40 blocks) + VACE
(8 blocks) forward for the positive AND negative prompt (run as one batch-2 forward), CFG combine
and the Euler update.  Synthetic data: random-init weights (N(0,0.02), seed 5), seeded latents /
contexts / VACE context of the real shapes (no checkpoints or datasets are reachable offline).

  python bench.py [--gpus N --steps K --warmup W]

N > 1: one process per GPU, Ulysses SP over all N ranks over RCCL (VSTYLER_OPTS=cfg_parallel=1 selects
CFG parallelism; sp_comm=native,sp_graph=1 captures the collectives into the step's hipGraph).  Under torchrun (WORLD_SIZE set) WORLD_SIZE must equal N; without a launcher this
process spawns the N ranks itself (launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR
127.0.0.1 / MASTER_PORT per child, rank 0 prints the line, exit code = the worst child's) and refuses
when fewer than N GPUs are visible.  The line carries `rccl_world` and every rank's device and
ms/step; `n_gpus` is the process group's size.

Prints one JSON line with `roofline` (self-attention kernel, HIP-event timed inside the timed
region) and, on rank 0 at N=1, `cpu_baseline` (the CPU oracle on a bounded token sample).
"""
import argparse
import json
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-styler_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

MODELS = {
    "14B": dict(dim=5120, ffn_dim=13824, num_heads=40, num_layers=40, vace_layers=tuple(range(0, 40, 5))),
    "1.3B": dict(dim=1536, ffn_dim=8960, num_heads=12, num_layers=30, vace_layers=tuple(range(0, 30, 2))),
}
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)


def step_flops(m, S, L=512, B=2):
    """Algorithmic FLOPs of one CFG step (SURVEY.md §8d / BASELINE.md §2)."""
    D, F, nm, nv = m["dim"], m["ffn_dim"], m["num_layers"], len(m["vace_layers"])
    blk = 12 * S * D * D + 4 * S * D * F + 4 * S * S * D + 4 * L * D * D + 4 * S * L * D
    fwd = (nm + nv) * blk + (nv + 1) * 2 * S * D * D + 2 * S * D * (64 + 384 + 64) + 2 * L * D * (4096 + D)
    return B * fwd


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(m, S, rows=2048):
    """Oracle (PyTorch-CPU restatement, oracle/wan_oracle.py) on a bounded sample of the step: one
    main DiT block and one VACE block (DiT block + after_proj, wan_video_vace.py:13-24) for `rows`
    query tokens each -- their projections, norms, RoPE, attention against the full S-token K/V,
    cross-attention, FFN -- extrapolated as (N_main t_main + N_vace t_vace) x S/rows x 2 (CFG).
    Threads: OMP_NUM_THREADS when set (the GPU box's CPU share), else the CPUs this process may run
    on (os.sched_getaffinity); the CPU model and os.cpu_count() are reported beside it."""
    from oracle import wan_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    D, F, H = m["dim"], m["ffn_dim"], m["num_heads"]
    g = torch.Generator().manual_seed(0)
    bf = torch.bfloat16

    def w(*s):
        return (0.02 * torch.randn(*s, generator=g)).to(bf)
    Wb = {}
    for a in ("self_attn.", "cross_attn."):
        for l in "qkvo":
            Wb[a + l + ".weight"], Wb[a + l + ".bias"] = w(D, D), w(D)
        Wb[a + "norm_q.weight"], Wb[a + "norm_k.weight"] = 1 + w(D), 1 + w(D)
    Wb["norm3.weight"], Wb["norm3.bias"] = 1 + w(D), w(D)
    Wb["ffn.0.weight"], Wb["ffn.0.bias"], Wb["ffn.2.weight"], Wb["ffn.2.bias"] = w(F, D), w(F), w(D, F), w(D)
    Wb["modulation"] = w(1, 6, D)
    Wb["after_proj.weight"], Wb["after_proj.bias"] = w(D, D), w(D)
    kfull = torch.randn(1, S, D, generator=g).to(bf)
    vfull = torch.randn(1, S, D, generator=g).to(bf)
    ctx = torch.randn(1, 512, D, generator=g).to(bf)
    t_mod = w(1, 6, D)

    def block(n, vace):
        x = torch.randn(1, n, D, generator=g).to(bf)
        freqs = O.rope_freqs(1, n // 64, 64)      # a (1, n/64, 64) token grid: RoPE tables hold 1024 positions
        t0 = time.perf_counter()
        mod = O.bf(Wb["modulation"].float() + t_mod.float())
        sh, sc, ga, sh2, sc2, ga2 = mod.chunk(6, dim=1)
        h = O.modulate(O.layer_norm(x), sh, sc)
        q = O.rope_apply(O.rms_norm(O.linear(h, Wb["self_attn.q.weight"], Wb["self_attn.q.bias"]),
                                    Wb["self_attn.norm_q.weight"]), freqs, H)
        k = O.rope_apply(O.rms_norm(O.linear(h, Wb["self_attn.k.weight"], Wb["self_attn.k.bias"]),
                                    Wb["self_attn.norm_k.weight"]), freqs, H)
        v = O.linear(h, Wb["self_attn.v.weight"], Wb["self_attn.v.bias"])
        kk = torch.cat([k, kfull[:, n:]], 1)
        vv = torch.cat([v, vfull[:, n:]], 1)
        o = O.attention(q, kk, vv, H)
        y = O.gate_residual(x, ga, O.linear(o, Wb["self_attn.o.weight"], Wb["self_attn.o.bias"]))
        y = O.add(y, O.cross_attention(O.layer_norm(y, 1e-6, Wb["norm3.weight"], Wb["norm3.bias"]), ctx, Wb,
                                       "cross_attn.", H))
        f = O.linear(O.gelu_tanh(O.linear(O.modulate(O.layer_norm(y), sh2, sc2), Wb["ffn.0.weight"],
                                          Wb["ffn.0.bias"])), Wb["ffn.2.weight"], Wb["ffn.2.bias"])
        y = O.gate_residual(y, ga2, f)
        if vace:
            O.linear(y, Wb["after_proj.weight"], Wb["after_proj.bias"])
        return time.perf_counter() - t0

    block(rows, True)                   # warm-up at full size (allocator, thread pool, caches)
    t_main = block(rows, False)
    t_vace = block(rows, True)
    nm, nv = m["num_layers"], len(m["vace_layers"])
    sec_per_step = (nm * t_main + nv * t_vace) * (S / rows) * 2
    return {"value": 1.0 / sec_per_step, "unit": "steps/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"oracle main DiT block ({t_main:.2f} s) and VACE block ({t_vace:.2f} s), each on {rows} of "
                      f"{S} query tokens ({100.0 * rows / S:.1f} %) against the full {S}-token K/V, extrapolated "
                      f"({nm} x main + {nv} x VACE) x {S}/{rows} tokens x 2 CFG = {sec_per_step:.0f} s/step"}


def pmc_traffic(path=os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r6", "pmc_attn_w4_r6b",
                                   "summary.txt")):
    """HBM bytes per self-attention launch from the committed rocprofv3 --pmc measurement of the same
    kernel at the same shape (scripts/pmc.sh attn: FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE,
    KB -> bytes, median over the profiled dispatches), or None."""
    try:
        txt = open(path).read()
        rd = float(re.search(r"HBM read\s+~\s+([0-9.]+) GB/dispatch", txt).group(1))
        wr = float(re.search(r"HBM write\s+~\s+([0-9.]+) GB/dispatch", txt).group(1))
        return int(round((rd + wr) * 1e9))
    except (OSError, AttributeError):
        return None


def e2e_components(dev, frames, height, width, step_s, steps=50):
    """End-to-end sec/video of the Ditto call (BASELINE metric 2): 2 prompts through UMT5-XXL,
    WanVideoUnit_VACE (2 tiled VAE encodes + mask latents), `steps` denoising steps at the measured
    step time, tiled VAE decode + uint8 conversion.  Random-init weights, synthetic frames; each
    component timed once after one warm-up call."""
    from vstyler.t5 import WanPrompter, WanTextEncoder
    from vstyler.vae import WanVideoVAE, vace_context, vae_output_to_u8

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, out

    te = WanTextEncoder(device=dev).init_random_(8)
    pr = WanPrompter()
    pr.fetch_models(te)
    g = torch.Generator(device=dev).manual_seed(2)
    ids = torch.randint(1, te.vocab, (1, 512), generator=g, device=dev)
    mask = torch.zeros(1, 512, dtype=torch.long, device=dev)
    mask[0, :48] = 1
    ids[0, 48:] = 0
    t5_s, _ = timed(lambda: (pr.encode_ids(ids, mask), pr.encode_ids(ids, mask)))
    del te, pr
    torch.cuda.empty_cache()
    vae = WanVideoVAE(device=dev).init_random_(6)
    video = torch.randint(0, 256, (frames, height, width, 3), generator=g, device=dev, dtype=torch.uint8)
    enc_s, vc = timed(lambda: vace_context(vae, video, None, tiled=True, tile_size=(30, 52), tile_stride=(15, 26)))
    lat = torch.randn(vc.shape[0], 16, *vc.shape[2:], generator=g, device=dev).to(torch.bfloat16)
    dec_s, _ = timed(lambda: vae_output_to_u8(vae.decode(lat, dev, tiled=True, tile_size=(30, 52),
                                                           tile_stride=(15, 26))[0]))
    del vae, vc
    torch.cuda.empty_cache()
    total = t5_s + enc_s + steps * step_s + dec_s
    return {"sec_per_video": round(total, 2), "unit": "s/video", "t5_2_prompts_s": round(t5_s, 4),
            "vace_2_vae_encodes_s": round(enc_s, 3), "denoise_s": round(steps * step_s, 2), "steps": steps,
            "vae_decode_u8_s": round(dec_s, 3),
            "note": "2 prompts x UMT5-XXL (512 tokens) + VACE unit (2 tiled encodes) + 50 x measured step + "
                    "tiled decode + uint8; random-init weights, synthetic frames"}


def e2e_measured(dev, dit, vace, ctx, frames, height, width, t5_s=None, steps=50):
    """One real WanVideoPipeline.__call__ (wan_video_new.py:416-560, as inference/infer_ditto.py:20-59
    calls it), timed from the call to the uint8 frames on the device: the VACE unit (2 tiled VAE
    encodes of a synthetic 832x480x73 control video + mask latents), the noise on the CPU generator,
    `steps` CFG-5 Euler steps (step 0 eager, hipGraph capture, replays), the tiled decode and the uint8
    conversion -- host glue included.  Prompt embeddings are passed (no tokenizer files offline); the
    two UMT5-XXL encodes are the separately timed `t5_s`.  Random-init weights."""
    from vstyler.pipeline import WanVideoPipeline
    from vstyler.vae import WanVideoVAE
    pipe = WanVideoPipeline(device=dev)
    pipe.dit, pipe.vace = dit, vace
    pipe.vae = WanVideoVAE(device=dev).init_random_(6)
    g = torch.Generator(device=dev).manual_seed(3)
    video = torch.randint(0, 256, (frames, height, width, 3), generator=g, device=dev, dtype=torch.uint8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = pipe(prompt_emb=ctx[0:1], negative_prompt_emb=ctx[1:2], vace_video=video, seed=0, height=height,
               width=width, num_frames=frames, num_inference_steps=steps, cfg_scale=5.0, output_type="u8")
    torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    shape = list(out.shape)
    del pipe, out, video
    torch.cuda.empty_cache()
    res = {"measured_call_s": round(sec, 2), "measured_output": shape, "measured_steps": steps,
           "measured_note": "one WanVideoPipeline.__call__(prompt_emb=, negative_prompt_emb=, vace_video=<73 "
                            "frames u8>, num_inference_steps=50, cfg_scale=5, output_type='u8'): VACE encodes "
                            "+ 50 steps + decode + uint8, host glue included"}
    if t5_s is not None:
        res["sec_per_video_measured"] = round(sec + t5_s, 2)
    return res


def _parallelism(sp, world):
    """'single', 'sp<N>' (Ulysses over N ranks) or 'cfg2' / 'cfg2_sp<u>' (CFG parallelism: one CFG
    sample per half of the ranks, Ulysses over the u ranks of a half)."""
    if world == 1 or sp is None:
        return "single"
    from vstyler.usp import CfgParallel
    if isinstance(sp, CfgParallel):
        return "cfg2" if sp.ulysses is None else f"cfg2_sp{sp.ulysses.world_size}"
    return f"sp{world}"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus():
    """GPUs this process could bind, without initialising HIP (torch.cuda.device_count() does not
    create a context on this image; the launcher must never touch the GPU before its children)."""
    return torch.cuda.device_count()


def rank_env(base, rank, world, port):
    """The environment rank `rank` of `world` gets: torchrun's variables, one GPU per rank
    (LOCAL_RANK == RANK on one node), rendezvous on 127.0.0.1."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def launch_ranks(n, argv, script=None, gpus=None, env=None, timeout=None):
    """`bench.py --gpus N` without an external launcher: N fresh child processes of `script` (this
    file), one per GPU, each with rank_env; the parent never touches the GPU (the reference's USP is
    one process per GPU, examples/wanvideo/README.md:220, wan_video_new.py:313-338).  Rank 0 prints
    the JSON line; the return value is 0 or the exit code of the first child to fail (every child
    still running then is terminated).  Fails fast (rc 2, no child started) when fewer than N GPUs are
    visible."""
    import subprocess
    gpus = visible_gpus() if gpus is None else gpus
    if gpus < n:
        print(f"[bench] --gpus {n} needs {n} visible GPUs, this node has {gpus}: refusing to time "
              f"fewer GPUs than asked", file=sys.stderr, flush=True)
        return 2
    script = script or os.path.abspath(__file__)
    port = _free_port()
    base = dict(os.environ if env is None else env)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=rank_env(base, r, n, port))
             for r in range(n)]

    def stop_children(signum, frame):       # a launcher killed from outside takes its ranks with it
        for p in procs:
            if p.poll() is None:
                p.terminate()
        sys.exit(128 + signum)
    import signal
    old_handlers = {sig: signal.signal(sig, stop_children) for sig in (signal.SIGTERM, signal.SIGINT)}
    rcs = [None] * n
    first_bad = None
    t0 = time.time()
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and first_bad is None:
                    first_bad = rcs[r]
        late = timeout is not None and time.time() - t0 > timeout
        if first_bad is not None or late:
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                try:
                    rcs[r] = p.wait(30) if rcs[r] is None else rcs[r]
                except subprocess.TimeoutExpired:
                    p.kill()
                    rcs[r] = p.wait()
            if first_bad is None:
                for sig, h in old_handlers.items():
                    signal.signal(sig, h)
                print(f"[bench] ranks still running after {timeout} s: terminated", file=sys.stderr, flush=True)
                return 124
            break
        time.sleep(0.2)
    for sig, h in old_handlers.items():
        signal.signal(sig, h)
    # the first child to fail is the cause (the ranks terminated after it report SIGTERM)
    return first_bad if first_bad is not None else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="14B", choices=list(MODELS))
    ap.add_argument("--frames", type=int, default=73)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--width", type=int, default=832)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=2048)
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay")
    ap.add_argument("--progress", action="store_true", help="sync + stderr line after every timed step")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end sec/video components")
    ap.add_argument("--no-e2e-call", action="store_true",
                    help="skip the measured 50-step WanVideoPipeline.__call__ (keep the composed e2e breakdown)")
    ap.add_argument("--config", default="bf16", choices=("bf16", "fp8"),
                    help="bf16: BASELINE config (50-step Euler, CFG 5); fp8: config 5 (fp8 block linears, "
                         "UniPC, CFG 1.2, shift 2, SLG block 2, VACE strength 0.975)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: this process only spawns the ranks (it never touches the GPU)
        rc = launch_ranks(args.gpus, sys.argv[1:])
        sys.exit(rc if rc >= 0 else 128 - rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if world > 1:
        import torch.distributed as dist
        from vstyler.usp import init_distributed, get_default_group
        local = init_distributed()
        dev = torch.device(f"cuda:{local}")
        sp = get_default_group()
        world = dist.get_world_size()
    else:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        sp = None

    from vstyler import model_fn_wan_video
    from vstyler import kernels as K
    from vstyler.flow_match import FlowMatchScheduler
    from vstyler.pipeline import DenoiseStepper
    from vstyler.models import TIMER, VaceWanModel, WanModel, init_random_
    from vstyler.options import host_option

    m = MODELS[args.model]
    T = (args.frames - 1) // 4 + 1
    Hl, Wl = args.height // 8, args.width // 8
    S = T * (Hl // 2) * (Wl // 2)
    dit = WanModel(dim=m["dim"], in_dim=16, ffn_dim=m["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256, eps=1e-6,
                   patch_size=(1, 2, 2), num_heads=m["num_heads"], num_layers=m["num_layers"], device=dev)
    vace = VaceWanModel(vace_layers=m["vace_layers"], dim=m["dim"], num_heads=m["num_heads"], ffn_dim=m["ffn_dim"],
                        device=dev)
    init_random_(dit, seed=5)
    init_random_(vace, seed=6)

    g = torch.Generator().manual_seed(1)
    latents = torch.randn(1, 16, T, Hl, Wl, generator=g).to(torch.bfloat16).to(dev)
    ctx = (0.1 * torch.randn(2, 512, 4096, generator=g))
    ctx[0, 32:] = 0
    ctx[1, 96:] = 0
    ctx = ctx.to(torch.bfloat16).to(dev)
    vc = torch.ones(1, 96, T, Hl, Wl)
    vc[:, :32] = torch.randn(1, 32, T, Hl, Wl, generator=g)
    vc = vc.to(torch.bfloat16).to(dev)
    use_graph = False
    if args.config == "fp8":
        # config 5: the sampler is stateful (UniPC multistep), so the W warmup steps run as their own
        # short sampler and the K timed steps as one K-step sampler (CFG 1.2, shift 2, SLG block 2
        # for step fractions in [0.2, 0.7], VACE strength 0.975), eager launches
        from vstyler.models import quantize_fp8_
        from vstyler.pipeline import WanVideoPipeline
        quantize_fp8_(dit)
        quantize_fp8_(vace)
        pipe = WanVideoPipeline(device=dev)
        pipe.dit, pipe.vace = dit, vace
        pipe.use_unified_sequence_parallel, pipe.sp_group = sp is not None, sp
        kw = dict(vace_scale=0.975, cfg_scale=1.2, sigma_shift=2.0, slg_blocks=(2,))
        if args.warmup > 0:
            pipe.denoise_unipc(latents, ctx[0:1], ctx[1:2], vc, num_inference_steps=args.warmup, **kw)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        TIMER.reset()
        TIMER.enabled = True
        t0 = time.perf_counter()
        pipe.denoise_unipc(latents, ctx[0:1], ctx[1:2], vc, num_inference_steps=args.steps, **kw)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    else:
        sched = FlowMatchScheduler(shift=5, sigma_min=0.0, extra_one_step=True)
        n_total = args.warmup + args.steps
        sched.set_timesteps(max(n_total, 2), shift=5.0)
        ts = sched.timesteps.to(torch.bfloat16).to(dev)
        ds = torch.tensor([sched.delta(i) for i in range(len(sched.timesteps))], dtype=torch.float32, device=dev)

        def step_fn(t_buf, d_buf):
            v = model_fn_wan_video(dit, vace=vace, latents=latents, timestep=t_buf, context=ctx, vace_context=vc,
                                   use_unified_sequence_parallel=sp is not None, sp_group=sp)
            K.cfg_euler_dev(v[0:1], v[1:2], latents, 5.0, d_buf)

        # the product's step runner: step 0 eager, then one hipGraph capture replayed per step (under
        # Ulysses SP with the RCCL collectives inside the graph).  Capture happens inside the warmup.
        from vstyler.pipeline import sp_graph_ok
        use_graph = not args.no_graph and args.warmup >= 1 and (world == 1 or sp_graph_ok(sp))
        from vstyler.usp import plan_native_comms
        stepper = DenoiseStepper(step_fn, ts, ds, use_graph=use_graph, plan=sp,
                                 comms=plan_native_comms(sp) if use_graph and sp is not None else ())
        for i in range(args.warmup):
            stepper(i)
            torch.cuda.synchronize()
            print(f"[bench] warmup step {i} done", file=sys.stderr, flush=True)
        use_graph = use_graph and stepper.graph is not None     # a failed capture falls back to eager
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        TIMER.reset()
        TIMER.enabled = not use_graph     # eager: attention events inside the timed steps
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.warmup, n_total):
            stepper(i)
            if args.progress:
                torch.cuda.synchronize()
                print(f"[bench] step {i} done", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if use_graph:
            # ROCm refuses event nodes inside a graph: time the attention launches on one instrumented
            # eager step of the same workload right after the timed replays
            TIMER.enabled = True
            step_fn(stepper.t_buf, stepper.d_buf)
            torch.cuda.synchronize()
    TIMER.enabled = False
    attn_ms, attn_n = TIMER.mean_ms("self_attn")
    attn_tf = TIMER.tflops("self_attn")       # summed launch FLOPs / summed launch time
    ranks_info = None
    if world > 1:
        # every rank's own ms/step and device, so the record shows RCCL formed `world` ranks on
        # `world` distinct GPUs; the step time is the slowest rank's
        props = torch.cuda.get_device_properties(dev)
        mine = torch.tensor([elapsed, float(dev.index), float(getattr(props, "pci_bus_id", -1)),
                             float(getattr(props, "pci_device_id", -1))], dtype=torch.float64, device=dev)
        every = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        ranks_info = [{"rank": r, "device": int(e[1]), "pci_bus": int(e[2]), "pci_device": int(e[3]),
                       "ms_per_step": round(1000 * float(e[0]) / args.steps, 2)} for r, e in enumerate(every)]
        elapsed = max(float(e[0]) for e in every)

    default_shape = (args.model, args.width, args.height, args.frames) == ("14B", 832, 480, 73)
    ms_per_step = 1000 * elapsed / args.steps
    value = args.steps / elapsed
    fl_step = step_flops(m, S)
    # self-attention: 4*S_q*S_kv*d per head and sample, recorded per launch (vstyler.models.attn_flops):
    # one launch per block holds both CFG samples and all heads at SP=1; under Ulysses SP a rank's
    # launch holds H/p heads, one sample per launch with the micro-batch overlap
    achieved = attn_tf
    attn_flops = achieved * 1e12 * attn_ms / 1000
    out = {
        "metric": f"denoising steps/sec, Wan2.1-VACE-{args.model} {args.width}x{args.height}x{args.frames}"
                  + (" [config 5: fp8 e4m3 block linears, UniPC, CFG 1.2, SLG]" if args.config == "fp8" else ""),
        "value": round(value, 5), "unit": "steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None,
        "dtype": "fp8_e4m3 (block linears) + bf16 (attention, norms)" if args.config == "fp8" else "bf16",
        "data": "synthetic (random-init weights, seeded latents/contexts/VACE context)",
        "config": {"workload": f"Wan2.1-VACE-{args.model} {args.width}x{args.height}x{args.frames}: "
                               f"{m['num_layers']} DiT + {len(m['vace_layers'])} VACE blocks, "
                               + ("CFG 1.2 as one batch-2 forward + UniPC (config 5)" if args.config == "fp8"
                                  else "CFG 5.0 as one batch-2 forward + Euler"),
                   "model": f"Wan2.1-VACE-{args.model}", "global_batch": 1, "seq_len": S,
                   "latent_shape": [1, 16, T, Hl, Wl], "parallelism": _parallelism(sp, world),
                   "lora": "merged (zero runtime cost, as the reference's GeneralLoRALoader)",
                   "cfg_shared_prefix": bool(host_option("cfg_prefix")),
                   "step_exec": "hipGraph replay" if use_graph else "eager launches",
                   "sampler": ("UniPC bh2 order 2, cfg 1.2, shift 2.0, SLG block 2 @ 0.2-0.7, VACE 0.975"
                               if args.config == "fp8" else "flow-match Euler, cfg 5.0, shift 5.0")},
        "rccl_world": dist.get_world_size() if world > 1 else 1,
        "ranks": ranks_info,
        "model_tflops_per_step": round(fl_step / 1e12, 1),
        "mfu_bf16": round(fl_step * value / world / 1e12 / PEAK_BF16_TFLOPS, 4),
        "roofline": {"kernel": "attn_fwd_w4 (self-attention)", "bound": "mfma",
                     "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                     # the committed PMC measurement is of the default workload (14B 832x480x73)
                     "traffic": pmc_traffic() if world == 1 and default_shape else None,
                     "traffic_source": "rocprofv3 --pmc FETCH_SIZE*2+WRITE_SIZE per launch, profiles/r6/pmc_attn_w4_r6b "
                                       "(same kernel, same shape; algorithmic Q+K+V+O = 2.43e9 B)",
                     "avg_launch_ms": round(attn_ms, 3), "launches": attn_n,
                     "timing": "HIP events on the launch stream, " + ("one instrumented eager step after the "
                               "timed hipGraph replays" if use_graph else "every launch of the timed steps"),
                     "flops_per_launch": round(attn_flops, -6)},
    }
    if world == 1 and not args.no_e2e and args.config == "bf16":
        out["e2e"] = e2e_components(dev, args.frames, args.height, args.width, elapsed / args.steps)
        if not args.no_e2e_call:
            del stepper
            out["e2e"].update(e2e_measured(dev, dit, vace, ctx, args.frames, args.height, args.width,
                                           t5_s=out["e2e"]["t5_2_prompts_s"]))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(m, S, rows=args.cpu_rows)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
