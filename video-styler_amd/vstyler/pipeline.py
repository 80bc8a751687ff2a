"""WanVideoPipeline / model_fn_wan_video with the reference call surface
(diffsynth/pipelines/wan_video_new.py:32-560, 1260-1468), running on libvstyler kernels.

Differences from the reference that are performance-only (same per-sample arithmetic):
  * CFG runs as one batch-2 forward (posi, nega) instead of two batch-1 forwards; the per-batch
    head modulation (mod + t[b]) equals the reference's batch-1 broadcast (wan_video_dit.py:267);
  * sigma table on the host, Euler+CFG fused into one kernel (no per-step host sync);
  * Ulysses SP shards the VACE branch too (the reference runs VACE unsharded).
"""
import os
from dataclasses import dataclass
from typing import Optional, Union

import torch

from . import kernels as K
from .flow_match import FlowMatchScheduler
from .models import RunCtx, Workspace, WanModel, VaceWanModel
from .options import host_option

BF16 = torch.bfloat16

_WS = {}


def _workspace(device):
    key = str(torch.device(device))
    if key not in _WS:
        _WS[key] = Workspace(device)
    return _WS[key]


_UNSUPPORTED = ("clip_feature", "y", "reference_latents", "audio_embeds", "motion_latents", "s2v_pose_latents",
                "motion_bucket_id", "pose_latents", "face_pixel_values", "control_camera_latents_input",
                "sliding_window_size")


def model_fn_wan_video(dit: WanModel, motion_controller=None, vace: VaceWanModel = None, animate_adapter=None,
                       latents: torch.Tensor = None, timestep: torch.Tensor = None, context: torch.Tensor = None,
                       vace_context=None, vace_scale=1.0, use_unified_sequence_parallel: bool = False,
                       sp_group=None, slg_blocks=(), tea_cache=None, cfg_sample=0, **kwargs):
    """One DiT(+VACE) forward (wan_video_new.py:1338-1468) -> [B,16,T,H,W] bf16 velocity.

    slg_blocks: skip-layer guidance (config 5, ComfyUI WanVideoSLG): the listed main blocks are
    skipped for CFG sample 1 (the unconditional pass), run for sample 0 only.  cfg_sample: which
    CFG sample a batch-1 forward computes (1: it skips the slg_blocks) -- set by the CFG-parallel
    split below.

    `context` is [B, L, text_dim]; latents/timestep/vace_context with batch 1 are broadcast to B
    (the cfg_merge convention of wan_video_new.py:1361-1364).

    sp_group may be a vstyler.usp.CfgParallel: a batch-2 (CFG) forward then runs as this rank's
    sample only (batch 1, Ulysses over its half of the ranks) and the two samples' outputs are
    all-gathered across the halves -- the same [2,16,T,H,W] as the batched forward."""
    for name in _UNSUPPORTED:
        if kwargs.get(name) is not None:
            raise NotImplementedError(f"model_fn_wan_video: '{name}' is outside the Ditto hot path")
    if use_unified_sequence_parallel:
        from .usp import CfgParallel, get_default_group
        plan = sp_group if sp_group is not None else get_default_group()
        if isinstance(plan, CfgParallel):
            if context.shape[0] != 2 or tea_cache is not None:
                sp_group = plan.full        # no CFG pair to split (or a TeaCache step): Ulysses over all
            else:
                c = plan.cfg_rank

                def mine(tn):
                    return tn[c:c + 1] if tn is not None and tn.dim() > 0 and tn.shape[0] == 2 else tn
                ts = timestep.reshape(-1)
                local = model_fn_wan_video(dit, motion_controller, vace, animate_adapter, latents=mine(latents),
                                           timestep=mine(ts), context=context[c:c + 1],
                                           vace_context=mine(vace_context), vace_scale=vace_scale,
                                           use_unified_sequence_parallel=plan.ulysses is not None,
                                           sp_group=plan.ulysses, slg_blocks=slg_blocks, cfg_sample=c, **kwargs)
                out = torch.empty((2,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
                plan.gather_cfg(out, local)
                return out
    device = latents.device
    ws = _workspace(device)
    B, L = context.shape[0], context.shape[1]
    # every CFG sample starts from the same rows when the latents, the timestep (and the VACE context)
    # are shared (the cfg_merge broadcast below): the first blocks' self-attention halves are then
    # computed once for all samples (DiTBlock shared_prefix)
    shared = B > 1 and latents.shape[0] == 1 and timestep.numel() == 1
    shared_vace = shared and vace_context is not None and vace_context.shape[0] == 1
    if latents.shape[0] != B:
        latents = latents.expand(B, *latents.shape[1:])
    latents = latents.to(BF16).contiguous()
    timestep = timestep.reshape(-1).to(device=device, dtype=BF16)
    if timestep.shape[0] != B:
        timestep = timestep.expand(B).contiguous()

    t, t_mod = dit.time_embed(timestep, ws)
    ctx = dit.text_embed(context.to(BF16), ws)
    x, grid = dit.patch_embedding(latents, ws, "x")
    S = grid[0] * grid[1] * grid[2]

    sp = None
    if use_unified_sequence_parallel:
        sp = sp_group
        if sp is None:
            from .usp import get_default_group
            sp = get_default_group()
        if sp is not None and sp.world_size == 1 and not getattr(sp, "force_collectives", False):
            sp = None
    rc = RunCtx(B, S, grid, dit.rope(device), ctx, L, ws)

    vace_x = None
    if vace_context is not None and vace is not None:
        vc = vace_context.to(BF16)
        if vc.shape[0] != B:
            vc = vc.expand(B, *vc.shape[1:])
        vace_x, _ = vace.vace_patch_embedding(vc.contiguous(), ws, "vace")

    # TeaCache (wan_video_new.py:1398-1402): decided on one prompt's t_mod before the blocks
    tea_skip = tea_cache.check(dit, x, t_mod[0:1]) if tea_cache is not None else False
    if sp is not None:
        x, vace_x, rc = sp.shard_tokens(x, vace_x, rc)

    if tea_skip:
        tea_cache.update(x)                                     # :1418-1419 (VACE not needed)
    else:
        if tea_cache is not None:
            tea_cache.begin(x)
        rc.t_emb = t
        hints = vace(x, vace_x, t_mod, rc, shared_prefix=shared_vace) if vace_x is not None else None
        vmap = vace.vace_layers_mapping if hints is not None else {}
        nblk = len(dit.blocks)
        # a batch-1 forward of CFG sample 1 (CFG-parallel rank) skips the slg blocks outright
        slg_here = B > 1 or cfg_sample == 1
        for i, blk in enumerate(dit.blocks):
            if B == 1 and cfg_sample == 1 and i in slg_blocks:
                continue
            hint = hints[vmap[i]] if i in vmap else None
            skip = B > 1 and i in slg_blocks
            # the next consumer of x, whose LayerNorm this block's FFN-down epilogue can take over
            # (not a skip-layer-guidance block, which runs on one sample's rows only or not at all)
            if i + 1 < nblk:
                nxt = None if (slg_here and i + 1 in slg_blocks) else dit.blocks[i + 1]
            else:
                nxt = None if tea_cache is not None else dit.head
            blk(x, t_mod, rc, hint=hint, hint_scale=float(vace_scale), only_batch=0 if skip else None, nxt=nxt,
                shared_prefix=shared and i == 0)
        if tea_cache is not None:
            tea_cache.store(x)                                  # :1455-1456
    out = dit.head(x, t, rc)
    if sp is not None:
        out = sp.gather_tokens(out, rc)
    T, H2, W2 = grid
    lat = torch.empty((B, dit.out_dim, T, 2 * H2, 2 * W2), device=device, dtype=BF16)
    K.unpatchify(out, lat)
    return lat


@dataclass
class ModelConfig:
    """diffsynth/utils/__init__.py:158-218, offline: resolves local files only (no ModelScope)."""
    path: Union[str, list, None] = None
    model_id: str = None
    origin_file_pattern: Union[str, list, None] = None
    download_resource: str = "ModelScope"
    offload_device: Optional[Union[str, torch.device]] = None
    offload_dtype: Optional[torch.dtype] = None
    local_model_path: str = None
    skip_download: bool = False

    def download_if_necessary(self, use_usp=False):
        if isinstance(self.path, str) and any(ch in self.path for ch in "*?["):
            import glob
            files = sorted(glob.glob(self.path))
            if not files:
                raise FileNotFoundError(f"no local files match {self.path}")
            self.path = files[0] if len(files) == 1 else files
        if self.path is not None:
            return
        if self.model_id is None:
            raise ValueError('No valid model files. Please use `ModelConfig(path="xxx")` or '
                             '`ModelConfig(model_id="xxx/yyy", origin_file_pattern="zzz")`.')
        import glob
        root = os.path.join(self.local_model_path or "./models", self.model_id)
        pattern = self.origin_file_pattern or ""
        if pattern == "" or pattern.endswith("/"):
            self.path = os.path.join(root, pattern)
            if not os.path.isdir(self.path):
                raise FileNotFoundError(f"{self.path} not found (offline build: no ModelScope download)")
            return
        files = sorted(glob.glob(os.path.join(root, pattern)))
        if not files:
            raise FileNotFoundError(f"no local files match {os.path.join(root, pattern)} "
                                    "(offline build: no ModelScope download)")
        self.path = files[0] if len(files) == 1 else files


# wan_video_new.py:352-363: the files every Wan2.1 release ships identically are read from one
# model_id, so a ./models tree laid out by the reference's downloads holds them only there
REDIRECT_COMMON_FILES = {
    "models_t5_umt5-xxl-enc-bf16.pth": "Wan-AI/Wan2.1-T2V-1.3B",
    "Wan2.1_VAE.pth": "Wan-AI/Wan2.1-T2V-1.3B",
    "models_clip_open-clip-xlm-roberta-large-vit-huge-14.pth": "Wan-AI/Wan2.1-I2V-14B-480P",
}


def redirect_model_configs(model_configs):
    """Rewrites model_id in place for the common files, with the reference's notice
    (wan_video_new.py:352-363).  Configs without a model_id or file pattern are left alone."""
    for mc in model_configs:
        if mc.origin_file_pattern is None or mc.model_id is None:
            continue
        if not isinstance(mc.origin_file_pattern, str):
            continue
        target = REDIRECT_COMMON_FILES.get(mc.origin_file_pattern)
        if target is not None and mc.model_id != target:
            print(f"To avoid repeatedly downloading model files, ({mc.model_id}, {mc.origin_file_pattern}) is "
                  f"redirected to ({target}, {mc.origin_file_pattern}). You can use `redirect_common_files=False` "
                  "to disable file redirection.")
            mc.model_id = target


def sp_graph_ok(plan):
    """True when the sequence-parallel plan's collectives can be captured into the step's hipGraph:
    host options sp_graph=1 and sp_comm=native (RCCL through libvstyler's vs_sp_*) -- not
    torch.distributed's RCCL, whose process-group stream the capture does not survive on this
    image's HIP (segfault in hipStreamEndCapture, profiles/r3/sp_graph_probe_faulthandler.log), and
    not host-staged substitutes (tests).  NativeComm in side-stream mode keeps its exchange/compute
    overlap in the graph: DenoiseStepper binds its comm stream to the capture origin and forks the
    compute (usp.NativeComm).  Opt-in: only world size 1 has run on hardware
    (test_ulysses_rccl_world1_graph_capture); SP steps run eager by default."""
    if not host_option("sp_graph"):
        return False
    if plan is None:
        from .usp import get_default_group
        plan = get_default_group()
    if plan is None:
        return True
    return all(getattr(p, "capturable", True) for p in
               (plan, getattr(plan, "ulysses", None), getattr(plan, "full", None)) if p is not None)


class DenoiseStepper:
    """Runs CFG denoising steps over device-resident state.  `step_fn(t_buf, d_buf)` enqueues one
    whole step (model_fn + fused CFG/Euler) reading the bf16 timestep and the fp32 dsigma from the
    two device slots.  The first call runs eagerly (sizing every Workspace buffer); the step is then
    captured once into a hipGraph and every later call refreshes the two slots and replays it.
    The eager step and the capture run on one dedicated stream, so the split-tail workspaces that
    libvstyler keeps per (device, stream) and allocates in the eager step are the ones the captured
    launches use (a capture on a fresh stream could not allocate them and would launch unsplit).

    comms: side-stream NativeComm objects of an SP plan (usp.plan_native_comms).  With a graph they
    are bound to the stepper's stream -- the capture origin -- and the step's compute runs on a
    second stream forked from it and joined back, so the collectives overlap the compute inside
    the graph while RCCL itself only ever runs on the origin stream.  plan: the step's SP plan (None
    without SP): the capture is refused while a side-stream communicator reachable from it is not
    bound to the capture stream (usp.unbound_side_comms)."""

    def __init__(self, step_fn, timesteps_bf16, dsigmas_f32, use_graph=True, on_replay=None, comms=(), plan=None):
        self.step_fn, self.ts, self.ds = step_fn, timesteps_bf16, dsigmas_f32
        self.t_buf, self.d_buf = timesteps_bf16[0:1].clone(), dsigmas_f32[0:1].clone()
        self.use_graph, self.graph, self.on_replay = use_graph, None, on_replay
        dev = self.t_buf.device
        self.stream = torch.cuda.Stream(device=dev) if use_graph else None
        self.comms = list(comms) if use_graph else []
        self.plan = plan
        self.compute = torch.cuda.Stream(device=dev) if self.comms else None

    def _run(self):
        if self.compute is None:
            self.step_fn(self.t_buf, self.d_buf)
            return
        self.compute.wait_stream(self.stream)          # fork
        with torch.cuda.stream(self.compute):
            self.step_fn(self.t_buf, self.d_buf)
        self.stream.wait_stream(self.compute)          # join

    def __call__(self, i):
        self.t_buf.copy_(self.ts[i:i + 1])
        self.d_buf.copy_(self.ds[i:i + 1])
        if self.graph is not None:
            self.graph.replay()
            if self.on_replay is not None:
                self.on_replay()
            return
        if not self.use_graph:
            self.step_fn(self.t_buf, self.d_buf)
            return
        cur = torch.cuda.current_stream(self.t_buf.device)
        self.stream.wait_stream(cur)
        old = [c.bind_stream(self.stream) for c in self.comms]
        try:
            with torch.cuda.stream(self.stream):
                self._run()
                self.capture()
        finally:
            for c, s in zip(self.comms, old):
                c.bind_stream(s)
        cur.wait_stream(self.stream)

    def capture(self):
        g = torch.cuda.CUDAGraph()
        err = None
        stray = []
        if self.plan is not None:
            from .usp import unbound_side_comms
            stray = unbound_side_comms(self.stream, self.plan)
        if stray:                   # RCCL forked into the capture from a side stream: never capture
            err = RuntimeError(f"{len(stray)} side-stream communicator(s) not bound to the capture stream")
        else:
            try:
                with torch.cuda.graph(g, stream=self.stream):
                    self._run()
            except Exception as e:      # e.g. a collective backend that cannot be captured: stay eager
                err = e
        # the decision is collective: with several ranks replaying graphs whose collectives must
        # pair up, one rank falling back to eager steps while the others replay would deadlock or
        # mismatch, so every rank keeps its graph only if every rank captured one
        if not self._all_ranks_agree(err is None):
            import warnings
            why = repr(err) if err is not None else "another rank's capture failed"
            warnings.warn(f"hipGraph capture of the denoising step failed ({why}); running eager steps")
            self.use_graph = False
            return
        self.graph = g

    def _all_ranks_agree(self, ok):
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return ok
        dev = self.t_buf.device if dist.get_backend() == "nccl" else torch.device("cpu")
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())


class WanVideoPipeline:
    """The Ditto drop-in (wan_video_new.py:32).  DiT/VACE/Euler/CFG on libvstyler kernels."""

    def __init__(self, device="cuda", torch_dtype=BF16, tokenizer_path=None):
        self.device = device
        self.torch_dtype = torch_dtype
        self.scheduler = FlowMatchScheduler(shift=5, sigma_min=0.0, extra_one_step=True)
        self.text_encoder = None
        self.prompter = None
        self.image_encoder = None
        self.dit: WanModel = None
        self.dit2 = None
        self.vae = None
        self.vace: VaceWanModel = None
        self.vace2 = None
        self.motion_controller = None
        self.animate_adapter = None
        self.model_fn = model_fn_wan_video
        self.height_division_factor = 16
        self.width_division_factor = 16
        self.time_division_factor = 4
        self.time_division_remainder = 1
        self.use_unified_sequence_parallel = False
        self.sp_group = None
        self.vram_management_enabled = False

    # ---------------------------------------------------------------- loading
    @staticmethod
    def from_pretrained(torch_dtype=BF16, device="cuda", model_configs=(), tokenizer_config=None,
                        audio_processor_config=None, redirect_common_files=True, use_usp=False):
        """wan_video_new.py:341-413 (local files only)."""
        from .loader import load_models
        if redirect_common_files:
            redirect_model_configs(model_configs)
        pipe = WanVideoPipeline(device=device, torch_dtype=torch_dtype)
        if use_usp:
            pipe.initialize_usp()
            device = pipe.device
        paths = []
        for mc in model_configs:
            mc.download_if_necessary(use_usp=use_usp)
            paths.append(mc.path)
        models = load_models(paths, device=device)
        pipe.dit = models.get("wan_video_dit")
        pipe.vace = models.get("wan_video_vace")
        pipe.vae = models.get("wan_video_vae")
        pipe.text_encoder = models.get("wan_video_text_encoder")
        if pipe.text_encoder is not None:
            from .t5 import WanPrompter
            tok = None
            if tokenizer_config is None:
                # the reference's default (wan_video_new.py:346): ./models/Wan-AI/Wan2.1-T2V-1.3B/google/*
                tokenizer_config = ModelConfig(model_id="Wan-AI/Wan2.1-T2V-1.3B", origin_file_pattern="google/*")
                try:
                    tokenizer_config.download_if_necessary()
                    tok = tokenizer_config.path
                except FileNotFoundError:
                    tok = None   # no local tokenizer: prompts need encode_ids / prompt_emb=
            else:
                tokenizer_config.download_if_necessary()
                tok = tokenizer_config.path
            if isinstance(tok, list):
                tok = os.path.dirname(tok[0])
            pipe.prompter = WanPrompter(tokenizer_path=tok)
            pipe.prompter.fetch_models(pipe.text_encoder)
        if use_usp:
            pipe.enable_usp()
        return pipe

    def load_lora(self, module, lora_config=None, alpha=1, hotload=False, state_dict=None):
        """wan_video_new.py:80-106."""
        from .lora import load_lora_state_dict, merge_lora, hotload_lora
        lora = state_dict if state_dict is not None else load_lora_state_dict(lora_config, self.device)
        if hotload:
            return hotload_lora(module, lora, alpha)
        return merge_lora(module, lora, alpha)

    def enable_vram_management(self, num_persistent_param_in_dit=None, vram_limit=None, vram_buffer=0.5):
        """wan_video_new.py:124.  On MI355X (288 GB HBM) every weight stays resident, so there is no
        offload state machine; LayerNorms already run in fp32 (WanAutoCastLayerNorm semantics)."""
        self.vram_management_enabled = True

    def initialize_usp(self):
        from .usp import init_distributed
        rank = init_distributed()
        self.device = f"cuda:{rank}"

    def enable_usp(self):
        from .usp import get_default_group
        self.sp_group = get_default_group()
        self.use_unified_sequence_parallel = True

    # ---------------------------------------------------------------- helpers
    def check_resize_height_width(self, height, width, num_frames=None):
        """utils/__init__.py:43-57."""
        if height % self.height_division_factor != 0:
            height = (height + self.height_division_factor - 1) // self.height_division_factor * self.height_division_factor
        if width % self.width_division_factor != 0:
            width = (width + self.width_division_factor - 1) // self.width_division_factor * self.width_division_factor
        if num_frames is None:
            return height, width
        if num_frames % self.time_division_factor != self.time_division_remainder:
            num_frames = (num_frames + self.time_division_factor - 1) // self.time_division_factor * \
                self.time_division_factor + self.time_division_remainder
        return height, width, num_frames

    def generate_noise(self, shape, seed=None, rand_device="cpu", rand_torch_dtype=torch.float32):
        """utils/__init__.py:117-122 (same CPU generator stream -> identical noise)."""
        generator = None if seed is None else torch.Generator(rand_device).manual_seed(seed)
        noise = torch.randn(shape, generator=generator, device=rand_device, dtype=rand_torch_dtype)
        return noise.to(dtype=self.torch_dtype, device=self.device)

    # ---------------------------------------------------------------- denoise
    def denoise(self, latents, context_posi, context_nega, vace_context=None, vace_scale=1.0, cfg_scale=5.0,
                num_inference_steps=50, sigma_shift=5.0, denoising_strength=1.0, progress_bar_cmd=None,
                use_graph=None, tea_cache=None):
        """The loop of wan_video_new.py:515-542 (cfg_merge batched), returns the final latents.

        Step 0 runs eagerly (it also sizes the Workspace); the whole step -- model_fn (DiT + VACE,
        CFG as one batch-2 forward) + fused CFG/Euler update -- is then captured once into a hipGraph
        (torch.cuda.CUDAGraph over hipStreamBeginCapture) and replayed for every later step.  The
        graph reads the step's bf16 timestep and fp32 dsigma from two device slots refreshed before
        each replay, so one capture serves all steps.  Under Ulysses SP the RCCL collectives (async
        all-to-alls on RCCL's stream, event-ordered) are captured with the step only with host option
        sp_graph=1 (sp_graph_ok); eager with use_graph=False / host option graph=0."""
        self.scheduler.set_timesteps(num_inference_steps, denoising_strength=denoising_strength, shift=sigma_shift)
        n_steps = len(self.scheduler.timesteps)
        use_cfg = cfg_scale != 1.0
        if use_graph is None:
            use_graph = bool(host_option("graph"))
        # TeaCache decides per step on the host (wan_video_new.py:1173-1192): eager steps
        use_graph = use_graph and n_steps > 1 and tea_cache is None and \
            (not self.use_unified_sequence_parallel or sp_graph_ok(self.sp_group))
        ctx = torch.cat([context_posi, context_nega], 0) if use_cfg else context_posi
        latents = latents.to(device=self.device, dtype=BF16).contiguous().clone()
        ts = self.scheduler.timesteps.to(dtype=BF16).to(self.device)                     # :526
        ds = torch.tensor([self.scheduler.delta(i) for i in range(n_steps)], dtype=torch.float32,
                          device=self.device)

        def step(t_buf, d_buf):
            v = self.model_fn(dit=self.dit, vace=self.vace, latents=latents, timestep=t_buf, context=ctx,
                              vace_context=vace_context, vace_scale=vace_scale,
                              use_unified_sequence_parallel=self.use_unified_sequence_parallel,
                              sp_group=self.sp_group, tea_cache=tea_cache)
            K.cfg_euler_dev(v[0:1], v[1:2] if use_cfg else None, latents, cfg_scale, d_buf)

        comms, plan = (), None
        if self.use_unified_sequence_parallel:
            from .usp import get_default_group, plan_native_comms
            plan = self.sp_group if self.sp_group is not None else get_default_group()
            comms = plan_native_comms(plan) if use_graph else ()
        stepper = DenoiseStepper(step, ts, ds, use_graph, comms=comms, plan=plan)
        steps = range(n_steps)
        if progress_bar_cmd is not None:
            steps = progress_bar_cmd(steps)
        for i in steps:
            stepper(i)
        self.last_graph = stepper.graph
        return latents

    def denoise_unipc(self, latents, context_posi, context_nega, vace_context=None, vace_scale=1.0,
                      cfg_scale=1.2, num_inference_steps=4, sigma_shift=2.0, slg_blocks=(), slg_range=(0.2, 0.7),
                      progress_bar_cmd=None):
        """Config 5's sampler (ditto_comfyui_workflow.json WanVideoSampler 4 / 1.2 / 2.0 / unipc with
        WanVideoSLG): FlowUniPCMultistepScheduler (vstyler.unipc) on fp32 latents, CFG as one
        batch-2 forward, skip-layer guidance on the uncond sample for step fractions in slg_range.
        CFG combine in bf16 (wan_video_new.py:535 semantics), model input bf16 each step."""
        from .unipc import FlowUniPCMultistepScheduler, cast
        sched = FlowUniPCMultistepScheduler(shift=1.0)
        sched.set_timesteps(num_inference_steps, shift=sigma_shift)
        use_cfg = cfg_scale != 1.0
        ctx = torch.cat([context_posi, context_nega], 0) if use_cfg else context_posi
        lat32 = latents.to(device=self.device, dtype=torch.float32).contiguous().clone()
        lat16 = torch.empty(lat32.shape, dtype=BF16, device=self.device)
        v16 = torch.empty(lat32.shape, dtype=BF16, device=self.device)
        v32 = torch.empty_like(lat32)
        n = len(sched.timesteps)
        steps = range(n)
        if progress_bar_cmd is not None:
            steps = progress_bar_cmd(steps)
        for i in steps:
            t = sched.timesteps[i]
            cast(lat32, lat16)
            frac = i / n
            slg = tuple(slg_blocks) if slg_range[0] <= frac <= slg_range[1] else ()
            v = self.model_fn(dit=self.dit, vace=self.vace, latents=lat16, timestep=t.reshape(1).to(
                dtype=BF16, device=self.device), context=ctx, vace_context=vace_context, vace_scale=vace_scale,
                use_unified_sequence_parallel=self.use_unified_sequence_parallel, sp_group=self.sp_group,
                slg_blocks=slg)
            v16.zero_()
            K.cfg_euler(v[0:1], v[1:2] if use_cfg else None, v16, cfg_scale, 1.0)   # v16 = cfg combine
            cast(v16, v32)
            lat32 = sched.step(v32, t, lat32)[0]
        return cast(lat32, torch.empty(lat32.shape, dtype=BF16, device=self.device))

    @torch.no_grad()
    def __call__(self, prompt=None, negative_prompt="", input_image=None, end_image=None, input_video=None,
                 denoising_strength=1.0, vace_video=None, vace_video_mask=None, vace_reference_image=None,
                 vace_scale=1.0, seed=None, rand_device="cpu", height=480, width=832, num_frames=81,
                 cfg_scale=5.0, cfg_merge=False, switch_DiT_boundary=0.875, num_inference_steps=50,
                 sigma_shift=5.0, motion_bucket_id=None, tiled=True, tile_size=(30, 52), tile_stride=(15, 26),
                 sliding_window_size=None, sliding_window_stride=None, tea_cache_l1_thresh=None,
                 tea_cache_model_id="", progress_bar_cmd=None,
                 # extensions of this build (the DiT path without T5/VAE):
                 prompt_emb=None, negative_prompt_emb=None, vace_context=None, output_type="video", **kwargs):
        """wan_video_new.py:416-560 for the Ditto path (T2V/VACE, no image/audio/camera inputs)."""
        for name, val in (("input_image", input_image), ("end_image", end_image), ("input_video", input_video),
                          ("motion_bucket_id", motion_bucket_id), ("sliding_window_size", sliding_window_size)):
            if val is not None:
                raise NotImplementedError(f"{name} is outside the Ditto hot path of this build")
        height, width, num_frames = self.check_resize_height_width(height, width, num_frames)
        T = (num_frames - 1) // 4 + 1
        # WanVideoUnit_NoiseInitializer (wan_video_new.py:578-587): f reference images add f latent
        # frames, and the noise is rolled so the last f frames come first
        nref = 0
        if vace_reference_image is not None:
            nref = len(vace_reference_image) if isinstance(vace_reference_image, (list, tuple)) else 1
        noise = self.generate_noise((1, 16, T + nref, height // 8, width // 8), seed=seed, rand_device=rand_device)
        if nref:
            noise = torch.cat((noise[:, :, -nref:], noise[:, :, :-nref]), dim=2)
        if prompt_emb is None:
            prompt_emb = self.encode_prompt(prompt)
        if negative_prompt_emb is None and cfg_scale != 1.0:
            negative_prompt_emb = self.encode_prompt(negative_prompt)
        if vace_context is None and (vace_video is not None or vace_video_mask is not None or nref):
            vace_context = self.encode_vace(vace_video, vace_video_mask, height, width, num_frames, tiled,
                                            tile_size, tile_stride, vace_reference_image)
        tea_cache = None
        if tea_cache_l1_thresh is not None:                # WanVideoUnit_TeaCache (:936-947)
            from .teacache import TeaCache
            tea_cache = TeaCache(num_inference_steps, rel_l1_thresh=tea_cache_l1_thresh, model_id=tea_cache_model_id)
        latents = self.denoise(noise, prompt_emb.to(self.device), None if negative_prompt_emb is None else
                               negative_prompt_emb.to(self.device),
                               None if vace_context is None else vace_context.to(self.device), vace_scale,
                               cfg_scale, num_inference_steps, sigma_shift, denoising_strength, progress_bar_cmd,
                               tea_cache=tea_cache)
        self.last_tea_cache = tea_cache
        if nref:                                            # :545-550
            latents = latents[:, :, nref:].contiguous()
        if output_type == "latents":
            return latents
        if self.vae is None:
            raise RuntimeError("VAE decode requires a loaded Wan2.1 VAE (or use output_type='latents')")
        video = self.vae.decode(latents, device=self.device, tiled=tiled, tile_size=tile_size, tile_stride=tile_stride)
        return self.vae_output_to_video(video, output_type)

    def encode_prompt(self, prompt):
        if self.text_encoder is None or self.prompter is None:
            raise NotImplementedError("T5 text encoder not loaded: pass prompt_emb=/negative_prompt_emb=")
        return self.prompter.encode_prompt(prompt, device=self.device)

    def encode_vace(self, vace_video, vace_video_mask, height, width, num_frames, tiled, tile_size, tile_stride,
                    vace_reference_image=None):
        """WanVideoUnit_VACE (wan_video_new.py:861-920): 2 tiled VAE encodes + mask latents (+ one
        encode per reference image)."""
        if self.vae is None:
            raise RuntimeError("VACE video encoding requires a loaded Wan2.1 VAE (or pass vace_context=)")
        from .vae import vace_context
        if vace_video is not None and not isinstance(vace_video, torch.Tensor):
            vace_video = list(vace_video)[:num_frames]
        if vace_video_mask is not None and not isinstance(vace_video_mask, torch.Tensor):
            vace_video_mask = list(vace_video_mask)[:num_frames]
        return vace_context(self.vae, vace_video, vace_video_mask, num_frames, height, width, tiled, tile_size,
                            tile_stride, vace_reference_image)

    def vae_output_to_video(self, vae_output, output_type="video"):
        """BasePipeline.vae_output_to_video (utils/__init__.py:76-91): uint8 conversion on the GPU;
        output_type "u8" returns the (T, H, W, 3) uint8 device tensor, "video" PIL images."""
        from .vae import vae_output_to_u8
        u8 = vae_output_to_u8(vae_output[0])
        if output_type == "u8":
            return u8
        from PIL import Image
        return [Image.fromarray(f) for f in u8.cpu().numpy()]
