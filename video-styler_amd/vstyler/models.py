"""Wan2.1 DiT + VACE branch on MI355X.

Parameter containers keep the reference's module names and shapes (so a reference state dict
loads by name and reproduces the reference's md5 key-layout hash, models/utils.py:148-182); the
forward passes are sequences of libvstyler kernels (vstyler.kernels), never torch math.

Reference: diffsynth/models/wan_video_dit.py (DiTBlock :196-230, Head :253-269, WanModel
:272-352), diffsynth/models/wan_video_vace.py (:5-87), model_fn_wan_video
(diffsynth/pipelines/wan_video_new.py:1260-1468).
"""
import math

import torch
import torch.nn as nn

from . import kernels as K
from .options import host_option

BF16 = torch.bfloat16


def _param(*shape, device=None, dtype=BF16):
    return nn.Parameter(torch.empty(*shape, device=device, dtype=dtype), requires_grad=False)


class Linear(nn.Module):
    """Weight [out, in] + bias, bf16 (the nn.Linear layout the MFMA GEMM reads K-contiguous)."""

    def __init__(self, in_features, out_features, bias=True, device=None, dtype=BF16):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = _param(out_features, in_features, device=device, dtype=dtype)
        self.bias = _param(out_features, device=device, dtype=dtype) if bias else None


class Q8:
    """An activation already quantised for fp8_linear (x8 e4m3 bytes [M, K], per-row scale [M]): what
    ln_into() hands to linear() / fused_linear() when the consumer is an fp8 layer."""

    def __init__(self, x8, scale):
        self.x8, self.scale = x8, scale
        self.shape = x8.shape


def _fp8_consumer(target):
    """True when `target` (a Linear, or a module whose fused projections run as one GEMM) consumes
    its input through fp8_linear."""
    if isinstance(target, AttentionParams):
        f = _fused_views(target)
        return f is not None and f[2] is not None
    return getattr(target, "weight_fp8", None) is not None and getattr(target, "lora_A", None) is None


def ln_into(x, h, ws, target, eps, **ln):
    """LayerNorm(+modulate) of x for `target`'s projection: into the bf16 buffer h, or -- when target
    runs fp8_linear -- straight into its quantised activation (vs_layernorm_modulate_fp8: the bf16 row
    is never stored and not re-read; bit-identical)."""
    if target is not None and _fp8_consumer(target):
        M, D = x.shape
        return Q8(*K.layernorm_modulate_fp8(x, ws.get("fp8_x", (M, D), torch.uint8),
                                            ws.get("fp8_scale", (M,), torch.float32), eps, **ln))
    K.layernorm_modulate(x, h, eps, **ln)
    return h


def linear(lin, x, out, ws, **epi):
    """Linear through vs_gemm; a hot-loaded LoRA (lin.lora_A = alpha*A, lin.lora_B = B) is fused as
    the GEMM's second K phase (AutoWrappedLinear, vram_management/layers.py:173-188).  A layer
    converted by quantize_fp8_ runs the fp8 path of AutoWrappedLinear.fp8_linear (:115-151):
    per-row activation quantisation (or the Q8 input ln_into made) + e4m3 MFMA GEMM with the same
    fused epilogue."""
    w8 = getattr(lin, "weight_fp8", None)
    if w8 is not None:
        if getattr(lin, "lora_A", None) is not None:
            raise NotImplementedError("hot-loaded LoRA on an fp8 layer: merge the LoRA before quantize_fp8_")
        if isinstance(x, Q8):
            return K.gemm_fp8(x.x8, x.scale, w8, out, bias=lin.bias, **epi)
        M, Kd = x.shape
        x8 = ws.get("fp8_x", (M, Kd), torch.uint8)
        sc = ws.get("fp8_scale", (M,), torch.float32)
        K.quant_fp8_rows(x, x8, sc)
        return K.gemm_fp8(x8, sc, w8, out, bias=lin.bias, **epi)
    if isinstance(x, Q8):
        raise ValueError("a quantised activation for a bf16 layer")
    la = getattr(lin, "lora_A", None)
    a2 = w2 = None
    if la is not None:
        t = ws.get("lora_t", (x.shape[0], la.shape[0]))
        K.gemm(x, la, t)
        a2, w2 = t, lin.lora_B
    return K.gemm(x, lin.weight, out, bias=lin.bias, a2=a2, w2=w2, **epi)


def _fusable_lt(lin, M, epilogue):
    """True when `lin` on M rows with the residual `epilogue` would run as a staged product + a separate
    epilogue pass (vs_gemm_route_epi != 0: the vendor-library route of the A/B build only; the
    product library fuses every epilogue), i.e. when that pass could fuse with the LayerNorm that
    follows (vs_residual_layernorm) with the same rounding points.  Otherwise the residual epilogue is
    fused into the GEMM and the LayerNorm runs alone.  A hot-loaded LoRA keeps the MFMA kernel's fused
    epilogue.  Host option fuse_res_ln=0 disables."""
    if getattr(lin, "lora_A", None) is not None or not host_option("fuse_res_ln"):
        return False
    fp8 = getattr(lin, "weight_fp8", None) is not None
    return K.gemm_route(M, lin.out_features, lin.in_features, epilogue=epilogue, fp8=fp8)


def quantize_fp8_(module):
    """Give every block Linear (self/cross-attention q/k/v/o, FFN; DiT and VACE blocks) an e4m3fn
    copy of its weight (weight.to(float8_e4m3fn), as fp8_linear casts it, layers.py:133) used by
    linear(); embeddings, VACE before/after projections and the head stay bf16."""
    n = 0
    for blk in [m for m in module.modules() if isinstance(m, DiTBlock)]:
        for att in (blk.self_attn, blk.cross_attn):
            att._fw8 = None
            if _fused_views(att) is not None:       # fused q|k|v / k|v: one e4m3 buffer, per-Linear views
                att._fw8 = att._fw.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
        for lin in (blk.self_attn.q, blk.self_attn.k, blk.self_attn.v, blk.self_attn.o, blk.cross_attn.q,
                    blk.cross_attn.k, blk.cross_attn.v, blk.cross_attn.o, blk.ffn[0], blk.ffn[2]):
            lin.weight_fp8 = lin.weight.detach().to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
            n += 1
        for att in (blk.self_attn, blk.cross_attn):
            if att._fw8 is not None:
                d = att.dim
                for i, name in enumerate(att.fused):
                    getattr(att, name).weight_fp8 = att._fw8[i * d:(i + 1) * d]
    return n


class PatchEmbed(nn.Module):
    """Conv3d(in, dim, k=s=(1,2,2)) parameters (wan_video_dit.py:306-307)."""

    def __init__(self, in_dim, dim, device=None):
        super().__init__()
        self.in_dim, self.dim = in_dim, dim
        self.weight = _param(dim, in_dim, 1, 2, 2, device=device)
        self.bias = _param(dim, device=device)

    def forward(self, lat, ws, tag):
        B, C, T, H, W = lat.shape
        S = T * (H // 2) * (W // 2)
        cols = ws.get(tag + ".cols", (B * S, C * 4))
        K.patchify(lat.contiguous(), cols)
        out = ws.get(tag + ".out", (B * S, self.dim))
        K.gemm(cols, self.weight.view(self.dim, C * 4), out, bias=self.bias)
        return out, (T, H // 2, W // 2)


class RMSNormW(nn.Module):
    def __init__(self, dim, device=None):
        super().__init__()
        self.weight = _param(dim, device=device)


class LayerNormAffine(nn.Module):
    def __init__(self, dim, device=None):
        super().__init__()
        self.weight = _param(dim, device=device)
        self.bias = _param(dim, device=device)


class AttentionParams(nn.Module):
    """q/k/v/o Linears + QK norms under the reference's key names.  The Linears listed in `fused`
    (same input: q|k|v of self-attention, k|v of cross-attention) keep their weights and biases as
    row slices of one [n*dim, dim] / [n*dim] buffer, so their projections run as ONE GEMM
    (fused_linear); state-dict loading, LoRA merging and init all write through the slices."""

    def __init__(self, dim, num_heads, device=None, fused=()):
        super().__init__()
        self.dim, self.num_heads = dim, num_heads
        self.q = Linear(dim, dim, device=device)
        self.k = Linear(dim, dim, device=device)
        self.v = Linear(dim, dim, device=device)
        self.o = Linear(dim, dim, device=device)
        self.norm_q = RMSNormW(dim, device=device)
        self.norm_k = RMSNormW(dim, device=device)
        self.fused = tuple(fused)
        self._fw = self._fb = self._fw8 = None
        if self.fused:
            n = len(self.fused)
            self._fw = torch.empty(n * dim, dim, device=device, dtype=BF16)
            self._fb = torch.empty(n * dim, device=device, dtype=BF16)
            for i, name in enumerate(self.fused):
                lin = getattr(self, name)
                lin.weight = nn.Parameter(self._fw[i * dim:(i + 1) * dim], requires_grad=False)
                lin.bias = nn.Parameter(self._fb[i * dim:(i + 1) * dim], requires_grad=False)


def _fused_views(mod):
    """(W, b, W8 or None) when the fused Linears still alias the fused buffers (nothing rebound
    their parameters, no hot-loaded LoRA, fp8 copies all present or all absent), else None."""
    if not getattr(mod, "fused", ()) or mod._fw is None:
        return None
    d = mod.dim
    fp8 = [getattr(getattr(mod, n), "weight_fp8", None) is not None for n in mod.fused]
    if any(fp8) and (not all(fp8) or mod._fw8 is None):
        return None
    for i, name in enumerate(mod.fused):
        lin = getattr(mod, name)
        if getattr(lin, "lora_A", None) is not None:
            return None
        if lin.weight.data_ptr() != mod._fw[i * d].data_ptr() or lin.bias is None or \
                lin.bias.data_ptr() != mod._fb[i * d:].data_ptr():
            return None
        if fp8[i] and lin.weight_fp8.data_ptr() != mod._fw8[i * d].data_ptr():
            return None
    return mod._fw, mod._fb, (mod._fw8 if all(fp8) else None)


def fused_linear(mod, x, ws, tag):
    """All of mod.fused's projections of x as one GEMM into a [M, n*dim] buffer (column block i =
    Linear i), or None when the fusion does not apply (the caller runs them one by one)."""
    f = _fused_views(mod)
    if f is None:
        return None
    W, b, W8 = f
    out = ws.get("fused" + tag, (x.shape[0], W.shape[0]))
    if W8 is not None and isinstance(x, Q8):
        return K.gemm_fp8(x.x8, x.scale, W8, out, bias=b)
    if W8 is not None:
        M, Kd = x.shape
        x8 = ws.get("fp8_x", (M, Kd), torch.uint8)
        sc = ws.get("fp8_scale", (M,), torch.float32)
        K.quant_fp8_rows(x, x8, sc)
        return K.gemm_fp8(x8, sc, W8, out, bias=b)
    return K.gemm(x, W, out, bias=b)


class Sequential3(nn.Module):
    """Holds modules at indices 0 and 2 (Linear, act, Linear) to keep the reference's key names."""

    def __init__(self, first, last):
        super().__init__()
        self.add_module("0", first)
        self.add_module("2", last)

    def __getitem__(self, i):
        return getattr(self, str(i))


class Workspace:
    """Scratch buffers reused across blocks/steps (allocated once per shape; kernels never allocate)."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}

    def get(self, name, shape, dtype=BF16):
        shape = tuple(int(s) for s in shape)
        t = self.bufs.get(name)
        if t is None or t.shape != shape or t.dtype != dtype:
            t = torch.empty(shape, device=self.device, dtype=dtype)
            if host_option("ws_poison"):    # debugging aid: NaN-fill so a read-before-write shows up
                t.view(torch.uint8).fill_(0xFF)
            self.bufs[name] = t
        return t


class KernelTimer:
    """Optional HIP-event bracketing of chosen launches (bench.py roofline): events are recorded on
    the stream the kernel is launched on (torch's current stream), elapsed times read afterwards.
    Inactive while a hipGraph is being captured (ROCm refuses external event nodes in graphs)."""

    def __init__(self):
        self.enabled = False
        self.events = {}

    def start(self, name, flops=0.0):
        """flops: the launch's algorithmic FLOPs (tflops() divides their sum by the summed time)."""
        if not self.enabled or torch.cuda.is_current_stream_capturing():
            return None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        self.events.setdefault(name, []).append((e0, e1, float(flops)))
        return e1

    def stop(self, e1):
        if e1 is not None:
            e1.record()

    def mean_ms(self, name):
        ev = self.events.get(name, [])
        if not ev:
            return None, 0
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev), len(ev)

    def tflops(self, name):
        """Summed FLOPs / summed launch time of the bracketed launches (TFLOP/s), or None."""
        ev = self.events.get(name, [])
        if not ev:
            return None
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b, _ in ev)
        return sum(f for _, _, f in ev) / (ms / 1000.0) / 1e12 if ms > 0 else None

    def reset(self):
        self.events = {}


TIMER = KernelTimer()


def attn_flops(q, k, batch):
    """4 Sq Skv (heads x d) per sample: QK^T and PV of one attention launch (q: [batch Sq, heads d])."""
    return 4.0 * (q.shape[0] // batch) * (k.shape[0] // batch) * q.shape[1] * batch


class RunCtx:
    """Per-forward constants shared by all blocks: batch/token geometry, RoPE table, SP info."""

    def __init__(self, batch, seq, grid, rope, ctx, ctx_len, ws, sp=None, token_offset=0):
        self.batch, self.seq, self.grid, self.rope = batch, seq, grid, rope
        self.ctx, self.ctx_len, self.ws = ctx, ctx_len, ws
        self.sp = sp                    # vstyler.usp.UlyssesGroup or None
        self.token_offset = token_offset
        # set by a block whose FFN-down residual was fused with the next consumer's LayerNorm
        # (DiTBlock.forward nxt=): the ws buffer holding the next block's modulation, whose h
        # buffers then already hold its modulated LN1
        self.pre_mod = None
        self.mod_slot = 0
        self.t_emb = None               # the time embedding t [B, D] (the head's modulation input)


class DiTBlock(nn.Module):
    """wan_video_dit.py:196-230 parameters; forward = fused kernel sequence on [B*S, D] rows."""

    def __init__(self, dim, num_heads, ffn_dim, eps=1e-6, device=None):
        super().__init__()
        self.dim, self.num_heads, self.ffn_dim, self.eps = dim, num_heads, ffn_dim, eps
        self.self_attn = AttentionParams(dim, num_heads, device, fused=("q", "k", "v"))
        self.cross_attn = AttentionParams(dim, num_heads, device, fused=("k", "v"))
        self.norm3 = LayerNormAffine(dim, device)
        self.ffn = Sequential3(Linear(dim, ffn_dim, device=device), Linear(ffn_dim, dim, device=device))
        self.modulation = _param(1, 6, dim, device=device)

    def forward(self, x, t_mod, rc, hint=None, hint_scale=1.0, only_batch=None, nxt=None, shared_prefix=False):
        """x: [B*S, D] updated in place.  t_mod: [B, 6, D].  hint: [B*S, D] added after the block.
        only_batch: run the block for that CFG sample only (skip-layer guidance leaves the others'
        rows untouched).  nxt: the module that consumes x next (a DiTBlock or the Head) when it runs
        on all rows: the FFN-down gate-residual (+ VACE hint) is then fused with its modulated
        LayerNorm (vs_residual_layernorm, one pass over the rows instead of two).

        Four phases per micro-batch: (1) LN1 + q/k/v + QK-RMSNorm/RoPE, (2) self-attention,
        (3) o-proj (gated residual) + LN3, (4) cross-attention, FFN (gated residual + VACE hint).
        Without SP the whole CFG batch is one micro-batch.  Under Ulysses SP with overlap on, each
        CFG sample is its own micro-batch for phases 1-3, issued 1(0) 1(1) 2(0) 2(1) 3(0) 3(1): sample
        0's q|k|v all-to-all runs under sample 1's projections, sample 1's under sample 0's
        attention, sample 0's return exchange under sample 1's attention and sample 1's under sample
        0's o-proj; phase 4 then runs once on both samples' rows (GEMMs of 2S/p rows instead of two
        of S/p: host option sp_merge_ffn=0 keeps it per sample).

        shared_prefix (r6): the caller guarantees that every CFG sample's rows of x and of t_mod are
        equal (the first DiT block and the first VACE block, when the latents, the timestep and the VACE
        context are shared -- they differ only through the context, which phase 4 first reads), so
        phases 1-3 run on sample 0's rows alone and their outputs (x after the gated o-proj, the LN3
        rows) are copied to the other samples before phase 4 runs on all rows -- its cross-attention
        query too comes from sample 0's rows alone: the same per-row arithmetic, bit-identical
        (tests/test_model_gpu.py), half the self-attention of those blocks."""
        B, S, D, ws = rc.batch, rc.seq, self.dim, rc.ws
        if rc.pre_mod is not None:          # the previous block already ran this one's LN1
            mod, ln1_done = rc.pre_mod, True
            rc.pre_mod = None
        else:
            rc.mod_slot ^= 1
            mod, ln1_done = ws.get(f"mod{rc.mod_slot}", (B, 6, D)), False
            K.mod_add(self.modulation.view(6, D), t_mod, mod, 6 * D, D)   # :218-219
        sp = rc.sp
        shared = shared_prefix and B > 1 and only_batch is None and bool(host_option("cfg_prefix"))
        if only_batch is not None:
            assert not ln1_done, "a skip-layer-guidance block cannot start from a fused LN1"
            parts = [self._part(x, mod, rc, only_batch, 1, hint, f".{only_batch}")]
        elif shared:
            parts = [self._part(x, mod, rc, 0, 1, hint, ".0")]
        elif sp is not None and B > 1 and getattr(sp, "overlap", False):
            parts = [self._part(x, mod, rc, b, 1, hint, f".{b}") for b in range(B)]
        else:
            parts = [self._part(x, mod, rc, 0, B, hint, "")]
        for p in parts:
            p["ln1_done"] = ln1_done
        # phase 4 on all rows at once (the overlapped SP micro-batches, the shared prefix)
        tail = self._part(x, mod, rc, 0, B, hint, "") if shared or (len(parts) > 1 and
                                                                    host_option("sp_merge_ffn")) else None
        # the fused FFN-down epilogue needs the consumer's modulation first (its own mod buffer)
        fuse = None
        if nxt is not None and only_batch is None and \
                _fusable_lt(self.ffn[2], (tail or parts[0])["M"], K.VS_EPI_GATE_RES) and \
                host_option("fuse_ffn_ln"):
            if isinstance(nxt, DiTBlock):
                nslot = rc.mod_slot ^ 1
                nmod = ws.get(f"mod{nslot}", (B, 6, D))
                K.mod_add(nxt.modulation.view(6, D), t_mod, nmod, 6 * D, D)
                fuse = dict(shift=nmod[:, 0], scale=nmod[:, 1], bstride=6 * D, mod=nmod, slot=nslot)
            elif isinstance(nxt, Head) and (len(parts) == 1 or tail is not None):
                hm = nxt.modulation_for(rc.t_emb, rc)
                fuse = dict(shift=hm[:, 0], scale=hm[:, 1], bstride=2 * D, mod=None)
        for p in parts:
            self._phase_qkv(p, rc)
        for p in parts:
            self._phase_attn(p, rc)
        for p in parts:
            self._phase_o(p, rc, direct=tail is None)
            if tail is None:
                self._phase_cross_ffn(p, rc, hint_scale, fuse)
        if shared:                          # sample 0's phase 1-3 results are every sample's: x, and the
            xs = x.view(B, S, D)            # cross-attention query (from sample 0's LN3 rows in h)
            xs[1:].copy_(xs[0:1].expand(B - 1, S, D))
            tail["shared_q"] = True
        if tail is not None:
            self._phase_cross_ffn(tail, rc, hint_scale, fuse)
        if fuse is not None:
            if fuse["mod"] is not None:
                rc.pre_mod = fuse["mod"]
                rc.mod_slot = fuse["slot"]
            else:
                rc.head_ln_done = True
        return x

    def _part(self, x, mod, rc, b0, nb, hint, tag):
        S, D, L, ws = rc.seq, self.dim, rc.ctx_len, rc.ws
        r0, M = b0 * S, nb * S
        p = dict(nb=nb, M=M, b0=b0, x=x[r0:r0 + M], mod=mod[b0:b0 + nb], ctx=rc.ctx[b0 * L:(b0 + nb) * L],
                 hint=None if hint is None else hint[r0:r0 + M], tag=tag)
        for n in ("h", "q", "k", "v", "o"):     # row slices of the all-samples buffers
            p[n] = ws.get(n, (rc.batch * S, D))[r0:r0 + M]
        return p

    def _phase_qkv(self, p, rc):
        # --- self-attention inputs (wan_video_dit.py:225-226, :140-145)
        S, D, eps, ws = rc.seq, self.dim, self.eps, rc.ws
        mod, h, q, k, v = p["mod"], p["h"], p["q"], p["k"], p["v"]
        sa = self.self_attn
        if not p["ln1_done"]:
            h = ln_into(p["x"], h, ws, sa, eps, shift=mod[:, 0], scale=mod[:, 1], mod_bstride=6 * D,
                        rows_per_batch=S)
        qkv = fused_linear(sa, h, ws, "qkv" + p["tag"])
        if qkv is not None:            # one GEMM; q/k/v are column slices of [M, 3D]
            q, k, v = p["q"], p["k"], p["v"] = qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:]
        else:
            linear(sa.q, h, q, ws)
            linear(sa.k, h, k, ws)
            linear(sa.v, h, v, ws)
        K.rmsnorm_rope(q, sa.norm_q.weight, eps, rope=rc.rope, grid=rc.grid, rows_per_batch=S,
                       token_offset=rc.token_offset)
        K.rmsnorm_rope(k, sa.norm_k.weight, eps, rope=rc.rope, grid=rc.grid, rows_per_batch=S,
                       token_offset=rc.token_offset)
        if rc.sp is not None:
            p["xchg"] = rc.sp.exchange_start(q, k, v, self.num_heads, p["nb"], p["tag"])

    def _phase_attn(self, p, rc):
        if rc.sp is not None:
            rc.sp.attend(p["xchg"])
        else:
            ev = TIMER.start("self_attn", attn_flops(p["q"], p["k"], p["nb"]))
            K.attention(p["q"], p["k"], p["v"], p["o"], self.num_heads, p["nb"])
            TIMER.stop(ev)

    def _phase_o(self, p, rc, direct=True):
        """direct: this part's cross-attention runs next (its LN3 may go straight into an fp8 cross-q's
        quantised input); False: the merged SP tail reads the bf16 LN3 rows of every part."""
        S, D, eps, ws = rc.seq, self.dim, self.eps, rc.ws
        x, mod, h, o, M = p["x"], p["mod"], p["h"], p["o"], p["M"]
        if rc.sp is not None:
            rc.sp.finish(p["xchg"], o)
        sa = self.self_attn
        if _fusable_lt(sa.o, M, K.VS_EPI_GATE_RES):
            # hipBLASLt route: bf16(o Wo^T + b) staged, then gate-residual + LN3 in one pass
            y = ws.get("res_y" + p["tag"], (M, D))
            linear(sa.o, o, y, ws)
            K.residual_layernorm(y, x, h, eps, epilogue=K.VS_EPI_GATE_RES, gate=mod[:, 2], gate_bstride=6 * D,
                                 gate_rows=S, weight=self.norm3.weight, bias=self.norm3.bias)
        else:
            linear(sa.o, o, x, ws, epilogue=K.VS_EPI_GATE_RES, residual=x, gate=mod[:, 2],
                   gate_bstride=6 * D, rows_per_batch=S)
            # --- cross-attention (wan_video_dit.py:227, :171-186)
            p["h3"] = ln_into(x, h, ws, self.cross_attn.q if direct else None, eps, weight=self.norm3.weight,
                              bias=self.norm3.bias)

    def _phase_cross_ffn(self, p, rc, hint_scale, fuse=None):
        S, D, eps, ws = rc.seq, self.dim, self.eps, rc.ws
        x, mod, h, q, o, nb, M = p["x"], p["mod"], p["h"], p["q"], p["o"], p["nb"], p["M"]
        ca = self.cross_attn
        L = rc.ctx_len
        if p.get("shared_q"):               # equal rows per sample (shared prefix): one sample's query
            linear(ca.q, h[:S], q[:S], ws)
            K.rmsnorm_rope(q[:S], ca.norm_q.weight, eps)
            q.view(nb, S, D)[1:].copy_(q[:S].unsqueeze(0).expand(nb - 1, S, D))
        else:
            linear(ca.q, p.pop("h3", h), q, ws)
            K.rmsnorm_rope(q, ca.norm_q.weight, eps)
        kv = fused_linear(ca, p["ctx"], ws, "kvc" + p["tag"])
        if kv is not None:
            kc, vc = kv[:, :D], kv[:, D:]
        else:
            kc, vc = ws.get("kc" + p["tag"], (nb * L, D)), ws.get("vc" + p["tag"], (nb * L, D))
            linear(ca.k, p["ctx"], kc, ws)
            linear(ca.v, p["ctx"], vc, ws)
        K.rmsnorm_rope(kc, ca.norm_k.weight, eps)
        K.attention(q, kc, vc, o, self.num_heads, nb)
        if _fusable_lt(ca.o, M, K.VS_EPI_RES):
            y = ws.get("res_y" + p["tag"], (M, D))
            linear(ca.o, o, y, ws)
            K.residual_layernorm(y, x, h, eps, epilogue=K.VS_EPI_RES, alpha=1.0, shift=mod[:, 3], scale=mod[:, 4],
                                 mod_bstride=6 * D, rows_per_batch=S)
        else:
            linear(ca.o, o, x, ws, epilogue=K.VS_EPI_RES, residual=x)
            # --- FFN (wan_video_dit.py:228-229) + VACE hint (wan_video_new.py:1450)
            h = ln_into(x, h, ws, self.ffn[0], eps, shift=mod[:, 3], scale=mod[:, 4], mod_bstride=6 * D,
                        rows_per_batch=S)
        f = ws.get("f" + p["tag"], (M, self.ffn_dim))
        linear(self.ffn[0], h, f, ws, epilogue=K.VS_EPI_GELU)
        if fuse is not None:
            # bf16(f W2^T + b) staged, then x += gate * y (+ hint) and the next consumer's modulated
            # LayerNorm of the new x into h (its LN1 / the head's norm) in one pass
            y = ws.get("res_y" + p["tag"], (M, D))
            linear(self.ffn[2], f, y, ws)
            b0, nb = p["b0"], p["nb"]
            K.residual_layernorm(y, x, h, eps, epilogue=K.VS_EPI_GATE_RES, gate=mod[:, 5], gate_bstride=6 * D,
                                 gate_rows=S, hint=p["hint"], hint_scale=hint_scale,
                                 shift=fuse["shift"][b0:b0 + nb], scale=fuse["scale"][b0:b0 + nb],
                                 mod_bstride=fuse["bstride"], rows_per_batch=S)
        else:
            linear(self.ffn[2], f, x, ws, epilogue=K.VS_EPI_GATE_RES, residual=x,
                   gate=mod[:, 5], gate_bstride=6 * D, rows_per_batch=S, hint=p["hint"], hint_scale=hint_scale)


class Head(nn.Module):
    """wan_video_dit.py:253-269."""

    def __init__(self, dim, out_dim, patch_size, eps, device=None):
        super().__init__()
        self.dim, self.out_dim, self.eps = dim, out_dim, eps
        self.head = Linear(dim, out_dim * math.prod(patch_size), device=device)
        self.modulation = _param(1, 2, dim, device=device)

    def modulation_for(self, t, rc):
        """(modulation + t) [B, 2, D] (:267, per-batch t row) in its workspace buffer."""
        B, D = rc.batch, self.dim
        hm = rc.ws.get("head_mod", (B, 2, D))
        K.mod_add(self.modulation.view(2, D), t, hm, D, 0)
        return hm

    def forward(self, x, t, rc):
        B, S, D, ws = rc.batch, rc.seq, self.dim, rc.ws
        h = ws.get("h", (B * S, D))
        if getattr(rc, "head_ln_done", False):     # fused into the last block's FFN-down epilogue
            rc.head_ln_done = False
        else:
            hm = self.modulation_for(t, rc)
            K.layernorm_modulate(x, h, self.eps, shift=hm[:, 0], scale=hm[:, 1], mod_bstride=2 * D,
                                 rows_per_batch=S)
        out = ws.get("head_out", (B * S, self.head.out_features))
        K.gemm(h, self.head.weight, out, bias=self.head.bias)
        return out


def rope_table(head_dim=128, end=1024, theta=10000.0, device=None):
    """float32 [end, head_dim/2, 2] (cos, sin) of the 3-D RoPE (wan_video_dit.py:75-89), from fp64."""
    def freqs(dim):
        return 1.0 / (theta ** (torch.arange(0, dim, 2)[: dim // 2].double() / dim))
    f = torch.cat([freqs(head_dim - 2 * (head_dim // 3)), freqs(head_dim // 3), freqs(head_dim // 3)])
    ang = torch.outer(torch.arange(end).double(), f)
    tab = torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).float()
    return tab.to(device)


class WanModel(nn.Module):
    """wan_video_dit.py:272-337 (has_image_input=False path used by Wan2.1-VACE / T2V)."""

    def __init__(self, dim, in_dim, ffn_dim, out_dim, text_dim, freq_dim, eps, patch_size, num_heads,
                 num_layers, has_image_input=False, device=None, **kwargs):
        super().__init__()
        if has_image_input:
            raise NotImplementedError("image-conditioned Wan (I2V/FLF2V) is outside the Ditto hot path")
        if dim // num_heads != 128:
            raise NotImplementedError("head_dim must be 128 (all Wan2.1 models)")
        self.dim, self.in_dim, self.ffn_dim, self.out_dim = dim, in_dim, ffn_dim, out_dim
        self.text_dim, self.freq_dim, self.eps, self.num_heads = text_dim, freq_dim, eps, num_heads
        self.patch_size = tuple(patch_size)
        self.has_image_input = False
        self.seperated_timestep = False
        self.require_vae_embedding = True
        self.require_clip_embedding = True
        self.fuse_vae_embedding_in_latents = False
        self.patch_embedding = PatchEmbed(in_dim, dim, device)
        self.text_embedding = Sequential3(Linear(text_dim, dim, device=device), Linear(dim, dim, device=device))
        self.time_embedding = Sequential3(Linear(freq_dim, dim, device=device), Linear(dim, dim, device=device))
        self.time_projection = nn.Module()
        self.time_projection.add_module("1", Linear(dim, 6 * dim, device=device))
        self.blocks = nn.ModuleList([DiTBlock(dim, num_heads, ffn_dim, eps, device) for _ in range(num_layers)])
        self.head = Head(dim, out_dim, patch_size, eps, device)
        self._rope = None

    def rope(self, device):
        if self._rope is None or self._rope.device != torch.device(device):
            self._rope = rope_table(self.dim // self.num_heads, device=device)
        return self._rope

    def time_embed(self, timestep, ws):
        """t [B,D], t_mod [B,6,D] (wan_video_new.py:1351-1352)."""
        B, D = timestep.shape[0], self.dim
        s = ws.get("sinus", (B, self.freq_dim))
        K.time_sinusoid(timestep.contiguous(), s)
        u = ws.get("t_u", (B, D))
        K.gemm(s, self.time_embedding[0].weight, u, epilogue=K.VS_EPI_SILU, bias=self.time_embedding[0].bias)
        t = ws.get("t", (B, D))
        K.gemm(u, self.time_embedding[2].weight, t, bias=self.time_embedding[2].bias)
        st = ws.get("t_silu", (B, D))
        K.gemm(u, self.time_embedding[2].weight, st, epilogue=K.VS_EPI_SILU, bias=self.time_embedding[2].bias)
        tm = ws.get("t_mod", (B, 6 * D))
        proj = getattr(self.time_projection, "1")
        K.gemm(st, proj.weight, tm, bias=proj.bias)
        return t, tm.view(B, 6, D)

    def text_embed(self, context, ws):
        """[B*L, text_dim] -> [B*L, D] (wan_video_dit.py:308-312)."""
        BL = context.shape[0] * context.shape[1]
        c = context.reshape(BL, self.text_dim).contiguous()
        h = ws.get("ctx_h", (BL, self.dim))
        K.gemm(c, self.text_embedding[0].weight, h, epilogue=K.VS_EPI_GELU, bias=self.text_embedding[0].bias)
        out = ws.get("ctx", (BL, self.dim))
        K.gemm(h, self.text_embedding[2].weight, out, bias=self.text_embedding[2].bias)
        return out


class VaceWanAttentionBlock(DiTBlock):
    """wan_video_vace.py:5-24."""

    def __init__(self, dim, num_heads, ffn_dim, eps=1e-6, block_id=0, device=None):
        super().__init__(dim, num_heads, ffn_dim, eps, device)
        self.block_id = block_id
        if block_id == 0:
            self.before_proj = Linear(dim, dim, device=device)
        self.after_proj = Linear(dim, dim, device=device)


class VaceWanModel(nn.Module):
    """wan_video_vace.py:27-87; the hints are computed on the (possibly SP-sharded) token rows."""

    def __init__(self, vace_layers=tuple(range(0, 30, 2)), vace_in_dim=96, patch_size=(1, 2, 2),
                 has_image_input=False, dim=1536, num_heads=12, ffn_dim=8960, eps=1e-6, device=None):
        super().__init__()
        self.vace_layers = tuple(vace_layers)
        self.vace_in_dim = vace_in_dim
        self.vace_layers_mapping = {i: n for n, i in enumerate(self.vace_layers)}
        self.vace_blocks = nn.ModuleList([
            VaceWanAttentionBlock(dim, num_heads, ffn_dim, eps, block_id=i, device=device) for i in self.vace_layers])
        self.vace_patch_embedding = PatchEmbed(vace_in_dim, dim, device)
        self.dim = dim

    def forward(self, x, vace_cols_out, t_mod, rc, shared_prefix=False):
        """x: patch-embedded main tokens [B*S, D]; vace_cols_out: patch-embedded control tokens
        [B*S, D] (overwritten, becomes c).  Returns the list of hint buffers [B*S, D].  shared_prefix:
        every CFG sample's rows of x, of the control tokens and of t_mod are equal (DiTBlock)."""
        ws, D = rc.ws, self.dim
        M = rc.batch * rc.seq
        c = vace_cols_out
        hints = []
        nb = len(self.vace_blocks)
        # with a shared prefix block 0 reads sample 0's rows of c0 alone and overwrites the others
        # after its self-attention half, so before_proj runs on those rows only
        rows = rc.seq if shared_prefix and rc.batch > 1 and host_option("cfg_prefix") else M
        for n, blk in enumerate(self.vace_blocks):
            if n == 0:
                c0 = ws.get("vace_c", (M, D))
                linear(blk.before_proj, c[:rows], c0[:rows], ws, epilogue=K.VS_EPI_RES, residual=x[:rows])
                c = c0
            blk(c, t_mod, rc, nxt=self.vace_blocks[n + 1] if n + 1 < nb else None,
                shared_prefix=shared_prefix and n == 0)
            hint = ws.get(f"vace_hint{n}", (M, D))
            linear(blk.after_proj, c, hint, ws)
            hints.append(hint)
        return hints


def init_random_(module, seed=5, std=0.02):
    """Synthetic on-device init of SURVEY.md §8(d) (used by bench.py / smoke; real checkpoints load
    by name): N(0,std) weights, 0.01*N biases, modulation randn/sqrt(D), norm weights 1+0.1*N."""
    g = torch.Generator(device=next(module.parameters()).device).manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith("modulation"):
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) / p.shape[-1] ** 0.5)
            elif "norm" in name and name.endswith("weight"):
                p.copy_(1 + 0.1 * torch.randn(p.shape, generator=g, device=p.device))
            elif name.endswith("bias"):
                p.copy_(0.01 * torch.randn(p.shape, generator=g, device=p.device))
            else:
                p.normal_(0.0, std, generator=g)
    return module
