"""TEST INFRASTRUCTURE ONLY -- from-scratch PyTorch-CPU restatement of the Wan2.1(-VACE)
denoising path of the reference (Ditto on DiffSynth-Studio 1.1.8).

Every function cites the reference file:line whose semantics it restates (paths relative to
the reference root, `diffsynth/...`).  Arithmetic is fp32 (fp64 where the reference uses fp64)
with bf16 rounding at exactly the points where the reference's bf16 tensors are materialised.
Parity status: numerics "parity unpinned" (see oracle/__init__.py); structure pinned by KATs.

Nothing in `video-styler_amd/` imports this module.
"""
import hashlib
import math

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


# Accumulation dtype of linear()/attention().  fp32 is the oracle; fp64 is used only to measure the
# intrinsic bf16 noise floor of the computation (two valid orders of rounding), which sets the
# parity tolerances of the model-level tests (tests/golden/make_golden.py).
ACC_DTYPE = torch.float32


def bf(x):
    """Materialise as bf16 (round-to-nearest-even), the rounding point of a bf16 tensor op."""
    return x.to(BF16)


# --------------------------------------------------------------------------------------
# Model dimension table (models/wan_video_dit.py:509-536, models/wan_video_vace.py:27-48,100-110)
# --------------------------------------------------------------------------------------
WAN_CONFIGS = {
    "1.3B": dict(dim=1536, ffn_dim=8960, num_heads=12, num_layers=30, in_dim=16, out_dim=16,
                 text_dim=4096, freq_dim=256, eps=1e-6, vace_layers=tuple(range(0, 30, 2)), vace_in_dim=96),
    "14B": dict(dim=5120, ffn_dim=13824, num_heads=40, num_layers=40, in_dim=16, out_dim=16,
                text_dim=4096, freq_dim=256, eps=1e-6, vace_layers=tuple(range(0, 40, 5)), vace_in_dim=96),
    # scaled-down shape used by fast tests (head_dim stays 128 like every Wan model)
    "tiny": dict(dim=256, ffn_dim=512, num_heads=2, num_layers=4, in_dim=16, out_dim=16,
                 text_dim=4096, freq_dim=256, eps=1e-6, vace_layers=(0, 2), vace_in_dim=96),
    # eight heads, so Ulysses runs at world 2 / 4 / 8 with heads % world == 0 (the 14B model's 40 heads
    # give 5 per rank at SP = 8; tests/test_sp.py)
    "sp8": dict(dim=1024, ffn_dim=2048, num_heads=8, num_layers=3, in_dim=16, out_dim=16,
                text_dim=4096, freq_dim=256, eps=1e-6, vace_layers=(0, 2), vace_in_dim=96),
}


# --------------------------------------------------------------------------------------
# Flow-matching scheduler  (schedulers/flow_match.py:34-82, pipeline init wan_video_new.py:39)
# --------------------------------------------------------------------------------------
def set_timesteps(num_inference_steps, denoising_strength=1.0, shift=5.0,
                  sigma_min=0.0, sigma_max=1.0, num_train_timesteps=1000):
    """flow_match.py:34-58 with extra_one_step=True, no inverse/exponential/terminal shift."""
    sigma_start = sigma_min + (sigma_max - sigma_min) * denoising_strength
    sigmas = torch.linspace(sigma_start, sigma_min, num_inference_steps + 1)[:-1]
    sigmas = shift * sigmas / (1 + (shift - 1) * sigmas)
    timesteps = sigmas * num_train_timesteps
    return sigmas, timesteps


def euler_delta(sigmas, i):
    """flow_match.py:72-82: (sigma_{i+1} - sigma_i) as an fp32 0-d tensor; sigma_N := 0."""
    sigma = sigmas[i]
    sigma_ = sigmas[i + 1] if i + 1 < len(sigmas) else 0
    return sigma_ - sigma


def cfg_euler(v_pos, v_neg, latents, cfg_scale, dsigma):
    """wan_video_new.py:535 (CFG combine in bf16) + flow_match.py:81 (x + v*dsigma in bf16)."""
    diff = bf(v_pos.float() - v_neg.float())
    v = bf(v_neg.float() + bf(cfg_scale * diff.float()).float())
    upd = bf(v.float() * torch.as_tensor(dsigma, dtype=torch.float32))
    return bf(latents.float() + upd.float())


def generate_noise(shape, seed):
    """utils/__init__.py:117-122: CPU generator, fp32 randn, cast to bf16."""
    g = torch.Generator("cpu").manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float32).to(BF16)


# --------------------------------------------------------------------------------------
# Elementwise pieces of the DiT (models/wan_video_dit.py)
# --------------------------------------------------------------------------------------
def sinusoidal_embedding_1d(dim, position):
    """wan_video_dit.py:68-72: fp64 [cos || sin] of t*10000^(-i/(dim/2)), cast to position dtype."""
    half = dim // 2
    sinusoid = torch.outer(position.to(torch.float64),
                           torch.pow(10000, -torch.arange(half, dtype=torch.float64,
                                                          device=position.device).div(half)))
    x = torch.cat([torch.cos(sinusoid), torch.sin(sinusoid)], dim=1)
    return x.to(position.dtype)


def _freqs_1d(dim, end=1024, theta=10000.0):
    """wan_video_dit.py:83-89 (complex128 polar table)."""
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: (dim // 2)].double() / dim))
    freqs = torch.outer(torch.arange(end), freqs)
    return torch.polar(torch.ones_like(freqs), freqs)


def rope_tables(head_dim=128, end=1024):
    """wan_video_dit.py:75-80: temporal dim = d - 2*(d//3) (44 -> 22 pairs), h/w dims d//3 (42 -> 21)."""
    return (_freqs_1d(head_dim - 2 * (head_dim // 3), end), _freqs_1d(head_dim // 3, end),
            _freqs_1d(head_dim // 3, end))


def rope_freqs(f, h, w, head_dim=128):
    """wan_video_new.py:1392-1396: per-token (S,1,64) complex128, tokens ordered (f,h,w)."""
    tf, th, tw = rope_tables(head_dim)
    return torch.cat([
        tf[:f].view(f, 1, 1, -1).expand(f, h, w, -1),
        th[:h].view(1, h, 1, -1).expand(f, h, w, -1),
        tw[:w].view(1, 1, w, -1).expand(f, h, w, -1),
    ], dim=-1).reshape(f * h * w, 1, -1)


def rope_apply(x, freqs, num_heads):
    """wan_video_dit.py:92-97: interleaved pairs as complex128, multiply, cast back to bf16."""
    b, s, dm = x.shape
    xc = torch.view_as_complex(x.to(torch.float64).reshape(b, s, num_heads, -1, 2))
    out = torch.view_as_real(xc * freqs.to(x.device)).flatten(2)
    return out.to(x.dtype)


def rms_norm(x, weight, eps=1e-6):
    """wan_video_dit.py:100-111: fp32 norm over the full last dim, cast bf16, then * bf16 weight."""
    xf = x.float()
    n = bf(xf * torch.rsqrt(xf.pow(2).mean(dim=-1, keepdim=True) + eps))
    return bf(n.float() * weight.float())


def layer_norm(x, eps=1e-6, weight=None, bias=None):
    """vram_management/layers.py:89-91 (WanAutoCastLayerNorm): layer_norm in fp32, cast to bf16."""
    w = None if weight is None else weight.float()
    b = None if bias is None else bias.float()
    return bf(F.layer_norm(x.float(), (x.shape[-1],), w, b, eps))


def modulate(x, shift, scale):
    """wan_video_dit.py:64-65: x*(1+scale)+shift, every op a bf16 tensor op."""
    s1 = bf(1 + scale.float())
    return bf(bf(x.float() * s1.float()).float() + shift.float())


def gate_residual(x, gate, residual):
    """wan_video_dit.py:193-194 (GateModule): x + gate*residual in bf16."""
    return bf(x.float() + bf(gate.float() * residual.float()).float())


def add(a, b):
    return bf(a.float() + b.float())


def linear(x, w, b=None):
    """nn.Linear in bf16 (wan_video_dit.py:131-134 etc.): fp32 accumulation, + bias, one rounding."""
    y = x.to(ACC_DTYPE) @ w.to(ACC_DTYPE).t()
    if b is not None:
        y = y + b.to(ACC_DTYPE)
    return bf(y)


# fp8 path switch (config 5): when True, every Linear inside a DiT/VACE block runs as
# AutoWrappedLinear.fp8_linear (vram_management/layers.py:115-151); embeddings/head stay bf16.
FP8_BLOCK_LINEARS = False


# Hot-loaded (un-merged) LoRA terms of AutoWrappedLinear (layers.py:180-182): {id(weight): (alpha*A, B)};
# a block linear whose weight is listed runs lora_linear.
HOTLOAD = {}


def blk_linear(x, w, b=None):
    if id(w) in HOTLOAD:
        return lora_linear(x, w, b, *HOTLOAD[id(w)])
    return fp8_linear(x, w, b) if FP8_BLOCK_LINEARS else linear(x, w, b)


def gelu_tanh(x):
    return bf(F.gelu(x.float(), approximate="tanh"))


def silu(x):
    return bf(F.silu(x.float()))


# attention() evaluates the score matrix per (batch, head) and in query-row chunks once it would
# exceed this many elements (production shapes on the GPU: S = 29 640 -> 281 GB at once); the
# per-row arithmetic is the same softmax(q k^T / sqrt(d)) v in ACC_DTYPE either way.
ATTN_CHUNK_ELEMS = 1 << 28


def attention(q, k, v, num_heads):
    """wan_video_dit.py:28-61: softmax(q k^T / sqrt(d)) v, non-causal, no mask; fp32 math."""
    b, sq, dm = q.shape
    d = dm // num_heads
    qh = q.to(ACC_DTYPE).view(b, sq, num_heads, d).transpose(1, 2)
    kh = k.to(ACC_DTYPE).view(b, k.shape[1], num_heads, d).transpose(1, 2)
    vh = v.to(ACC_DTYPE).view(b, v.shape[1], num_heads, d).transpose(1, 2)
    skv = k.shape[1]
    if b * num_heads * sq * skv <= ATTN_CHUNK_ELEMS:
        p = torch.softmax((qh @ kh.transpose(-1, -2)) / math.sqrt(d), dim=-1)
        o = p @ vh
    else:
        o = torch.empty(b, num_heads, sq, d, dtype=ACC_DTYPE, device=q.device)
        rows = max(1, ATTN_CHUNK_ELEMS // skv)
        for i in range(b):
            for h in range(num_heads):
                kt = kh[i, h].transpose(0, 1)
                for r0 in range(0, sq, rows):
                    p = torch.softmax((qh[i, h, r0:r0 + rows] @ kt) / math.sqrt(d), dim=-1)
                    o[i, h, r0:r0 + rows] = p @ vh[i, h]
    return bf(o.transpose(1, 2).reshape(b, sq, dm))


def attention_rows(q, k, v, num_heads, rows):
    """Same as attention() but only for the query rows `rows` (full-size spot checks)."""
    return attention(q[:, rows], k, v, num_heads)


# --------------------------------------------------------------------------------------
# DiT block / head / embeddings (models/wan_video_dit.py)
# --------------------------------------------------------------------------------------
def self_attention(x, freqs, W, p, num_heads, eps=1e-6):
    """SelfAttention.forward, wan_video_dit.py:140-147."""
    q = rms_norm(blk_linear(x, W[p + "q.weight"], W[p + "q.bias"]), W[p + "norm_q.weight"], eps)
    k = rms_norm(blk_linear(x, W[p + "k.weight"], W[p + "k.bias"]), W[p + "norm_k.weight"], eps)
    v = blk_linear(x, W[p + "v.weight"], W[p + "v.bias"])
    q = rope_apply(q, freqs, num_heads)
    k = rope_apply(k, freqs, num_heads)
    o = attention(q, k, v, num_heads)
    return blk_linear(o, W[p + "o.weight"], W[p + "o.bias"])


def cross_attention(x, ctx, W, p, num_heads, eps=1e-6):
    """CrossAttention.forward (has_image_input=False), wan_video_dit.py:171-186."""
    q = rms_norm(blk_linear(x, W[p + "q.weight"], W[p + "q.bias"]), W[p + "norm_q.weight"], eps)
    k = rms_norm(blk_linear(ctx, W[p + "k.weight"], W[p + "k.bias"]), W[p + "norm_k.weight"], eps)
    v = blk_linear(ctx, W[p + "v.weight"], W[p + "v.bias"])
    o = attention(q, k, v, num_heads)
    return blk_linear(o, W[p + "o.weight"], W[p + "o.bias"])


def dit_block(x, ctx, t_mod, freqs, W, p, num_heads, eps=1e-6):
    """DiTBlock.forward, wan_video_dit.py:214-230 (t_mod of shape (B,6,D))."""
    mod = bf(W[p + "modulation"].float() + t_mod.float())          # :218-219, bf16 add
    shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp = mod.chunk(6, dim=1)
    h = modulate(layer_norm(x, eps), shift_msa, scale_msa)        # :225
    x = gate_residual(x, gate_msa, self_attention(h, freqs, W, p + "self_attn.", num_heads, eps))
    h = layer_norm(x, eps, W[p + "norm3.weight"], W[p + "norm3.bias"])
    x = add(x, cross_attention(h, ctx, W, p + "cross_attn.", num_heads, eps))   # :227
    h = modulate(layer_norm(x, eps), shift_mlp, scale_mlp)        # :228
    f = blk_linear(gelu_tanh(blk_linear(h, W[p + "ffn.0.weight"], W[p + "ffn.0.bias"])),
               W[p + "ffn.2.weight"], W[p + "ffn.2.bias"])
    return gate_residual(x, gate_mlp, f)                           # :229


def patchify(lat, weight, bias):
    """Conv3d k=s=(1,2,2) (wan_video_dit.py:306-307,339-345) + rearrange b c f h w -> b (f h w) c
    (wan_video_new.py:1381-1382).  Returns (tokens (B,S,D), (f,h,w))."""
    b, c, f, hh, ww = lat.shape
    h, w = hh // 2, ww // 2
    cols = lat.float().view(b, c, f, h, 2, w, 2).permute(0, 2, 3, 5, 1, 4, 6).reshape(b, f * h * w, c * 4)
    y = cols @ weight.float().reshape(weight.shape[0], c * 4).t() + bias.float()
    return bf(y), (f, h, w)


def head(x, t, W, eps=1e-6):
    """Head.forward, wan_video_dit.py:262-269 (2-D t branch: per-batch shift/scale = mod + t)."""
    mod = W["head.modulation"].float()                                   # (1,2,D)
    shift = bf(mod[:, 0] + t.float()).unsqueeze(1)                       # (B,1,D)
    scale = bf(mod[:, 1] + t.float()).unsqueeze(1)
    return linear(modulate(layer_norm(x, eps), shift, scale), W["head.head.weight"], W["head.head.bias"])


def unpatchify(x, fhw, out_dim=16):
    """wan_video_dit.py:347-352: 'b (f h w) (x y z c) -> b c (f x) (h y) (w z)', patch (1,2,2)."""
    f, h, w = fhw
    b = x.shape[0]
    return x.view(b, f, h, w, 1, 2, 2, out_dim).permute(0, 7, 1, 4, 2, 5, 3, 6).reshape(b, out_dim, f, 2 * h, 2 * w)


def time_embed(timestep, W, dim):
    """wan_video_new.py:1351-1352 / wan_video_dit.py:313-319: t (B,D) and t_mod (B,6,D)."""
    s = sinusoidal_embedding_1d(256, timestep)
    t = linear(silu(linear(s, W["time_embedding.0.weight"], W["time_embedding.0.bias"])),
               W["time_embedding.2.weight"], W["time_embedding.2.bias"])
    t_mod = linear(silu(t), W["time_projection.1.weight"], W["time_projection.1.bias"])
    return t, t_mod.unflatten(1, (6, dim))


def text_embed(context, W):
    """wan_video_dit.py:308-312 applied at wan_video_new.py:1357."""
    h = gelu_tanh(linear(context, W["text_embedding.0.weight"], W["text_embedding.0.bias"]))
    return linear(h, W["text_embedding.2.weight"], W["text_embedding.2.bias"])


def vace_forward(x, vace_context, ctx, t_mod, freqs, W, vace_layers, num_heads, eps=1e-6):
    """VaceWanModel.forward + VaceWanAttentionBlock.forward (models/wan_video_vace.py:13-24,53-87)."""
    c, _ = patchify(vace_context, W["vace_patch_embedding.weight"], W["vace_patch_embedding.bias"])
    hints = []
    for n in range(len(vace_layers)):
        p = f"vace_blocks.{n}."
        if n == 0:
            c = add(linear(c, W[p + "before_proj.weight"], W[p + "before_proj.bias"]), x)
        c = dit_block(c, ctx, t_mod, freqs, W, p, num_heads, eps)
        hints.append(linear(c, W[p + "after_proj.weight"], W[p + "after_proj.bias"]))
    return hints


class TeaCacheOracle:
    """TeaCache, wan_video_new.py:1154-1203 (check / store / update on bf16 CPU tensors)."""
    COEFFICIENTS = {
        "Wan2.1-T2V-1.3B": [-5.21862437e+04, 9.23041404e+03, -5.28275948e+02, 1.36987616e+01, -4.99875664e-02],
        "Wan2.1-T2V-14B": [-3.03318725e+05, 4.90537029e+04, -2.65530556e+03, 5.87365115e+01, -3.15583525e-01],
        "Wan2.1-I2V-14B-480P": [2.57151496e+05, -3.54229917e+04, 1.40286849e+03, -1.35890334e+01, 1.32517977e-01],
        "Wan2.1-I2V-14B-720P": [8.10705460e+03, 2.13393892e+03, -3.72934672e+02, 1.66203073e+01, -4.17769401e-02],
    }

    def __init__(self, num_inference_steps, rel_l1_thresh, model_id):
        self.n, self.thresh, self.coef = num_inference_steps, rel_l1_thresh, self.COEFFICIENTS[model_id]
        self.step, self.acc, self.prev_mod, self.prev_hidden, self.residual = 0, 0, None, None, None
        self.decisions = []

    def check(self, x, t_mod):
        import numpy as np
        mod = t_mod.clone()
        if self.step == 0 or self.step == self.n - 1:
            calc, self.acc = True, 0
        else:
            self.acc += np.poly1d(self.coef)(((mod - self.prev_mod).abs().mean() / self.prev_mod.abs().mean()).item())
            calc = not self.acc < self.thresh
            if calc:
                self.acc = 0
        self.prev_mod = mod
        self.step = (self.step + 1) % self.n
        if calc:
            self.prev_hidden = x.clone()
        self.decisions.append(calc)
        return not calc

    def store(self, x):
        self.residual = x - self.prev_hidden
        self.prev_hidden = None

    def update(self, x):
        return x + self.residual


def model_fn(W, cfg, latents, timestep, context, vace_context=None, vace_scale=1.0, num_layers=None,
             skip_blocks=(), tea_cache=None):
    """model_fn_wan_video, wan_video_new.py:1338-1468 (non-S2V, non-animate, no sliding window,
    no SP; TeaCache as :1398-1402,1418-1419,1455-1456).  `timestep` is the (B,) bf16 tensor of
    wan_video_new.py:526.
    skip_blocks: skip-layer guidance of config 5 (ComfyUI WanVideoSLG, external): the listed main
    blocks -- and the VACE hint added after them -- are skipped."""
    D, H, eps = cfg["dim"], cfg["num_heads"], cfg["eps"]
    L = cfg["num_layers"] if num_layers is None else num_layers
    t, t_mod = time_embed(timestep, W, D)
    ctx = text_embed(context, W)
    x, (f, h, w) = patchify(latents, W["patch_embedding.weight"], W["patch_embedding.bias"])
    freqs = rope_freqs(f, h, w, D // H)
    hints = None
    vmap = {}
    tea_update = tea_cache.check(x, t_mod) if tea_cache is not None else False
    if tea_update:                                                # :1418-1419
        x = tea_cache.update(x)
    else:
        if vace_context is not None:
            hints = vace_forward(x, vace_context, ctx, t_mod, freqs, W, cfg["vace_layers"], H, eps)
            vmap = {layer: n for n, layer in enumerate(cfg["vace_layers"])}
        for i in range(L):
            if i in skip_blocks:
                continue
            x = dit_block(x, ctx, t_mod, freqs, W, f"blocks.{i}.", H, eps)
            if hints is not None and i in vmap:                   # :1445-1450
                x = add(x, bf(hints[vmap[i]].float() * vace_scale))
        if tea_cache is not None:
            tea_cache.store(x)                                    # :1455-1456
    x = head(x, t, W, eps)
    return unpatchify(x, (f, h, w), cfg["out_dim"])


def dit_block_rows(x, ctx, t_mod, freqs, W, p, num_heads, rows, eps=1e-6):
    """dit_block (wan_video_dit.py:214-230) evaluated for the token rows `rows` of x only.  Every op
    of the block is token-local except self-attention's keys / values, which come from every row of
    x (LayerNorm + modulate + k / v projections + k's RMSNorm / RoPE over all S rows); the query rows,
    the output projection, cross-attention, the FFN and both gate-residuals run on `rows` alone.
    Per row the arithmetic is dit_block's, so the result equals dit_block(x, ...)[:, rows]."""
    mod = bf(W[p + "modulation"].float() + t_mod.float())
    shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp = mod.chunk(6, dim=1)
    h = modulate(layer_norm(x, eps), shift_msa, scale_msa)
    a = p + "self_attn."
    hr = h[:, rows]
    q = rope_apply(rms_norm(blk_linear(hr, W[a + "q.weight"], W[a + "q.bias"]), W[a + "norm_q.weight"], eps),
                   freqs[rows.to(freqs.device)], num_heads)
    k = rope_apply(rms_norm(blk_linear(h, W[a + "k.weight"], W[a + "k.bias"]), W[a + "norm_k.weight"], eps),
                   freqs, num_heads)
    v = blk_linear(h, W[a + "v.weight"], W[a + "v.bias"])
    o = blk_linear(attention(q, k, v, num_heads), W[a + "o.weight"], W[a + "o.bias"])
    del h, k, v
    xr = gate_residual(x[:, rows], gate_msa, o)
    hr = layer_norm(xr, eps, W[p + "norm3.weight"], W[p + "norm3.bias"])
    xr = add(xr, cross_attention(hr, ctx, W, p + "cross_attn.", num_heads, eps))
    hr = modulate(layer_norm(xr, eps), shift_mlp, scale_mlp)
    f = blk_linear(gelu_tanh(blk_linear(hr, W[p + "ffn.0.weight"], W[p + "ffn.0.bias"])),
                   W[p + "ffn.2.weight"], W[p + "ffn.2.bias"])
    return gate_residual(xr, gate_mlp, f)


def model_fn_rows(W, cfg, latents, timestep, context, vace_context, rows, vace_scale=1.0):
    """model_fn (wan_video_new.py:1338-1468) of a ONE-block DiT with at most one VACE block, at the
    token rows `rows` only: the head's output tokens (B, len(rows), 4 * out_dim) before unpatchify
    (wan_video_dit.py:347-352).  Full-size parity without the S x S attention of every row: the
    self-attention keys / values still come from all S tokens (dit_block_rows), so at S = 111 600
    (1280x720x121) a few hundred sampled rows cost seconds instead of minutes."""
    D, H, eps = cfg["dim"], cfg["num_heads"], cfg["eps"]
    assert cfg["num_layers"] == 1 and len(cfg["vace_layers"]) <= 1, "model_fn_rows: a one-block pair"
    t, t_mod = time_embed(timestep, W, D)
    ctx = text_embed(context, W)
    x, (f, h, w) = patchify(latents, W["patch_embedding.weight"], W["patch_embedding.bias"])
    freqs = rope_freqs(f, h, w, D // H)
    hint = None
    if vace_context is not None and cfg["vace_layers"]:
        c, _ = patchify(vace_context, W["vace_patch_embedding.weight"], W["vace_patch_embedding.bias"])
        c = add(linear(c, W["vace_blocks.0.before_proj.weight"], W["vace_blocks.0.before_proj.bias"]), x)
        c = dit_block_rows(c, ctx, t_mod, freqs, W, "vace_blocks.0.", H, rows, eps)
        hint = linear(c, W["vace_blocks.0.after_proj.weight"], W["vace_blocks.0.after_proj.bias"])
    xr = dit_block_rows(x, ctx, t_mod, freqs, W, "blocks.0.", H, rows, eps)
    if hint is not None and 0 in cfg["vace_layers"]:
        xr = add(xr, bf(hint.float() * vace_scale))
    return head(xr, t, W, eps)


def patchify_output(out, patch=(1, 2, 2)):
    """The inverse of unpatchify: (B, C, F, 2h, 2w) -> tokens (B, F*h*w, 4*C) in the head's column
    order (x y z c), so product outputs can be compared at token rows."""
    b, c, ff, hh, ww = out.shape
    h, w = hh // patch[1], ww // patch[2]
    return out.view(b, c, ff, 1, h, 2, w, 2).permute(0, 2, 4, 6, 3, 5, 7, 1).reshape(b, ff * h * w, 4 * c)


def denoise(W, cfg, latents, context_pos, context_neg, vace_context=None, num_inference_steps=2,
            cfg_scale=5.0, sigma_shift=5.0, vace_scale=1.0, num_layers=None, tea_caches=None):
    """WanVideoPipeline.__call__ denoise loop, wan_video_new.py:484,515-542 (cfg_merge=False).
    tea_caches: (posi, nega) TeaCacheOracle pair -- one per prompt, as WanVideoUnit_TeaCache."""
    sigmas, timesteps = set_timesteps(num_inference_steps, 1.0, sigma_shift)
    tp, tn = tea_caches if tea_caches is not None else (None, None)
    for i, ts in enumerate(timesteps):
        t = ts.unsqueeze(0).to(BF16).to(latents.device)              # :526
        vp = model_fn(W, cfg, latents, t, context_pos, vace_context, vace_scale, num_layers, tea_cache=tp)
        if cfg_scale != 1.0:
            vn = model_fn(W, cfg, latents, t, context_neg, vace_context, vace_scale, num_layers, tea_cache=tn)
            latents = cfg_euler(vp, vn, latents, cfg_scale, euler_delta(sigmas, i))
        else:
            latents = bf(latents.float() + bf(vp.float() * euler_delta(sigmas, i)).float())
    return latents


# --------------------------------------------------------------------------------------
# fp8 linear (AutoWrappedLinear.fp8_linear, vram_management/layers.py:115-151; e4m3fn, OCP)
# --------------------------------------------------------------------------------------
def fp8_quant_rows(x):
    """layers.py:124-135: scale_a = clamp(rowmax|x| / 448, min=1).float() -- the division and the
    clamp run on the bf16 x_max, so the quotient is rounded to bf16 before the clamp (:130-134) --
    then x8 = (x / (scale_a + 1e-8)) in fp32 (bf16 / fp32 tensors promote), cast to float8_e4m3fn.
    Returns (x8 as float8_e4m3fn, scale_a [M, 1] fp32)."""
    x2 = x.reshape(-1, x.shape[-1])
    x_max = torch.max(torch.abs(x2), dim=-1, keepdim=True).values
    scale_a = torch.clamp(x_max.to(BF16) / 448.0, min=1.0).float()
    x8 = (x2.float() / (scale_a + 1e-8)).to(torch.float8_e4m3fn)
    return x8, scale_a


def fp8_linear(x, w, b):
    """layers.py:115-151 with torch._scaled_mm restated: (x8 . w8^T) * scale_a * 1 + bias in fp32,
    one bf16 rounding.  w is the bf16 weight (cast to e4m3fn, :133) or already e4m3fn."""
    x8, sa = fp8_quant_rows(x)
    w8 = w if w.dtype == torch.float8_e4m3fn else w.to(torch.float8_e4m3fn)
    acc = x8.to(ACC_DTYPE) @ w8.to(ACC_DTYPE).T
    out = acc * sa.to(ACC_DTYPE)
    if b is not None:
        out = out + b.to(ACC_DTYPE)
    return out.to(BF16).reshape(*x.shape[:-1], w.shape[0])


def denoise_unipc(W, cfg, latents, context_pos, context_neg, vace_context=None, vace_scale=1.0, cfg_scale=1.2,
                  num_inference_steps=4, sigma_shift=2.0, slg_blocks=(), slg_range=(0.2, 0.7)):
    """Config 5's sampler chain (ditto_comfyui_workflow.json: WanVideoSampler 4 steps / cfg 1.2 /
    shift 2.0 / unipc, WanVideoSLG): UniPC on fp32 latents (oracle/unipc_oracle.py), model input
    bf16, CFG combined in bf16 as wan_video_new.py:535, SLG on the uncond pass.  The ComfyUI wrapper
    itself is external (not in the reference): parity unpinned."""
    from .unipc_oracle import UniPCOracle
    sched = UniPCOracle(shift=1.0)
    sched.set_timesteps(num_inference_steps, shift=sigma_shift)
    x = latents.float()
    n = len(sched.timesteps)
    for i, t in enumerate(sched.timesteps):
        tb = t.reshape(1).to(BF16)
        lat = x.to(BF16)
        vp = model_fn(W, cfg, lat, tb, context_pos, vace_context, vace_scale)
        if cfg_scale != 1.0:
            skip = tuple(slg_blocks) if slg_range[0] <= i / n <= slg_range[1] else ()
            vn = model_fn(W, cfg, lat, tb, context_neg, vace_context, vace_scale, skip_blocks=skip)
            v = bf(vn.float() + bf(cfg_scale * bf(vp.float() - vn.float()).float()).float())
        else:
            v = vp
        x = sched.step(v.float(), t, x)
    return x.to(BF16)


# --------------------------------------------------------------------------------------
# LoRA merge (lora/__init__.py:11-45) and unmerged hot-load form (vram_management/layers.py:180-182)
# --------------------------------------------------------------------------------------
def lora_merge(weight, lora_up, lora_down, alpha):
    """GeneralLoRALoader.load: W <- W + alpha*(B@A), every op in bf16."""
    wl = bf(alpha * bf(lora_up.float() @ lora_down.float()).float())
    return bf(weight.float() + wl.float())


def lora_linear(x, w, b, lora_a, lora_b):
    """AutoWrappedLinear hot-load: out + x @ A^T @ B^T (A already scaled by alpha), bf16 ops."""
    out = linear(x, w, b)
    t = bf(x.float() @ lora_a.float().t())
    return bf(out.float() + bf(t.float() @ lora_b.float().t()).float())


# --------------------------------------------------------------------------------------
# Seeded random-init weights with the reference's state-dict layout
# --------------------------------------------------------------------------------------
def dit_param_shapes(cfg):
    """Parameter names/shapes of WanModel (has_image_input=False), wan_video_dit.py:272-337."""
    D, F_, t_dim, f_dim = cfg["dim"], cfg["ffn_dim"], cfg["text_dim"], cfg["freq_dim"]
    s = {
        "patch_embedding.weight": (D, cfg["in_dim"], 1, 2, 2), "patch_embedding.bias": (D,),
        "text_embedding.0.weight": (D, t_dim), "text_embedding.0.bias": (D,),
        "text_embedding.2.weight": (D, D), "text_embedding.2.bias": (D,),
        "time_embedding.0.weight": (D, f_dim), "time_embedding.0.bias": (D,),
        "time_embedding.2.weight": (D, D), "time_embedding.2.bias": (D,),
        "time_projection.1.weight": (6 * D, D), "time_projection.1.bias": (6 * D,),
        "head.head.weight": (cfg["out_dim"] * 4, D), "head.head.bias": (cfg["out_dim"] * 4,),
        "head.modulation": (1, 2, D),
    }
    for i in range(cfg["num_layers"]):
        s.update(block_param_shapes(cfg, f"blocks.{i}."))
    return s


def block_param_shapes(cfg, p):
    D, F_ = cfg["dim"], cfg["ffn_dim"]
    s = {}
    for a in ("self_attn.", "cross_attn."):
        for l in "qkvo":
            s[p + a + l + ".weight"] = (D, D)
            s[p + a + l + ".bias"] = (D,)
        s[p + a + "norm_q.weight"] = (D,)
        s[p + a + "norm_k.weight"] = (D,)
    s[p + "norm3.weight"] = (D,)
    s[p + "norm3.bias"] = (D,)
    s[p + "ffn.0.weight"] = (F_, D)
    s[p + "ffn.0.bias"] = (F_,)
    s[p + "ffn.2.weight"] = (D, F_)
    s[p + "ffn.2.bias"] = (D,)
    s[p + "modulation"] = (1, 6, D)
    return s


def vace_param_shapes(cfg):
    """VaceWanModel parameters, wan_video_vace.py:5-51."""
    D = cfg["dim"]
    s = {"vace_patch_embedding.weight": (D, cfg["vace_in_dim"], 1, 2, 2), "vace_patch_embedding.bias": (D,)}
    for n in range(len(cfg["vace_layers"])):
        p = f"vace_blocks.{n}."
        s.update(block_param_shapes(cfg, p))
        if n == 0:
            s[p + "before_proj.weight"] = (D, D)
            s[p + "before_proj.bias"] = (D,)
        s[p + "after_proj.weight"] = (D, D)
        s[p + "after_proj.bias"] = (D,)
    return s


def hash_state_dict_keys(shapes):
    """models/utils.py:148-182 (convert_state_dict_keys_to_single_str + md5), on {key: shape}."""
    keys = []
    for key, shape in shapes.items():
        keys.append(key + ":" + "_".join(map(str, list(shape))))
        keys.append(key)
    keys.sort()
    return hashlib.md5(",".join(keys).encode("UTF-8")).hexdigest()


def init_weight(name, shape, gen, dim):
    """Synthetic init of SURVEY.md §8(d): N(0,0.02) weights, 0.01*N biases, modulation randn/sqrt(D),
    norm weights 1+0.1*N (so the weight multiply is exercised)."""
    if name.endswith("modulation"):
        return (torch.randn(shape, generator=gen) / dim ** 0.5).to(BF16)
    if "norm" in name and name.endswith("weight"):
        return (1 + 0.1 * torch.randn(shape, generator=gen)).to(BF16)
    if name.endswith("bias"):
        return (0.01 * torch.randn(shape, generator=gen)).to(BF16)
    return (0.02 * torch.randn(shape, generator=gen)).to(BF16)


def random_weights(cfg, seed=5, vace=True, num_layers=None):
    cfg = dict(cfg)
    if num_layers is not None:
        cfg["num_layers"] = num_layers
    shapes = dit_param_shapes(cfg)
    if vace:
        shapes.update(vace_param_shapes(cfg))
    gen = torch.Generator("cpu").manual_seed(seed)
    return {k: init_weight(k, s, gen, cfg["dim"]) for k, s in shapes.items()}


def synthetic_inputs(cfg, frames, height, width, seed_latent=1, batch=1):
    """SURVEY.md §8(d) synthetic inputs: latents seed 1, contexts seeds 2/3, vace_context seed 4."""
    T = (frames - 1) // 4 + 1
    lat = generate_noise((batch, cfg["in_dim"], T, height // 8, width // 8), seed_latent)

    def ctx(seed, n_valid):
        g = torch.Generator("cpu").manual_seed(seed)
        c = 0.1 * torch.randn((batch, 512, cfg["text_dim"]), generator=g)
        c[:, n_valid:] = 0
        return c.to(BF16)

    g = torch.Generator("cpu").manual_seed(4)
    vc = torch.empty((batch, cfg["vace_in_dim"], T, height // 8, width // 8))
    vc[:, :16] = 0.1 * torch.randn((batch, 16, T, height // 8, width // 8), generator=g)
    vc[:, 16:32] = torch.randn((batch, 16, T, height // 8, width // 8), generator=g)
    vc[:, 32:] = 1.0
    return lat, ctx(2, 32), ctx(3, 96), vc.to(BF16)
