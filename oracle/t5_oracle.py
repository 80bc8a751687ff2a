"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the UMT5-XXL text encoder of the reference
(diffsynth/models/wan_video_text_encoder.py:1-255) and of WanPrompter.encode_prompt's masking
(diffsynth/prompters/wan_prompter.py:98-109), at the bf16 rounding points of a bf16 model: every
tensor op (norm, q/k/v/o, scores, bias add, softmax output, PV, the tanh-GELU's individual ops,
gated product, residual adds) is rounded to bf16 where the reference materialises a bf16 tensor.
Matmuls accumulate in `wan_oracle.ACC_DTYPE`.  Parity: structure pinned by the registry md5
`9c8818c2cbea55eca56c7b447df170da` (configs/model_config.py:161); numerics unpinned.
"""
import math

import torch
import torch.nn.functional as F

from . import wan_oracle as _wo

BF16 = torch.bfloat16

# WanTextEncoder defaults (wan_video_text_encoder.py:209-219)
T5_CONFIG = dict(vocab=256384, dim=4096, dim_attn=4096, dim_ffn=10240, num_heads=64, num_layers=24,
                 num_buckets=32)


def t5_param_shapes(cfg=T5_CONFIG):
    d, da, df, n = cfg["dim"], cfg["dim_attn"], cfg["dim_ffn"], cfg["num_heads"]
    s = {"token_embedding.weight": (cfg["vocab"], d), "norm.weight": (d,)}
    for i in range(cfg["num_layers"]):
        p = f"blocks.{i}."
        s[p + "norm1.weight"] = (d,)
        s[p + "attn.q.weight"] = (da, d)
        s[p + "attn.k.weight"] = (da, d)
        s[p + "attn.v.weight"] = (da, d)
        s[p + "attn.o.weight"] = (d, da)
        s[p + "norm2.weight"] = (d,)
        s[p + "ffn.gate.0.weight"] = (df, d)
        s[p + "ffn.fc1.weight"] = (df, d)
        s[p + "ffn.fc2.weight"] = (d, df)
        s[p + "pos_embedding.embedding.weight"] = (cfg["num_buckets"], n)
    return s


def random_t5_weights(cfg, seed=8):
    """init_weights-like scales (wan_video_text_encoder.py:191-205), bf16."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in t5_param_shapes(cfg).items():
        if name.endswith("norm1.weight") or name.endswith("norm2.weight") or name == "norm.weight":
            t = 1.0 + 0.1 * torch.randn(shape, generator=g)
        elif "pos_embedding" in name:
            t = torch.randn(shape, generator=g) * 0.5
        elif name == "token_embedding.weight":
            t = torch.randn(shape, generator=g)
        else:
            t = torch.randn(shape, generator=g) / math.sqrt(shape[1])
        out[name] = t.to(BF16)
    return out


def _lin(x, w):
    acc = _wo.ACC_DTYPE
    return (x.to(acc) @ w.to(acc).t()).to(BF16)


def t5_layer_norm(x, w, eps=1e-6):
    """T5LayerNorm (:21-35): bf16 x * rsqrt(mean(x.float()^2) + eps) -> bf16 -> * weight (bf16)."""
    y = x * torch.rsqrt(x.float().pow(2).mean(dim=-1, keepdim=True) + eps)
    return w * y.type_as(w)


def gelu_bf16(x):
    """GELU (:15-19) evaluated as the reference's chain of bf16 tensor ops on the GPU: every op in fp32
    opmath, one bf16 rounding per op (torch.pow(x, 3.) = x*x*x in fp32 there; torch's CPU bf16
    kernel would round after each multiply, so the rounding points are written out explicitly)."""
    f = lambda t: t.float()  # noqa: E731
    x3 = (f(x) * f(x) * f(x)).to(BF16)
    t = (0.044715 * f(x3)).to(BF16)
    t = (f(x) + f(t)).to(BF16)
    t = (math.sqrt(2.0 / math.pi) * f(t)).to(BF16)
    t = torch.tanh(f(t)).to(BF16)
    t = (1.0 + f(t)).to(BF16)
    h = (0.5 * f(x)).to(BF16)
    return (f(h) * f(t)).to(BF16)


def relative_position_bucket(lq, lk, num_buckets=32, max_dist=128):
    """T5RelativeEmbedding._relative_position_bucket (:166-188), bidirectional."""
    rel_pos = torch.arange(lk).unsqueeze(0) - torch.arange(lq).unsqueeze(1)
    nb = num_buckets // 2
    rel_buckets = (rel_pos > 0).long() * nb
    rel_pos = torch.abs(rel_pos)
    max_exact = nb // 2
    rel_pos_large = max_exact + (torch.log(rel_pos.float() / max_exact) / math.log(max_dist / max_exact) *
                                 (nb - max_exact)).long()
    rel_pos_large = torch.min(rel_pos_large, torch.full_like(rel_pos_large, nb - 1))
    return rel_buckets + torch.where(rel_pos < max_exact, rel_pos, rel_pos_large)


def t5_attention(x, W, p, mask, buckets, num_heads):
    """T5Attention.forward (:53-87) with the block's own relative-position bias (shared_pos False)."""
    b, L, _ = x.shape
    q = _lin(x, W[p + "attn.q.weight"]).view(b, L, num_heads, -1)
    k = _lin(x, W[p + "attn.k.weight"]).view(b, L, num_heads, -1)
    v = _lin(x, W[p + "attn.v.weight"]).view(b, L, num_heads, -1)
    pos_bias = W[p + "pos_embedding.embedding.weight"][buckets].permute(2, 0, 1).unsqueeze(0)   # [1,N,L,L]
    attn_bias = x.new_zeros(b, num_heads, L, L)
    attn_bias += pos_bias
    attn_bias.masked_fill_(mask.view(b, 1, 1, -1) == 0, torch.finfo(x.dtype).min)
    acc = _wo.ACC_DTYPE
    s = torch.einsum("binc,bjnc->bnij", q.to(acc), k.to(acc)).to(BF16) + attn_bias
    attn = F.softmax(s.float(), dim=-1).type_as(s)
    o = torch.einsum("bnij,bjnc->binc", attn.to(acc), v.to(acc)).to(BF16)
    return _lin(o.reshape(b, L, -1), W[p + "attn.o.weight"])


def t5_encode(ids, mask, W, cfg=T5_CONFIG):
    """WanTextEncoder.forward (:242-252) + WanPrompter.encode_prompt's zeroing (wan_prompter.py:98-109)."""
    x = W["token_embedding.weight"][ids]
    buckets = relative_position_bucket(ids.shape[1], ids.shape[1], cfg["num_buckets"])
    for i in range(cfg["num_layers"]):
        p = f"blocks.{i}."
        x = x + t5_attention(t5_layer_norm(x, W[p + "norm1.weight"]), W, p, mask, buckets, cfg["num_heads"])
        h = t5_layer_norm(x, W[p + "norm2.weight"])
        f = _lin(h, W[p + "ffn.fc1.weight"]) * gelu_bf16(_lin(h, W[p + "ffn.gate.0.weight"]))
        x = x + _lin(f, W[p + "ffn.fc2.weight"])
    x = t5_layer_norm(x, W["norm.weight"])
    for v in mask.gt(0).sum(dim=1).long():
        x[:, v:] = 0
    return x
