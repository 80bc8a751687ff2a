"""UMT5-XXL text encoder on gfx950 (replaces diffsynth/models/wan_video_text_encoder.py and the
encode path of diffsynth/prompters/wan_prompter.py).

Per block: T5 RMS norm (vs_rmsnorm_rope, no RoPE), q/k/v/o and gate/fc1/fc2 as vs_gemm (no bias,
residual adds fused as the VS_EPI_RES epilogue), per-head scores / PV as the batched-GEMM mode of
vs_vae_conv (head_dim 64, no 1/sqrt(d) scaling: T5 :80), the relative-position bias + padding mask +
softmax in one pass (vs_t5_bias_softmax, bucket table computed on the host exactly as the
reference), the gated tanh-GELU product in bf16 op order (vs_t5_gelu_mul).  Parameters load by the
reference's state-dict names (registry md5 9c8818c2..., configs/model_config.py:161).
"""
import math

import torch

from . import _lib
from . import kernels as K
from .vae import batched_gemm

BF16 = torch.bfloat16


def relative_position_bucket(lq, lk, num_buckets=32, max_dist=128):
    """T5RelativeEmbedding._relative_position_bucket (wan_video_text_encoder.py:166-188), bidirectional
    -- host integer/fp32 arithmetic identical to the reference, computed once per length."""
    rel_pos = torch.arange(lk).unsqueeze(0) - torch.arange(lq).unsqueeze(1)
    nb = num_buckets // 2
    rel_buckets = (rel_pos > 0).long() * nb
    rel_pos = torch.abs(rel_pos)
    max_exact = nb // 2
    large = max_exact + (torch.log(rel_pos.float() / max_exact) / math.log(max_dist / max_exact) *
                         (nb - max_exact)).long()
    large = torch.min(large, torch.full_like(large, nb - 1))
    return rel_buckets + torch.where(rel_pos < max_exact, rel_pos, large)


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


class WanTextEncoder:
    """WanTextEncoder (wan_video_text_encoder.py:209-252), shared_pos=False."""

    def __init__(self, vocab=256384, dim=4096, dim_attn=4096, dim_ffn=10240, num_heads=64, num_layers=24,
                 num_buckets=32, eps=1e-6, device="cuda"):
        if dim_attn // num_heads != 64 or dim_attn % num_heads:
            raise NotImplementedError("UMT5 head_dim 64 only")
        self.vocab, self.dim, self.dim_attn, self.dim_ffn = vocab, dim, dim_attn, dim_ffn
        self.num_heads, self.num_layers, self.num_buckets, self.eps = num_heads, num_layers, num_buckets, eps
        self.device = torch.device(device)
        self.w = {}
        self._buckets = {}

    def load_state_dict(self, sd):
        self.w = {k: v.detach().to(device=self.device, dtype=BF16).contiguous() for k, v in sd.items()}
        return self

    def state_dict_shapes(self):
        d, da, df, n = self.dim, self.dim_attn, self.dim_ffn, self.num_heads
        out = {"token_embedding.weight": (self.vocab, d), "norm.weight": (d,)}
        for i in range(self.num_layers):
            p = f"blocks.{i}."
            out.update({p + "norm1.weight": (d,), p + "attn.q.weight": (da, d), p + "attn.k.weight": (da, d),
                        p + "attn.v.weight": (da, d), p + "attn.o.weight": (d, da), p + "norm2.weight": (d,),
                        p + "ffn.gate.0.weight": (df, d), p + "ffn.fc1.weight": (df, d),
                        p + "ffn.fc2.weight": (d, df), p + "pos_embedding.embedding.weight": (self.num_buckets, n)})
        return out

    def init_random_(self, seed=8):
        """Synthetic on-device weights (bench): N(0, 1/fan_in) matrices, N(0,1) embeddings, norms 1+0.1*N."""
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.w = {}
        for name, shape in self.state_dict_shapes().items():
            if name.endswith("norm1.weight") or name.endswith("norm2.weight") or name == "norm.weight":
                t = 1.0 + 0.1 * torch.randn(shape, generator=g, device=self.device)
            elif "embedding" in name:
                t = torch.randn(shape, generator=g, device=self.device) * (0.5 if "pos_" in name else 1.0)
            else:
                t = torch.randn(shape, generator=g, device=self.device) / math.sqrt(shape[1])
            self.w[name] = t.to(BF16)
        return self

    def _bucket_table(self, L):
        if L not in self._buckets:
            self._buckets[L] = relative_position_bucket(L, L, self.num_buckets).to(torch.int32).to(self.device)
        return self._buckets[L]

    def _norm(self, x, w, out):
        out.copy_(x)
        return K.rmsnorm_rope(out, w, self.eps)

    def forward(self, ids, mask):
        """ids int64 [B, L], mask [B, L] (1 token / 0 padding) -> [B, L, dim] bf16 (before the
        prompter's zeroing of padded rows)."""
        lib = _lib.load()
        ids = ids.to(device=self.device, dtype=torch.long).contiguous()
        if int(ids.min()) < 0 or int(ids.max()) >= self.vocab:
            raise ValueError("token id out of range")
        B, L = ids.shape
        D, N, hd = self.dim, self.num_heads, self.dim_attn // self.num_heads
        M = B * L
        Lp = (L + 31) // 32 * 32
        dev = self.device
        st = _stream(ids)
        emb = self.w["token_embedding.weight"]
        x = torch.empty((M, D), dtype=BF16, device=dev)
        _lib.check(lib.vs_embed_rows(ids.data_ptr(), emb.data_ptr(), emb.stride(0), emb.shape[0], x.data_ptr(),
                                     D, M, D, st))
        keymask = (mask.to(dev) != 0).to(torch.int32).contiguous()
        buckets = self._bucket_table(L)
        h = torch.empty_like(x)
        q = torch.empty((M, self.dim_attn), dtype=BF16, device=dev)
        k, v, o = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
        s = torch.empty((N, L, Lp), dtype=torch.float32, device=dev)
        p = torch.empty((N, L, Lp), dtype=BF16, device=dev)
        vt = torch.empty((N, hd, Lp), dtype=BF16, device=dev)
        f1 = torch.empty((M, self.dim_ffn), dtype=BF16, device=dev)
        g = torch.empty_like(f1)
        for i in range(self.num_layers):
            pre = f"blocks.{i}."
            W = lambda n: self.w[pre + n]  # noqa: E731
            self._norm(x, W("norm1.weight"), h)
            K.gemm(h, W("attn.q.weight"), q)
            K.gemm(h, W("attn.k.weight"), k)
            K.gemm(h, W("attn.v.weight"), v)
            pos = W("pos_embedding.embedding.weight")
            for b in range(B):
                qb, kb, vb, ob = (t[b * L:(b + 1) * L] for t in (q, k, v, o))
                da = self.dim_attn
                # scores per head z: A = q rows (head z = columns 64z..), B = k rows, fp32, no scaling
                batched_gemm(qb, hd, da, L, hd, kb, hd, da, L, s, L * Lp, Lp, N, out_f32=True, alpha=1.0)
                _lib.check(lib.vs_t5_bias_softmax(s.data_ptr(), L * Lp, Lp, p.data_ptr(), L * Lp, Lp,
                                                  buckets.data_ptr(), pos.data_ptr(), N, 0,
                                                  keymask[b].data_ptr(), L, N, st))
                _lib.check(lib.vs_vae_transpose(vb.data_ptr(), hd, da, vt.data_ptr(), hd * Lp, Lp, N, L, hd, st))
                batched_gemm(p, L * Lp, Lp, L, Lp, vt, hd * Lp, Lp, hd, ob, hd, da, N)
            K.gemm(o, W("attn.o.weight"), x, epilogue=K.VS_EPI_RES, residual=x)
            self._norm(x, W("norm2.weight"), h)
            K.gemm(h, W("ffn.fc1.weight"), f1)
            K.gemm(h, W("ffn.gate.0.weight"), g)
            _lib.check(lib.vs_t5_gelu_mul(f1.data_ptr(), g.data_ptr(), f1.data_ptr(), f1.numel(), st))
            K.gemm(f1, W("ffn.fc2.weight"), x, epilogue=K.VS_EPI_RES, residual=x)
        K.rmsnorm_rope(x, self.w["norm.weight"], self.eps)
        return x.view(B, L, D)

    __call__ = forward


class WanPrompter:
    """WanPrompter (diffsynth/prompters/wan_prompter.py:84-109): tokenizer on the host (a local
    google/umt5-xxl tokenizer directory; no download), encoder on the GPU."""

    def __init__(self, tokenizer_path=None, text_len=512):
        self.text_len = text_len
        self.text_encoder = None
        self.tokenizer = None
        if tokenizer_path is not None:
            from transformers import AutoTokenizer
            self.tokenizer = AutoTokenizer.from_pretrained(tokenizer_path)

    def fetch_models(self, text_encoder=None):
        self.text_encoder = text_encoder

    def tokenize(self, prompt):
        """HuggingfaceTokenizer(seq_len=text_len, clean='whitespace') (wan_prompter.py:33-70)."""
        if self.tokenizer is None:
            raise RuntimeError("no local tokenizer: pass token ids to encode_ids()")
        import re
        text = re.sub(r"\s+", " ", prompt).strip()
        out = self.tokenizer([text], padding="max_length", truncation=True, max_length=self.text_len,
                             add_special_tokens=True, return_attention_mask=True, return_tensors="pt")
        return out.input_ids, out.attention_mask

    def encode_ids(self, ids, mask):
        """encode_prompt after tokenisation (:98-109): encoder output with padded rows zeroed (the
        reference zeroes rows >= every sequence's length in every batch entry)."""
        emb = self.text_encoder(ids, mask)
        for n in mask.gt(0).sum(dim=1).long().tolist():
            emb[:, n:] = 0
        return emb

    def encode_prompt(self, prompt, positive=True, device="cuda"):
        ids, mask = self.tokenize(prompt)
        return self.encode_ids(ids, mask)
