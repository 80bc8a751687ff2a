"""The VAE AttentionBlock's flash kernel (csrc/vae_attention.hip, vs_vae_attention) against a float64
torch softmax attention, and against the fp32-score GEMM route it replaces (vstyler/vae.py
_attn_block(flash=False)).  Reference: diffsynth/models/wan_video_vae.py:304-342 (one head per frame,
F.scaled_dot_product_attention with the default 1/sqrt(C) scale).

Tolerance: the kernel rounds P = softmax to bf16 before P.V (as the GEMM route) and the output to bf16:
relative L2 <= 4e-3, max-abs <= 2 % of the reference's largest magnitude.  Shapes: the Wan2.1 width
C = 384 at the 832x480 latent frame (60 x 104 = 6240 pixels, 195 key tiles), ragged pixel counts
(1, 31, 33, 100: a partial last key tile, query rows past the end), C = 128 / 256, strided qkv rows,
and sharp score distributions (the exact two-pass softmax's max handling)."""
import math

import pytest
import torch

from gpu_util import err

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _run(qkv, nz, rows, c, ld):
    from vstyler import _lib
    lib = _lib.load()
    out = torch.full((nz, rows, c), float("nan"), dtype=BF16, device="cuda")
    _lib.check(lib.vs_vae_attention(qkv.data_ptr(), rows * ld, ld, out.data_ptr(), rows * c, c, nz, rows, c,
                                    torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return out


def _ref(qkv, c):
    q, k, v = (qkv[..., i * c:(i + 1) * c].double() for i in range(3))
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(c), dim=-1)
    return p @ v


def _inputs(nz, rows, c, ld, qscale, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn((nz, rows, ld), generator=g, device="cuda")
    x[..., :c] *= qscale
    return x.to(BF16)


@pytest.mark.parametrize("c,rows,nz,ld_pad,qscale", [
    (384, 6240, 2, 0, 1.0),      # Wan2.1 middle width at the 832x480 latent frame
    (384, 100, 3, 0, 1.0),
    (384, 33, 2, 64, 4.0),
    (384, 1, 2, 0, 1.0),
    (256, 31, 2, 8, 1.0),
    (128, 1000, 2, 0, 1.0),
    (128, 257, 1, 0, 16.0),      # near one-hot rows
])
def test_vae_attention_vs_float64(c, rows, nz, ld_pad, qscale):
    ld = 3 * c + ld_pad
    qkv = _inputs(nz, rows, c, ld, qscale, seed=c + rows)
    got = _run(qkv, nz, rows, c, ld)
    ref = _ref(qkv[..., :3 * c], c)
    assert torch.isfinite(got.float()).all()
    mx, rel = err(got, ref)
    assert rel <= 4e-3 and mx <= 2e-2 * ref.abs().max().item(), (c, rows, mx, rel)


def test_vae_attention_block_flash_vs_gemm_route():
    """The whole AttentionBlock (RMS norm, to_qkv, attention, proj + residual) through the flash kernel
    and through the r1-r6 GEMM route at the Wan2.1 width on a 2-frame 24 x 40 latent."""
    from vstyler import vae
    c = 384
    g = torch.Generator().manual_seed(11)
    m = vae.WanVideoVAE(device="cuda")
    m.params = {"a.norm.gamma": (1 + 0.1 * torch.randn((c,), generator=g)).to(BF16).cuda()}
    w_qkv = (torch.randn((3 * c, c, 1, 1), generator=g) / math.sqrt(c)).to(BF16)
    b_qkv = (0.1 * torch.randn((3 * c,), generator=g)).to(BF16)
    w_o = (torch.randn((c, c, 1, 1), generator=g) / math.sqrt(c)).to(BF16)
    b_o = (0.1 * torch.randn((c,), generator=g)).to(BF16)
    m.cw = {"a.to_qkv.": vae.ConvW(w_qkv, b_qkv, "cuda"), "a.proj.": vae.ConvW(w_o, b_o, "cuda")}
    x = torch.randn((1, 2, 24, 40, c), generator=g).to(BF16).cuda()
    flash = m._attn_block(x, "a.", flash=True)
    gemm = m._attn_block(x, "a.", flash=False)
    torch.cuda.synchronize()
    mx, rel = err(flash, gemm)
    assert rel <= 2e-3 and mx <= 6e-2, (mx, rel)
