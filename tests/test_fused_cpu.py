"""Fused q|k|v (self-attention) and k|v (cross-attention) projections: the Linears' parameters are
row-slice views of one buffer, so loading / merging / init write through and the block runs one
GEMM; anything that breaks the aliasing (rebinding a parameter, a hot-loaded LoRA, mixed fp8)
makes fused_linear fall back to the per-Linear GEMMs.  CPU-only (no kernels run)."""
import torch
import torch.nn as nn

from vstyler.models import DiTBlock, _fused_views

BF16 = torch.bfloat16


def _block():
    blk = DiTBlock(256, 2, 512, device="cpu")
    g = torch.Generator().manual_seed(3)
    sd = {k: torch.randn(v.shape, generator=g).to(BF16) for k, v in blk.state_dict().items()}
    blk.load_state_dict(sd)
    return blk, sd


def test_fused_views_alias_loaded_weights():
    blk, sd = _block()
    for att, names in ((blk.self_attn, ("q", "k", "v")), (blk.cross_attn, ("k", "v"))):
        f = _fused_views(att)
        assert f is not None
        W, b, W8 = f
        assert W8 is None
        for i, n in enumerate(names):
            pre = "self_attn." if att is blk.self_attn else "cross_attn."
            assert torch.equal(W[i * 256:(i + 1) * 256], sd[pre + n + ".weight"])
            assert torch.equal(b[i * 256:(i + 1) * 256], sd[pre + n + ".bias"])
    # the reference key layout is unchanged (no extra parameters or buffers)
    assert set(blk.state_dict()) == set(sd)


def test_in_place_updates_write_through():
    blk, _ = _block()
    with torch.no_grad():
        blk.self_attn.k.weight.add_(1.0)            # e.g. a LoRA merge writes in place
    W = _fused_views(blk.self_attn)[0]
    assert torch.equal(W[256:512], blk.self_attn.k.weight)


def test_fallback_when_aliasing_breaks():
    blk, _ = _block()
    blk.self_attn.v.weight = nn.Parameter(blk.self_attn.v.weight.detach().clone(), requires_grad=False)
    assert _fused_views(blk.self_attn) is None
    assert _fused_views(blk.cross_attn) is not None
    blk2, _ = _block()
    blk2.cross_attn.k.lora_A = torch.zeros(32, 256, dtype=BF16)     # hot-loaded LoRA
    assert _fused_views(blk2.cross_attn) is None
    blk3, _ = _block()
    blk3.self_attn.q.weight_fp8 = torch.zeros(256, 256, dtype=torch.uint8)   # fp8 on one Linear only
    assert _fused_views(blk3.self_attn) is None


def test_quantize_fp8_keeps_fusion():
    from vstyler.models import quantize_fp8_
    blk, _ = _block()
    assert quantize_fp8_(blk) == 10
    W, b, W8 = _fused_views(blk.self_attn)
    assert W8 is not None and W8.dtype == torch.uint8 and W8.shape == (768, 256)
    assert torch.equal(W8[256:512], blk.self_attn.k.weight_fp8)
    ref = blk.self_attn.k.weight.detach().to(torch.float8_e4m3fn).view(torch.uint8)
    assert torch.equal(blk.self_attn.k.weight_fp8, ref)


def test_fp8_row_scale_rounds_quotient_to_bf16():
    """fp8_linear (layers.py:130-134) divides and clamps the bf16 row max: the scale is
    bf16(max|x| / 448) clamped at 1, not the fp32 quotient."""
    from oracle import wan_oracle as O
    x = torch.zeros(3, 64, dtype=BF16)
    x[0, 5] = 1000.0      # 1000 / 448 = 2.2321...: bf16 2.234375
    x[1, 7] = -3000.0     # 6.6964... -> bf16 6.71875
    x[2, 1] = 100.0       # below 448: clamp to 1
    _, s = O.fp8_quant_rows(x)
    assert s.dtype == torch.float32
    assert torch.equal(s.view(-1), torch.tensor([2.234375, 6.71875, 1.0]))
    assert s[0].item() != 1000.0 / 448.0


def test_hotload_refuses_fp8_layers_atomically():
    """hotload_lora on a model with an fp8 layer raises before touching ANY module:
    the bf16 layer listed first keeps no adapter."""
    import pytest
    from vstyler.lora import hotload_lora
    blk, _ = _block()
    blk.cross_attn.o.weight_fp8 = torch.zeros(256, 256, dtype=torch.uint8)
    r = 16
    lora = {}
    for n in ("self_attn.q", "cross_attn.o"):
        lora[f"{n}.lora_A.default.weight"] = torch.ones(r, 256, dtype=BF16)
        lora[f"{n}.lora_B.default.weight"] = torch.ones(256, r, dtype=BF16)
    with pytest.raises(NotImplementedError, match="cross_attn.o"):
        hotload_lora(blk, lora)
    assert getattr(blk.self_attn.q, "lora_A", None) is None
    del blk.cross_attn.o.weight_fp8
    assert hotload_lora(blk, lora) == 2
    assert blk.self_attn.q.lora_A.shape == (64, 256) and blk.cross_attn.o.lora_B.shape == (256, 64)


def test_residual_ln_fusion_follows_the_gemm_route(monkeypatch):
    """models._fusable_lt asks vs_gemm_route_epi for the residual epilogue the unfused path would run:
    the residual + LayerNorm fusion (a staged GEMM output) is taken exactly when that GEMM would run
    as a staged product + epilogue pass -- never with the product library, whose GEMMs all fuse their
    epilogue (r5, include/vstyler.h), so the model never stages an output.  Host-only."""
    from vstyler import kernels as K
    from vstyler.models import _fusable_lt, quantize_fp8_
    o = nn.Linear(5120, 5120, dtype=BF16)              # o-proj / cross-attention o shape
    down = nn.Linear(13824, 5120, dtype=BF16)          # FFN-down
    for M in (59280, 7410):
        for lin, ep in ((o, K.VS_EPI_GATE_RES), (o, K.VS_EPI_RES), (down, K.VS_EPI_GATE_RES)):
            assert _fusable_lt(lin, M, ep) == K.gemm_route(M, lin.out_features, lin.in_features, epilogue=ep)
            assert _fusable_lt(lin, M, ep) is False
    blk, _ = _block()
    quantize_fp8_(blk)
    assert _fusable_lt(blk.self_attn.o, 59280, K.VS_EPI_GATE_RES) is False
