"""GPU parity of the fp8 path (config 5) against the oracle's restatement of
AutoWrappedLinear.fp8_linear (diffsynth/vram_management/layers.py:115-151).

Quantisation: bit-exact (scale and every e4m3 byte).  GEMM: bit-exact on integer-valued operands
(exact fp32 sums: pins the MFMA operand layout), and on random data within the bf16 rounding of a
differently ordered fp32 sum.  Model: tiny DiT+VACE with fp8 block linears vs the oracle with
FP8_BLOCK_LINEARS, within 1.5x the oracle's own fp32-vs-fp64 noise floor."""
import pytest
import torch

from gpu_util import err
from oracle import wan_oracle as O

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _k():
    from vstyler import kernels as K
    return K


@pytest.mark.parametrize("cols", [640, 5120, 13824, 16384, 20000])   # wave per row (<= 4 / 12 chunks), block per row, two-pass
def test_quant_fp8_rows_bit_exact(cols):
    K = _k()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(300, cols, generator=g)
    x[::3] *= 1000.0           # rows with max > 448: scale > 1
    x[1::7] *= 1e-3            # e4m3 subnormal range
    x = x.to(BF16)
    ref8, ref_s = O.fp8_quant_rows(x)
    x8 = torch.empty(300, cols, dtype=torch.uint8, device="cuda")
    sc = torch.empty(300, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    assert torch.equal(sc.cpu(), ref_s[:, 0])
    assert torch.equal(x8.cpu(), ref8.view(torch.uint8))


@pytest.mark.parametrize("D", [1536, 5120, 6144])
@pytest.mark.parametrize("mode", ["modulate", "affine"])
def test_layernorm_modulate_fp8_equals_two_passes(D, mode):
    """vs_layernorm_modulate_fp8 == vs_layernorm_modulate then vs_quant_fp8_rows, every byte and scale
    (the config-5 LN1 / LN3 / LN2 feeding fp8 linears, models.ln_into)."""
    K = _k()
    B, S = 2, 333
    g = torch.Generator(device="cuda").manual_seed(D)
    x = (2.0 * torch.randn(B * S, D, device="cuda", generator=g)).to(BF16)
    if mode == "modulate":
        mod = (0.3 * torch.randn(B, 6, D, device="cuda", generator=g)).to(BF16)
        mod[:, 1, :64] = 300.0     # large scales: outputs above 448 (per-row scale > 1)
        ln = dict(shift=mod[:, 0], scale=mod[:, 1], mod_bstride=6 * D, rows_per_batch=S)
    else:
        w = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).to(BF16)
        w[:64] = 300.0
        b = (0.1 * torch.randn(D, device="cuda", generator=g)).to(BF16)
        ln = dict(weight=w, bias=b)
    h = torch.empty(B * S, D, dtype=BF16, device="cuda")
    K.layernorm_modulate(x, h, 1e-6, **ln)
    ref8 = torch.empty(B * S, D, dtype=torch.uint8, device="cuda")
    refs = torch.empty(B * S, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(h, ref8, refs)
    x8 = torch.full((B * S, D), 7, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(B * S, dtype=torch.float32, device="cuda")
    K.layernorm_modulate_fp8(x, x8, sc, 1e-6, **ln)
    assert torch.equal(sc, refs)
    assert torch.equal(x8, ref8)
    assert (refs > 1).any()


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 128), (300, 520, 384), (1000, 768, 640)])   # K % 128 (vstyler.h)
def test_gemm_fp8_integer_exact(M, N, Kd):
    """Integer operands (exact in e4m3, exact fp32 sums) -> the result must match bit for bit."""
    K = _k()
    g = torch.Generator().manual_seed(M + N)
    x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    ref = O.fp8_linear(x, w, None)
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm_fp8(x8, sc, w.to(torch.float8_e4m3fn).view(torch.uint8).cuda(), out)
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("epi", ["bias", "gelu", "gate_res"])
def test_gemm_fp8_random_epilogues(epi):
    K = _k()
    M, N, Kd = 700, 1024, 1536
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, Kd, generator=g).to(BF16)
    w = (0.03 * torch.randn(N, Kd, generator=g)).to(BF16)
    b = (0.1 * torch.randn(N, generator=g)).to(BF16)
    y = O.fp8_linear(x, w, b)
    kw = dict(bias=b.cuda())
    if epi == "gelu":
        ref = O.gelu_tanh(y)
        kw["epilogue"] = K.VS_EPI_GELU
    elif epi == "gate_res":
        res = torch.randn(M, N, generator=g).to(BF16)
        gate = torch.randn(1, N, generator=g).to(BF16)
        ref = O.gate_residual(res, gate, y)
        kw.update(epilogue=K.VS_EPI_GATE_RES, residual=res.cuda(), gate=gate.cuda(), gate_bstride=N)
    else:
        ref = y
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    if epi == "gate_res":
        out.copy_(kw["residual"])
        kw["residual"] = out
    K.gemm_fp8(x8, sc, w.to(torch.float8_e4m3fn).view(torch.uint8).cuda(), out, **kw)
    d = (out.cpu().float() - ref.float()).abs()
    ulp = ref.float().abs().clamp_min(1e-3) * 2.0 ** -7
    assert (d <= 2 * ulp).float().mean().item() > 0.999, d.max().item()
    assert (out.cpu() == ref).float().mean().item() > 0.95


def test_model_fn_fp8_tiny_vs_oracle():
    from test_model_gpu import build
    from vstyler import model_fn_wan_video
    from vstyler.models import quantize_fp8_
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    dit, vace = build(cfg, W)
    assert quantize_fp8_(dit) + quantize_fp8_(vace) == 10 * (cfg["num_layers"] + len(cfg["vace_layers"]))
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([900.0]).to(BF16)
    old, oldacc = O.FP8_BLOCK_LINEARS, O.ACC_DTYPE
    try:
        O.FP8_BLOCK_LINEARS = True
        ref = O.model_fn(W, cfg, lat, t, cp, vc)
        O.ACC_DTYPE = torch.float64
        ref64 = O.model_fn(W, cfg, lat, t, cp, vc)
    finally:
        O.FP8_BLOCK_LINEARS, O.ACC_DTYPE = old, oldacc
    out = model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t.cuda(), context=cp.cuda(),
                             vace_context=vc.cuda())
    fmx, frl = err(ref64, ref)
    mx, rl = err(out, ref)
    print(f"fp8 tiny forward: max-abs {mx:.4g} rel-L2 {rl:.4g} (floor {fmx:.4g} / {frl:.4g})")
    assert rl <= 1.5 * frl + 2e-3 and mx <= 1.5 * fmx + 2e-2


def test_model_fn_fp8_ln_fusion_bit_identical(monkeypatch):
    """The config-5 forward with the LayerNorms writing fp8_linear's quantised activations directly
    (models.ln_into -> vs_layernorm_modulate_fp8) equals the forward with bf16 LN rows + a separate
    quantisation, bit for bit."""
    from test_model_gpu import build
    from vstyler import model_fn_wan_video, models
    from vstyler.models import quantize_fp8_
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=7)
    dit, vace = build(cfg, W)
    quantize_fp8_(dit)
    quantize_fp8_(vace)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    t = torch.tensor([700.0]).to(BF16).cuda()
    run = lambda: model_fn_wan_video(dit, vace=vace, latents=lat.cuda(), timestep=t, context=cp.cuda(),
                                     vace_context=vc.cuda()).clone()
    calls = []
    real = _k().layernorm_modulate_fp8

    def counted(*a, **k):
        calls.append(1)
        return real(*a, **k)
    monkeypatch.setattr(_k(), "layernorm_modulate_fp8", counted)
    fused = run()
    assert calls, "the fused LN -> fp8 path did not run"
    monkeypatch.setattr(models, "_fp8_consumer", lambda target: False)
    plain = run()
    assert torch.equal(fused, plain)


@pytest.mark.parametrize("epi", ["bias", "gelu", "gate_res", "res"])
def test_gemm_fp8_schedules_agree(epi, opt):
    """vs_gemm_fp8's schedules on random data: the 4-wave kernel with the XCD tile queues (default) and
    with the static lists bit-identical (same per-tile summation order), the 8-phase kernel (another
    MFMA shape, another order) within fp32 summation noise -- for every epilogue (r5: the
    vendor-library fp8 route these were compared with is gone)."""
    K = _k()
    M, N, Kd = 12300, 2048, 2560          # 49 x 8 = 392 tiles: the persistent walk + queue
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(M, Kd, device="cuda", generator=g).to(BF16)
    w8 = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(torch.float8_e4m3fn).view(torch.uint8)
    b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(BF16)
    res0 = torch.randn(M, N, device="cuda", generator=g).to(BF16)
    gate = (0.3 * torch.randn(2, N, device="cuda", generator=g)).to(BF16)
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x, x8, sc)
    outs = []
    for o in (dict(gemm_kernel=4, queue=1), dict(gemm_kernel=4, queue=0), dict(gemm_kernel=8)):
        opt(**o)
        out = res0.clone() if epi in ("gate_res", "res") else torch.empty(M, N, dtype=BF16, device="cuda")
        kw = dict(bias=b)
        if epi == "gelu":
            kw["epilogue"] = K.VS_EPI_GELU
        elif epi == "gate_res":
            kw.update(epilogue=K.VS_EPI_GATE_RES, residual=out, gate=gate, gate_bstride=N, rows_per_batch=M // 2)
        elif epi == "res":
            kw.update(epilogue=K.VS_EPI_RES, residual=out, alpha=0.5)
        K.gemm_fp8(x8, sc, w8, out, **kw)
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    rel = ((outs[2].float() - outs[0].float()).norm() / outs[0].float().norm()).item()
    assert rel < 2e-3, rel
