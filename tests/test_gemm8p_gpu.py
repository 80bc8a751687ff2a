"""The 256x256 GEMMs (gemm_bf16_tn_8p and gemm_bf16_tn_4w, csrc/gemm.hip) through vs_gemm, forced
onto the 256x256 schedule and each kernel (options gemm_tile=256, gemm_kernel=8 | 4).

Integer-valued operands keep every fp32 sum exact, so every output must equal the exact product
bit for bit (through each epilogue's reference rounding points, oracle/wan_oracle.py) for:
K-tile counts 1..6 (both buffer parities and every prefetch-tail branch of the phase schedule),
partial last row / column tiles, the un-merged LoRA second K phase (layers.py:180-182) and the
split tail (grid larger than the CU count).  Reference linears: wan_video_dit.py:131-134,157-160,
209-210 through AutoWrappedLinear (vram_management/layers.py:173-188)."""
import os

import pytest
import torch

from oracle import wan_oracle as O
from gpu_util import BF16

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["8p", "4w"])
def K(opt, request):
    """Both 256x256 kernels: gemm_bf16_tn_8p and gemm_bf16_tn_4w (option gemm_kernel); the LoRA second
    phase always runs on the 8-phase kernel."""
    opt(gemm_tile=256, gemm_kernel=8 if request.param == "8p" else 4)
    from vstyler import kernels
    return kernels


def ints(*shape, g, lo=-3, hi=4):
    return torch.randint(lo, hi, shape, generator=g, device="cuda").to(BF16)


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 64), (300, 260, 128), (513, 256, 192), (256, 520, 256),
                                    (700, 300, 320), (257, 1000, 384), (1024, 512, 5120), (512, 768, 13824)])
def test_gemm8p_integer_exact(K, M, N, Kd):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + Kd)
    a, w = ints(M, Kd, g=g), ints(N, Kd, g=g)
    w[:, 0] += (torch.arange(N, device="cuda") % 7).to(BF16)      # asymmetric: catches transposes
    b = ints(N, g=g, lo=-8, hi=9)
    out = torch.full((M, N), 7.0, dtype=BF16, device="cuda")
    K.gemm(a, w, out, bias=b)
    ref = (a.float() @ w.float().t() + b.float()).to(BF16)
    assert torch.equal(out, ref)


def test_gemm8p_epilogues_exact(K):
    M, N, Kd, S = 600, 520, 448, 300
    g = torch.Generator(device="cuda").manual_seed(3)
    a, w, b = ints(M, Kd, g=g), ints(N, Kd, g=g), ints(N, g=g, lo=-8, hi=9)
    y = (a.float() @ w.float().t() + b.float()).to(BF16).cpu()
    res = torch.randn(M, N, generator=torch.Generator().manual_seed(4)).to(BF16)
    gate = (0.25 * torch.randn(2, N, generator=torch.Generator().manual_seed(5))).to(BF16)
    hint = torch.randn(M, N, generator=torch.Generator().manual_seed(6)).to(BF16)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
    # GELU: the kernel's sigma form vs torch's tanh form differ by <= 1 ulp on the cancellation zone
    ref = O.gelu_tanh(y)
    d = (out.cpu().float() - ref.float()).abs()
    assert (d <= ref.float().abs() * 2 ** -7 + 1e-6).all()
    x = res.cuda()
    K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate.cuda(), gate_bstride=N,
           rows_per_batch=S, hint=hint.cuda(), hint_scale=0.5)
    ref = torch.cat([O.gate_residual(res[:S], gate[0], y[:S]), O.gate_residual(res[S:], gate[1], y[S:])])
    ref = O.add(ref, O.bf(hint.float() * 0.5))
    assert torch.equal(x.cpu(), ref)
    x = res.cuda()
    K.gemm(a, w, x, epilogue=K.VS_EPI_RES, bias=b, residual=x, alpha=0.125)
    assert torch.equal(x.cpu(), O.add(res, O.bf(0.125 * y.float())))


@pytest.mark.parametrize("Kd,r", [(256, 64), (320, 128), (5120, 128)])
def test_gemm8p_lora_second_phase_exact(K, Kd, r):
    M, N = 520, 384
    g = torch.Generator(device="cuda").manual_seed(Kd + r)
    x, w, b = ints(M, Kd, g=g), ints(N, Kd, g=g), ints(N, g=g, lo=-8, hi=9)
    t, lb = ints(M, r, g=g, lo=-2, hi=3), ints(N, r, g=g, lo=-2, hi=3)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(x, w, out, bias=b, a2=t, w2=lb)
    ref = (x.float() @ w.float().t() + t.float() @ lb.float().t() + b.float()).to(BF16)
    assert torch.equal(out, ref)


def test_gemm8p_split_tail_exact(K, opt):
    """272 tiles on 256 CUs: 256 whole tiles + 16 tail tiles as K pieces, summed by the combine."""
    M, N, Kd = 4352, 4096, 4096
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = torch.Generator(device="cuda").manual_seed(9)
    a, w, b = ints(M, Kd, g=g), ints(N, Kd, g=g), ints(N, g=g, lo=-8, hi=9)
    res = torch.randn(M, N, device="cuda", generator=g).to(BF16)
    gate = (0.25 * torch.randn(2, N, device="cuda", generator=g)).to(BF16)
    outs = {}
    for split in (True, False):
        opt(gemm_split=1 if split else 0)
        y = torch.empty(M, N, dtype=BF16, device="cuda")
        K.gemm(a, w, y, bias=b)
        x = res.clone()
        K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate, gate_bstride=N,
               rows_per_batch=M // 2, hint=res, hint_scale=0.5)
        outs[split] = (y, x)
    opt(gemm_split=1)
    assert torch.equal(outs[True][0], (a.float() @ w.float().t() + b.float()).to(BF16))
    for s_, u_ in zip(outs[True], outs[False]):
        assert torch.equal(s_, u_)
    if cus == 256:
        assert K.gemm_split_plan(M, N, Kd, cus)[1] == 16


def test_gemm8p_random_vs_fp32(K):
    M, N, Kd = 2000, 1536, 5120
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.randn(M, Kd, device="cuda", generator=g).to(BF16)
    w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(BF16)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a, w, out)
    ref = a.float() @ w.float().t()
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 4e-3, rel


@pytest.mark.parametrize("kern", ["8p", "4w"])
@pytest.mark.parametrize("M,N,Kd", [(256, 256, 128), (300, 520, 256), (1000, 768, 640), (520, 300, 5120),
                                    (512, 512, 384)])
def test_gemm_fp8_8p_integer_exact(M, N, Kd, kern, opt):
    """gemm_fp8_tn_8p / gemm_fp8_tn_4w (option gemm_kernel): integer operands exact in e4m3 with exact fp32 sums
    must reproduce oracle.fp8_linear (layers.py:115-151) bit for bit: pins the MX 32x32x64 operand
    maps, the fp8 chunk swizzle and the per-row scale."""
    from vstyler import kernels as K
    opt(gemm_kernel=8 if kern == "8p" else 4)
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
    x[::5] *= 512          # rows whose max exceeds 448: scale 2**k > 1
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    w[:, 0] += (torch.arange(N) % 5).to(BF16)
    b = torch.randint(-8, 9, (N,), generator=g).to(BF16)
    ref = O.fp8_linear(x, w, b)
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm_fp8(x8, sc, w.to(torch.float8_e4m3fn).view(torch.uint8).cuda(), out, bias=b.cuda())
    assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("kern", ["8p", "4w"])
def test_gemm_fp8_8p_split_tail_and_epilogue(kern, opt):
    """272 tiles: the split-tail pieces + combine (per-row scale applied after the sum) equal the
    unsplit kernel on integer data; gate-residual + hint epilogue bit-exact vs the oracle."""
    from vstyler import kernels as K
    opt(gemm_kernel=8 if kern == "8p" else 4)
    M, N, Kd, S = 4352, 4096, 1024, 2176
    g = torch.Generator().manual_seed(21)
    x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    b = torch.randint(-8, 9, (N,), generator=g).to(BF16)
    res = torch.randn(M, N, generator=g).to(BF16)
    gate = (0.25 * torch.randn(2, N, generator=g)).to(BF16)
    hint = torch.randn(M, N, generator=g).to(BF16)
    y = O.fp8_linear(x, w, b)
    ref = torch.cat([O.gate_residual(res[:S], gate[0], y[:S]), O.gate_residual(res[S:], gate[1], y[S:])])
    ref = O.add(ref, O.bf(hint.float() * 0.5))
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    w8 = w.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    outs = []
    for split in (True, False):
        opt(gemm_split=1 if split else 0)
        xo = res.cuda()
        K.gemm_fp8(x8, sc, w8, xo, epilogue=K.VS_EPI_GATE_RES, bias=b.cuda(), residual=xo, gate=gate.cuda(),
                   gate_bstride=N, rows_per_batch=S, hint=hint.cuda(), hint_scale=0.5)
        outs.append(xo.cpu())
    opt(gemm_split=1)
    assert torch.equal(outs[0], ref) and torch.equal(outs[1], ref)


def test_gemm_persistent_ragged_exact(K):
    """The persistent walk with ragged edges: 17 x 17 = 289 tiles of a 4100 x 4104 output (rows and
    columns past the matrix in the last tile row / column, dropped by the buffer range checks), 256
    persistent workgroups + the rest as whole tiles or split pieces; every epilogue mode bit-exact
    vs the oracle (the 8-phase kernel runs the same shapes under its own parametrisation)."""
    M, N, Kd, S = 4100, 4104, 1024, 2050
    g = torch.Generator(device="cuda").manual_seed(41)
    a, w, b = ints(M, Kd, g=g), ints(N, Kd, g=g), ints(N, g=g, lo=-8, hi=9)
    y = (a.float() @ w.float().t() + b.float()).to(BF16)
    out = torch.full((M, N), 7.0, dtype=BF16, device="cuda")
    K.gemm(a, w, out, bias=b)
    assert torch.equal(out, y)
    res = torch.randn(M, N, generator=torch.Generator().manual_seed(42)).to(BF16)
    gate = (0.25 * torch.randn(2, N, generator=torch.Generator().manual_seed(43))).to(BF16)
    hint = torch.randn(M, N, generator=torch.Generator().manual_seed(44)).to(BF16)
    x = res.cuda()
    K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate.cuda(), gate_bstride=N,
           rows_per_batch=S, hint=hint.cuda(), hint_scale=0.5)
    yc = y.cpu()
    ref = torch.cat([O.gate_residual(res[:S], gate[0], yc[:S]), O.gate_residual(res[S:], gate[1], yc[S:])])
    assert torch.equal(x.cpu(), O.add(ref, O.bf(hint.float() * 0.5)))
    x = res.cuda()
    K.gemm(a, w, x, epilogue=K.VS_EPI_RES, bias=b, residual=x, alpha=0.125)
    assert torch.equal(x.cpu(), O.add(res, O.bf(0.125 * yc.float())))


@pytest.mark.parametrize("kern", ["8p", "4w"])
def test_gemm_fp8_persistent_ragged_exact(kern, opt):
    """The fp8 kernels' persistent walk with ragged edges (289 tiles of 4100 x 4104): integer
    operands exact in e4m3 reproduce oracle.fp8_linear bit for bit."""
    from vstyler import kernels as K
    opt(gemm_kernel=8 if kern == "8p" else 4)
    M, N, Kd = 4100, 4104, 1024
    g = torch.Generator().manual_seed(45)
    x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
    x[::7] *= 512
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    b = torch.randint(-8, 9, (N,), generator=g).to(BF16)
    ref = O.fp8_linear(x, w, b)
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm_fp8(x8, sc, w.to(torch.float8_e4m3fn).view(torch.uint8).cuda(), out, bias=b.cuda())
    assert torch.equal(out.cpu(), ref)
