"""The persistent 4-wave GEMMs (gemm_bf16_tn_4w, gemm_fp8_tn_4w, csrc/gemm.hip) over grids of at least
twice the CU count, where a workgroup walks several tiles: the cross-tile DMA stream, the epilogue
stores drained under the next tile's first K-tile (the EPI_OPS counted waits), the tile-id hand-off
through LDS and the r5 XCD tile queues (own queue, stealing, remainder pool) -- ADVICE r4: the
289-tile tests keep one tile per workgroup.

Integer-valued operands keep every fp32 sum exact, so every output must equal the exact product
through each epilogue's reference rounding points (oracle/wan_oracle.py; reference linears
wan_video_dit.py:131-134,157-160,209-210 via AutoWrappedLinear, vram_management/layers.py:115-188)
bit for bit, under the queue schedule and the static lists (option queue=0), with ragged last tile
rows / columns.  The queue words must be zero again after every launch (graph replays depend on it).
"""
import pytest
import torch

from oracle import wan_oracle as O
from gpu_util import BF16

pytestmark = pytest.mark.gpu


def ints(*shape, g, lo=-3, hi=4):
    return torch.randint(lo, hi, shape, generator=g, device="cuda").to(BF16)


@pytest.fixture(params=["queue", "queue_piece_blocks", "queue_held_reserve", "static"])
def sched(opt, request):
    # queue: split-tail pieces from the queue's piece pool (r6 default); queue_piece_blocks: the
    # pieces as workgroups of their own after the persistent ones (r5, option piece_queue=0);
    # queue_held_reserve: the pool + 1-3 round grids keeping 1/16 of each round as pieces (2)
    opt(gemm_tile=256, gemm_kernel=4, queue=0 if request.param == "static" else 1,
        piece_queue={"queue_piece_blocks": 0, "queue_held_reserve": 2}.get(request.param, 1))
    from vstyler import kernels
    return kernels


def queue_words_zero(K):
    bufs = [b for (kind, _, _), b in K._SPLIT_WS.items() if kind == 5]
    torch.cuda.synchronize()
    return bool(bufs) and all(int(b.count_nonzero()) == 0 for b in bufs)


# (M, N, K): 561 tiles (2 per workgroup + a 49-tile remainder pool), 833 tiles (3 per workgroup: one
# queued tile per slot + a 65-tile remainder), 833 tiles at K = 4096 (a split tail: 768 main tiles
# = 3 per workgroup, 65 tail tiles as 3 K pieces), 1537 tiles (6 per workgroup, 1 left over), the
# Ulysses SP = 8 FFN-down (7410 rows, K 13 824: 580 tiles = 2 per workgroup + 68 tail tiles in K
# pieces, which the persistent blocks take from the piece pool since r6)
SHAPES = [(8200, 4104, 1024), (12300, 4104, 1024), (12300, 4104, 4096), (24580, 4104, 1024),
          (7410, 5120, 13824)]


@pytest.mark.parametrize("M,N,Kd", SHAPES)
def test_gemm_4w_multitile_every_epilogue_exact(sched, M, N, Kd):
    K = sched
    S = M // 2 + 37                                       # two CFG rows of gate (ragged batch split)
    g = torch.Generator(device="cuda").manual_seed(M + Kd)
    a, w, b = ints(M, Kd, g=g), ints(N, Kd, g=g), ints(N, g=g, lo=-8, hi=9)
    w[:, 0] += (torch.arange(N, device="cuda") % 7).to(BF16)      # asymmetric: catches transposes
    y = (a.float() @ w.float().t() + b.float()).to(BF16)
    out = torch.full((M, N), 7.0, dtype=BF16, device="cuda")
    K.gemm(a, w, out, bias=b)
    assert torch.equal(out, y)
    yc = y.cpu()
    K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
    ref = O.gelu_tanh(yc)      # sigma form vs torch's tanh form: <= 1 ulp in the cancellation zone
    d = (out.cpu().float() - ref.float()).abs()
    assert (d <= ref.float().abs() * 2 ** -7 + 1e-6).all()
    K.gemm(a, w, out, epilogue=K.VS_EPI_SILU, bias=b)
    d = (out.cpu().float() - O.silu(yc).float()).abs()
    assert (d <= O.silu(yc).float().abs() * 2 ** -7 + 1e-6).all()
    gr = torch.Generator().manual_seed(M)
    res = torch.randn(M, N, generator=gr).to(BF16)
    gate = (0.25 * torch.randn(2, N, generator=gr)).to(BF16)
    hint = torch.randn(M, N, generator=gr).to(BF16)
    gres = torch.cat([O.gate_residual(res[:S], gate[0], yc[:S]), O.gate_residual(res[S:], gate[1], yc[S:])])
    for with_hint in (False, True):
        x = res.cuda()
        K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate.cuda(), gate_bstride=N,
               rows_per_batch=S, hint=hint.cuda() if with_hint else None, hint_scale=0.5)
        ref = O.add(gres, O.bf(hint.float() * 0.5)) if with_hint else gres
        assert torch.equal(x.cpu(), ref), with_hint
    x = res.cuda()
    K.gemm(a, w, x, epilogue=K.VS_EPI_RES, bias=b, residual=x, alpha=0.125)
    assert torch.equal(x.cpu(), O.add(res, O.bf(0.125 * yc.float())))
    assert queue_words_zero(K) or K.get_option("queue") == 0


@pytest.mark.parametrize("M,N,Kd", [(8200, 4104, 1024), (12300, 4104, 1024), (12300, 4104, 4096)])
def test_gemm_fp8_4w_multitile_exact(sched, M, N, Kd):
    """gemm_fp8_tn_4w on the same multi-tile grids: integer operands exact in e4m3 reproduce
    oracle.fp8_linear (per-row activation scale) bit for bit, plain bias and gate-residual + hint."""
    K = sched
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randint(-4, 5, (M, Kd), generator=g).to(BF16)
    x[::7] *= 512          # rows whose max exceeds 448: scale 2**k > 1
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    w[:, 0] += (torch.arange(N) % 5).to(BF16)
    b = torch.randint(-8, 9, (N,), generator=g).to(BF16)
    x8 = torch.empty(M, Kd, dtype=torch.uint8, device="cuda")
    sc = torch.empty(M, dtype=torch.float32, device="cuda")
    K.quant_fp8_rows(x.cuda(), x8, sc)
    w8 = w.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    # the exact product on the GPU (integer operands, |sum| < 2^24), then the oracle's epilogue order
    acc = x8.view(torch.float8_e4m3fn).float() @ w8.view(torch.float8_e4m3fn).float().t()
    y = O.bf(acc * sc[:, None] + b.cuda().float()).cpu()
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm_fp8(x8, sc, w8, out, bias=b.cuda())
    assert torch.equal(out.cpu(), y)
    S = M // 2
    res = torch.randn(M, N, generator=g).to(BF16)
    gate = (0.25 * torch.randn(2, N, generator=g)).to(BF16)
    hint = torch.randn(M, N, generator=g).to(BF16)
    ref = torch.cat([O.gate_residual(res[:S], gate[0], y[:S]), O.gate_residual(res[S:], gate[1], y[S:])])
    ref = O.add(ref, O.bf(hint.float() * 0.5))
    xo = res.cuda()
    K.gemm_fp8(x8, sc, w8, xo, epilogue=K.VS_EPI_GATE_RES, bias=b.cuda(), residual=xo, gate=gate.cuda(),
               gate_bstride=N, rows_per_batch=S, hint=hint.cuda(), hint_scale=0.5)
    assert torch.equal(xo.cpu(), ref)
    assert queue_words_zero(K) or K.get_option("queue") == 0


def test_queue_repeat_and_graph_replay_bit_identical(opt):
    """The queue words return to zero after every launch, so back-to-back launches and hipGraph
    replays of a multi-tile GEMM give the eager result bit for bit (random data, 14B q|k|v-like N)."""
    from vstyler import kernels as K
    opt(gemm_tile=256)
    M, N, Kd = 9000, 6144, 2048
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.randn(M, Kd, device="cuda", generator=g).to(BF16)
    w = (0.05 * torch.randn(N, Kd, device="cuda", generator=g)).to(BF16)
    b = (0.1 * torch.randn(N, device="cuda", generator=g)).to(BF16)
    ref = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a, w, ref, epilogue=K.VS_EPI_GELU, bias=b)
    out = torch.empty_like(ref)
    for _ in range(3):
        out.zero_()
        K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
        assert torch.equal(out, ref)
    assert queue_words_zero(K)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):          # bind this stream's workspaces eagerly, then capture
        K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        K.gemm(a, w, out, epilogue=K.VS_EPI_GELU, bias=b)
    for _ in range(3):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    assert queue_words_zero(K)
    rel = ((ref.float() - O.gelu_tanh(O.bf(a.float() @ w.float().t() + b.float())).float()).norm()
           / ref.float().norm()).item()
    assert rel < 1e-2, rel
