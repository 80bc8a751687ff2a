"""Per-kernel parity: libvstyler (through the C ABI) vs the CPU oracle on the same seeded inputs.

Tolerances (bf16 path, fp32 accumulation): GEMM / attention rel-L2 <= 1e-2 and max-abs <= a few
bf16 ulps of the output scale; elementwise kernels bit-exact or <= 1 bf16 ulp (stated per test).
"""
import math

import pytest
import torch

from oracle import wan_oracle as O
from gpu_util import BF16, err

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (scale * torch.randn(*shape, generator=g)).to(BF16)


@pytest.fixture(params=["32", "16", "16c"])
def attn_mfma(request, opt):
    """Every attention test runs both MFMA shapes of attn_fwd_d128 (option attn_mfma); the 16x16x32 one
    with the optimistic softmax + redo (the default, "16") and with the checked kernel only ("16c",
    attn_nc=0)."""
    opt(attn_mfma=int(request.param[:2]))
    if request.param == "16c":
        opt(attn_nc=0)
    return request.param


@pytest.fixture(scope="module")
def K():
    from vstyler import kernels
    return kernels


@pytest.mark.parametrize("M,N,Kd", [(300, 320, 256), (1, 64, 64), (517, 1536, 1536), (128, 8960 // 4, 512)])
def test_gemm_bias(K, M, N, Kd):
    a, w, b = rnd(M, Kd, seed=1), rnd(N, Kd, scale=0.05, seed=2), rnd(N, scale=0.1, seed=3)
    ref = O.linear(a, w, b)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a.cuda(), w.cuda(), out, bias=b.cuda())
    mx, rl = err(out, ref)
    assert rl < 4e-3 and mx < 0.05 * ref.float().abs().max().item() + 1e-2, (mx, rl)


def test_gemm_asymmetric_exact(K):
    # integer-valued operands: fp32 accumulation is exact -> bit-exact result; catches C transposes
    M, N, Kd = 130, 132, 128
    g = torch.Generator().manual_seed(4)
    a = torch.randint(-3, 4, (M, Kd), generator=g).to(BF16)
    w = torch.randint(-3, 4, (N, Kd), generator=g).to(BF16)
    w[:, 0] += torch.arange(N).to(BF16) % 7
    ref = O.linear(a, w)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a.cuda(), w.cuda(), out)
    assert torch.equal(out.cpu(), ref)


def test_gemm_epilogues(K):
    M, N, Kd, S = 300, 256, 192, 150
    a, w, b = rnd(M, Kd, seed=5), rnd(N, Kd, scale=0.05, seed=6), rnd(N, scale=0.1, seed=7)
    y = O.linear(a, w, b)
    dev = lambda t: t.cuda()
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(dev(a), dev(w), out, epilogue=K.VS_EPI_GELU, bias=dev(b))
    assert err(out, O.gelu_tanh(y))[1] < 5e-3
    K.gemm(dev(a), dev(w), out, epilogue=K.VS_EPI_SILU, bias=dev(b))
    assert err(out, O.silu(y))[1] < 5e-3
    # gate-residual with per-batch gate rows (2 batches of S rows) + VACE hint
    res = rnd(M, N, seed=8)
    gate = rnd(2, N, scale=0.5, seed=9)
    hint = rnd(M, N, seed=10)
    ref = torch.cat([O.gate_residual(res[:S], gate[0], y[:S]), O.gate_residual(res[S:], gate[1], y[S:])])
    ref_h = O.add(ref, O.bf(hint.float() * 0.75))
    x = dev(res.clone())
    K.gemm(dev(a), dev(w), x, epilogue=K.VS_EPI_GATE_RES, bias=dev(b), residual=x, gate=dev(gate), gate_bstride=N,
           rows_per_batch=S)
    mx, rl = err(x, ref)
    assert rl < 4e-3, (mx, rl)
    x = dev(res.clone())
    K.gemm(dev(a), dev(w), x, epilogue=K.VS_EPI_GATE_RES, bias=dev(b), residual=x, gate=dev(gate), gate_bstride=N,
           rows_per_batch=S, hint=dev(hint), hint_scale=0.75)
    assert err(x, ref_h)[1] < 4e-3
    # residual add with alpha (LoRA merge form)
    x = dev(res.clone())
    K.gemm(dev(a), dev(w), x, epilogue=K.VS_EPI_RES, bias=dev(b), residual=x, alpha=0.5)
    assert err(x, O.add(res, O.bf(0.5 * y.float())))[1] < 4e-3


def test_gemm_split_tail_exact(K, opt):
    """Split tail of the 256x256 schedule: 18 x 16 = 288 tiles (last row and column partial) on
    256 CUs run 256 whole tiles and 32 tail tiles as 8 K pieces (7 x 576 + 128), summed and finished by the
    combine kernel.  Integer operands keep every fp32 sum exact, so the result must equal the
    exact product and, for every epilogue, the unsplit grid bit for bit."""
    M, N, Kd = 4452, 4000, 4160
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if cus == 256:
        assert K.gemm_split_plan(M, N, Kd, cus) == (256, 32, 8, 576)
    g = torch.Generator(device="cuda").manual_seed(80)
    a = torch.randint(-3, 4, (M, Kd), device="cuda", generator=g).to(BF16)
    w = torch.randint(-3, 4, (N, Kd), device="cuda", generator=g).to(BF16)
    b = torch.randint(-8, 9, (N,), device="cuda", generator=g).to(BF16)
    res = torch.randn(M, N, device="cuda", generator=g).to(BF16)
    gate = (0.25 * torch.randn(2, N, device="cuda", generator=g)).to(BF16)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(a, w, out, bias=b)
    ref = (a.float() @ w.float().t() + b.float()).to(BF16)
    assert torch.equal(out, ref)

    def run(split):
        opt(gemm_split=1 if split else 0)
        outs = []
        y = torch.empty(M, N, dtype=BF16, device="cuda")
        K.gemm(a, w, y, epilogue=K.VS_EPI_GELU, bias=b)
        outs.append(y)
        x = res.clone()
        K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate, gate_bstride=N,
               rows_per_batch=M // 2 + 1, hint=res, hint_scale=0.5)
        outs.append(x)
        x = res.clone()
        K.gemm(a, w, x, epilogue=K.VS_EPI_RES, residual=x, alpha=0.125)
        outs.append(x)
        return outs
    for s_, u_ in zip(run(True), run(False)):
        assert torch.equal(s_, u_)


def test_gemm_every_schedule_exact(K, opt):
    """Every GEMM schedule of vs_gemm on integer operands (every fp32 sum exact): the 128x128 kernel,
    the 8-phase and the 4-wave 256x256 kernels, the latter with the XCD tile queues and the static
    lists -- each epilogue (bias, GELU, SiLU, gate-residual with hint, residual) bit for bit the same
    (r5: the vendor-library route these once were compared with is gone; every one of these paths is
    reachable in the product, by shape or option)."""
    M, N, Kd = 4452, 4000, 4160
    g = torch.Generator(device="cuda").manual_seed(81)
    a = torch.randint(-3, 4, (M, Kd), device="cuda", generator=g).to(BF16)
    w = torch.randint(-3, 4, (N, Kd), device="cuda", generator=g).to(BF16)
    b = torch.randint(-8, 9, (N,), device="cuda", generator=g).to(BF16)
    res = torch.randn(M, N, device="cuda", generator=g).to(BF16)
    gate = (0.25 * torch.randn(2, N, device="cuda", generator=g)).to(BF16)

    def run(**o):
        opt(**o)
        outs = []
        for epi in (K.VS_EPI_BIAS, K.VS_EPI_GELU, K.VS_EPI_SILU):
            y = torch.empty(M, N, dtype=BF16, device="cuda")
            K.gemm(a, w, y, epilogue=epi, bias=b)
            outs.append(y)
        x = res.clone()
        K.gemm(a, w, x, epilogue=K.VS_EPI_GATE_RES, bias=b, residual=x, gate=gate, gate_bstride=N,
               rows_per_batch=M // 2 + 1, hint=res, hint_scale=0.5)
        outs.append(x)
        x = res.clone()
        K.gemm(a, w, x, epilogue=K.VS_EPI_RES, residual=x, alpha=0.125)
        outs.append(x)
        torch.cuda.synchronize()
        return outs
    ref = run(gemm_tile=128)
    assert torch.equal(ref[0], (a.float() @ w.float().t() + b.float()).to(BF16))
    for o in (dict(gemm_tile=256, gemm_kernel=8), dict(gemm_tile=256, gemm_kernel=4, queue=1),
              dict(gemm_tile=256, gemm_kernel=4, queue=0)):
        for i, (x, y) in enumerate(zip(run(**o), ref)):
            assert torch.equal(x, y), (o, i)


def test_gemm_lora_second_phase(K):
    M, N, Kd, r = 200, 320, 256, 128
    x, w, b = rnd(M, Kd, seed=11), rnd(N, Kd, scale=0.05, seed=12), rnd(N, scale=0.1, seed=13)
    la, lb = rnd(r, Kd, scale=0.05, seed=14), rnd(N, r, scale=0.05, seed=15)
    ref = O.lora_linear(x, w, b, la, lb)
    t = torch.empty(M, r, dtype=BF16, device="cuda")
    K.gemm(x.cuda(), la.cuda(), t)
    out = torch.empty(M, N, dtype=BF16, device="cuda")
    K.gemm(x.cuda(), w.cuda(), out, bias=b.cuda(), a2=t, w2=lb.cuda())
    assert err(out, ref)[1] < 5e-3


@pytest.mark.parametrize("B,Sq,Skv,H", [(1, 256, 256, 1), (2, 300, 300, 2), (2, 300, 77, 2), (1, 1000, 512, 3)])
def test_attention(attn_mfma, K, B, Sq, Skv, H):
    D = H * 128
    q, k, v = rnd(B, Sq, D, seed=20), rnd(B, Skv, D, seed=21), rnd(B, Skv, D, seed=22)
    ref = O.attention(q, k, v, H)
    out = torch.empty(B * Sq, D, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(B * Sq, D), k.cuda().view(B * Skv, D), v.cuda().view(B * Skv, D), out, H, B)
    mx, rl = err(out.view(B, Sq, D), ref)
    assert mx < 3e-2 and rl < 1e-2, (mx, rl)


@pytest.mark.parametrize("Skv", [1, 31, 32, 33, 63, 64, 65, 129])
def test_attention_key_tile_edges(attn_mfma, K, Skv):
    """Key counts around the 64-key tile and its two 32-key halves: the keys 0-31 half is masked
    and exponentiated inside the QK phase (split softmax), the keys 32-63 half in the PV phase."""
    B, Sq, H = 1, 300, 2
    D = H * 128
    q, k, v = rnd(B, Sq, D, seed=40), rnd(B, Skv, D, seed=41), rnd(B, Skv, D, seed=42)
    ref = O.attention(q, k, v, H)
    out = torch.empty(B * Sq, D, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(B * Sq, D), k.cuda().view(B * Skv, D), v.cuda().view(B * Skv, D), out, H, B)
    mx, rl = err(out.view(B, Sq, D), ref)
    assert mx < 3e-2 and rl < 1e-2, (mx, rl)


def test_attention_online_rescale_spike(attn_mfma, K):
    """Rule 26 of the CDNA guide: force the running-max rescale by a late large score."""
    B, S, H = 1, 512, 1
    q, k, v = rnd(B, S, 128, seed=30), rnd(B, S, 128, seed=31), rnd(B, S, 128, seed=32)
    q[0, 5] = 4.0
    k[0, 400] = 4.0          # tile 6 spikes query row 5's max
    ref = O.attention(q, k, v, H)
    out = torch.empty(S, 128, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(S, 128), k.cuda().view(S, 128), v.cuda().view(S, 128), out, H, B)
    mx, rl = err(out.view(B, S, 128), ref)
    assert mx < 3e-2, mx


def test_attention_overflow_spike(attn_mfma, K):
    """Scores that jump by far more than 128 in the exp2 domain (exp2 overflows to inf before the
    exact path runs): in the first tile, in a later tile's first and second 32-key halves."""
    B, S, H = 1, 512, 1
    q, k, v = rnd(B, S, 128, seed=33), rnd(B, S, 128, seed=34), rnd(B, S, 128, seed=35)
    for row, key in ((3, 10), (5, 300), (9, 360), (200, 511)):
        q[0, row] = 6.0
        k[0, key] = 6.0
    ref = O.attention(q, k, v, H)
    out = torch.empty(S, 128, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(S, 128), k.cuda().view(S, 128), v.cuda().view(S, 128), out, H, B)
    mx, rl = err(out.view(B, S, 128), ref)
    assert mx < 3e-2, mx


@pytest.mark.parametrize("late", [False, True])
def test_attention_first_tile_low_scores(attn_mfma, K, late):
    """Rows whose scores are all far below the initial reference max m = 0 (exp2 domain < -60):
    the first tile's partial sums fall under SUM_MIN, so it takes the exact path with S recomputed
    from K (its in-place exp2 underflowed).  late: only the first 64 keys are that low and the rest
    are ordinary, so the row's max then jumps by ~65 in a later tile (a second exact path)."""
    B, S, H = 1, 512, 1
    g = torch.Generator().manual_seed(36)
    u = torch.ones(128)
    k = (0.1 * torch.randn(B, S, 128, generator=g) + u).to(BF16)
    if late:
        k[0, 64:] = torch.randn(S - 64, 128, generator=g).to(BF16)
    q = torch.randn(B, S, 128, generator=g).to(BF16)
    for row in (0, 7, 200, 511):
        q[0, row] = (-4.0 * u + 0.01 * torch.randn(128, generator=g)).to(BF16)
    ref = O.attention(q, k, v := torch.randn(B, S, 128, generator=g).to(BF16), H)
    out = torch.empty(S, 128, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(S, 128), k.cuda().view(S, 128), v.cuda().view(S, 128), out, H, B)
    mx, rl = err(out.view(B, S, 128), ref)
    assert mx < 3e-2 and rl < 1e-2, (mx, rl)


def test_attention_rescale_many(attn_mfma, K):
    """Exact-path (rescale) decisions in the middle of the key sweep for many rows: row 7's max is
    raised three times in three different tiles, other rows once each, at keys spread over the
    sweep (rule 26: bounded random data alone never takes the branch after the first tile)."""
    B, S, H = 1, 2048, 2
    q, k, v = rnd(B, S, H * 128, seed=50), rnd(B, S, H * 128, seed=51), rnd(B, S, H * 128, seed=52)
    for key, row, a in ((300, 7, 0.3), (900, 7, 0.5), (1500, 7, 0.8), (130, 40, 0.4), (1999, 300, 0.6),
                        (64, 1000, 0.35), (1000, 2047, 0.7), (2047, 12, 0.9)):
        k[0, key] = (q[0, row].float() * a).to(BF16)
    ref = O.attention(q, k, v, H)
    out = torch.empty(S, H * 128, dtype=BF16, device="cuda")
    K.attention(q.cuda().view(S, H * 128), k.cuda().view(S, H * 128), v.cuda().view(S, H * 128), out, H, B)
    mx, rl = err(out.view(B, S, H * 128), ref)
    assert mx < 3e-2 and rl < 1e-2, (mx, rl)


def test_attention_kv_slab_beyond_4gb(attn_mfma, K):
    """K/V rows of stride 32768 so one (batch, head) slab spans 4.6 GB: the buffer descriptors are
    rebased per 64-key tile (the 1280x720x121 config's fused q|k|v rows span 3.4 GB).  Checked
    against a torch fp32 softmax(QK^T/sqrt(d))V on the GPU (test-side reference)."""
    Sq, Skv, ld = 256, 70000, 32768
    g = torch.Generator(device="cuda").manual_seed(60)
    q = torch.randn(Sq, 128, device="cuda", generator=g).to(BF16)
    k = torch.empty(Skv, ld, device="cuda", dtype=BF16)
    v = torch.empty(Skv, ld, device="cuda", dtype=BF16)
    k[:, :128] = torch.randn(Skv, 128, device="cuda", generator=g).to(BF16)
    v[:, :128] = torch.randn(Skv, 128, device="cuda", generator=g).to(BF16)
    k[:, 128:256] = 1e4          # neighbouring columns must never be read
    out = torch.empty(Sq, 128, dtype=BF16, device="cuda")
    K.attention(q, k[:, :128], v[:, :128], out, 1, 1)
    s = (q.float() @ k[:, :128].float().t()) * 128 ** -0.5
    ref = torch.softmax(s, -1) @ v[:, :128].float()
    del k, v
    mx = (out.float() - ref).abs().max().item()
    assert mx < 3e-2, mx


def test_attention_split_tail(attn_mfma, K, opt):
    """Split tail: 270 items on 256 CUs leave 14 items that run as 3 key ranges of 21 tiles each
    (the last ending in a partial tile) and are merged by the combine kernel.  Rows of whole and
    split items against a torch fp32 reference, and the split result against the unsplit grid."""
    B, Sq, Skv, H = 1, 23040, 4000, 3
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    plan = K.attention_split_plan(B, Sq, Skv, H, cus)
    if cus == 256:
        assert plan == (256, 14, 3, 21), plan
    g = torch.Generator(device="cuda").manual_seed(70)
    q = torch.randn(Sq, H * 128, device="cuda", generator=g).to(BF16)
    k = torch.randn(Skv, H * 128, device="cuda", generator=g).to(BF16)
    v = torch.randn(Skv, H * 128, device="cuda", generator=g).to(BF16)
    out = torch.empty_like(q)
    K.attention(q, k, v, out, H, B)
    opt(attn_split=0)
    whole = torch.empty_like(q)
    K.attention(q, k, v, whole, H, B)
    opt(attn_split=1)
    torch.cuda.synchronize()
    # items 256..269 = head 2, q-blocks 76..89 (rows 19456..23039) are the split tail
    rows = torch.cat([torch.arange(0, Sq, 997), torch.arange(19456, Sq, 61), torch.tensor([Sq - 1])]).cuda()
    for h in range(H):
        qs = q[rows, h * 128:(h + 1) * 128].float()
        ref = torch.softmax(qs @ k[:, h * 128:(h + 1) * 128].float().t() * 128 ** -0.5, -1) @ \
            v[:, h * 128:(h + 1) * 128].float()
        mx = (out[rows, h * 128:(h + 1) * 128].float() - ref).abs().max().item()
        assert mx < 3e-2, (h, mx)
    d = (out.float() - whole.float()).abs()
    assert d.max().item() < 2e-2, d.max().item()
    assert torch.equal(out[:19456], whole[:19456])        # whole items are untouched by the split
    assert torch.equal(out[:, :256], whole[:, :256])


@pytest.mark.parametrize("B,Sq,Skv,H", [(2, 7700, 7700, 10), (1, 12000, 4200, 24)])
def test_attention_long_items_switch_modes_bit_identical(attn_mfma, K, opt, B, Sq, Skv, H):
    """Persistent grids over long items (>= 64 key tiles: several items per CU, partial last q-block and
    key tile): the synchronous item switch (O stored and the next Q loaded at the switch) and one
    item per block are bit-identical."""
    D = H * 128
    g = torch.Generator(device="cuda").manual_seed(73)
    q = torch.randn(B * Sq, D, device="cuda", generator=g).to(BF16)
    k = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    v = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    outs = []
    for persist in (1, 0):
        opt(attn_persist=persist)
        o = torch.empty_like(q)
        K.attention(q, k, v, o, H, B)
        outs.append(o)
    opt(attn_persist=1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    rows = torch.tensor([0, 255, 256, Sq // 2, Sq - 1]).cuda()
    for b in range(B):
        for h in (0, H - 1):
            qs = q[b * Sq + rows, h * 128:(h + 1) * 128].float()
            ks = k[b * Skv:(b + 1) * Skv, h * 128:(h + 1) * 128].float()
            vs = v[b * Skv:(b + 1) * Skv, h * 128:(h + 1) * 128].float()
            ref = torch.softmax(qs @ ks.t() * 128 ** -0.5, -1) @ vs
            mx = (outs[0][b * Sq + rows, h * 128:(h + 1) * 128].float() - ref).abs().max().item()
            assert mx < 3e-2, (b, h, mx)


@pytest.mark.parametrize("B,Sq,Skv,H", [(2, 23000, 512, 3), (1, 20000, 500, 7), (2, 9000, 1000, 8)])
def test_attention_persistent_matches_one_item_per_block(attn_mfma, K, opt, B, Sq, Skv, H):
    """Persistent grid (one block per CU, several items each, the K/V pipeline running across item
    boundaries, the next item's Q prefetched through LDS): bit-identical to the one-item-per-block
    grid (option attn_persist=0) -- every item starts from m = 0 exactly as a fresh block -- and
    against a torch fp32 reference on rows of items at both ends of the blocks' item lists.  The
    shapes cross (batch, head) boundaries between a block's consecutive items, end in partial
    q-blocks, and have 8 key tiles (the cross-attention's 512 keys; 500: a partial last tile)."""
    D = H * 128
    g = torch.Generator(device="cuda").manual_seed(71)
    q = torch.randn(B * Sq, D, device="cuda", generator=g).to(BF16)
    k = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    v = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    out = torch.empty_like(q)
    K.attention(q, k, v, out, H, B)
    opt(attn_persist=0)
    ref1 = torch.empty_like(q)
    K.attention(q, k, v, ref1, H, B)
    opt(attn_persist=1)
    torch.cuda.synchronize()
    assert torch.equal(out, ref1)
    rows = torch.cat([torch.arange(0, Sq, 331), torch.tensor([255, 256, Sq - 1])]).cuda()
    for b in range(B):
        for h in range(H):
            qs = q[b * Sq + rows, h * 128:(h + 1) * 128].float()
            ks = k[b * Skv:(b + 1) * Skv, h * 128:(h + 1) * 128].float()
            vs = v[b * Skv:(b + 1) * Skv, h * 128:(h + 1) * 128].float()
            ref = torch.softmax(qs @ ks.t() * 128 ** -0.5, -1) @ vs
            mx = (out[b * Sq + rows, h * 128:(h + 1) * 128].float() - ref).abs().max().item()
            assert mx < 3e-2, (b, h, mx)


def _flags_zero(K):
    """The kind-4 workspaces' count, done and per-item flags (ints [0, 2 + cap)) are zero."""
    bufs = [b for (kind, _, _), b in K._SPLIT_WS.items() if kind == 4]
    def head(b):
        ints = b.view(torch.int32)
        return ints[:2 + (ints.numel() - 2) // 2]
    return bool(bufs) and all(int(head(b).count_nonzero()) == 0 for b in bufs)


@pytest.mark.parametrize("split", [False, True])
def test_attention_nc_redo(K, opt, split):
    """Optimistic softmax (no running max, row sums on MFMA) + redo: items with a row whose sum
    leaves [2^-64, 2^64] -- an overflow spike (score ~ +590 in the exp2 domain), a row whose every
    score is ~ -190 (all p underflow) -- are recomputed by the checked kernel and match it bit for
    bit; the other items stay within the bf16 tolerance of it; the item flags are all zero again
    afterwards.  split: the spikes sit in split-tail items (flagged by the combine kernel)."""
    opt(attn_mfma=16)
    B, Sq, Skv, H = 1, 23040, 4000, 3          # 256 whole items + a 14-item split tail on 256 CUs
    g = torch.Generator(device="cuda").manual_seed(75)
    q = torch.randn(Sq, H * 128, device="cuda", generator=g).to(BF16)
    k = torch.randn(Skv, H * 128, device="cuda", generator=g).to(BF16)
    v = torch.randn(Skv, H * 128, device="cuda", generator=g).to(BF16)
    u = torch.ones(128, device="cuda", dtype=BF16)
    # (head, query row): spike rows against key 1234 of that head, low rows against every key
    spikes = [(2, 20000), (2, 22000)] if split else [(0, 300), (1, 5000)]
    lows = [(2, 21000)] if split else [(0, 9000)]
    for h, r in lows:           # keys of that head ~ N(1, 1): the row's scores ~ -20 * 128 / sqrt(128)
        k[:, h * 128:(h + 1) * 128] += 1.0
        q[r, h * 128:(h + 1) * 128] = -20.0 * u
    for h, r in spikes:
        q[r, h * 128:(h + 1) * 128] = 6.0 * u
        k[1234, h * 128:(h + 1) * 128] = 6.0 * u
    out = torch.empty_like(q)
    K.attention(q, k, v, out, H, B)
    torch.cuda.synchronize()
    assert _flags_zero(K)
    opt(attn_nc=0, attn_split=0)       # the redo runs every item unsplit
    chk = torch.empty_like(q)
    K.attention(q, k, v, chk, H, B)
    torch.cuda.synchronize()
    flagged = torch.zeros(Sq, H, dtype=torch.bool, device="cuda")
    for h, r in spikes + lows:
        flagged[r // 256 * 256:(r // 256 + 1) * 256, h] = True
    o3, c3 = out.view(Sq, H, 128), chk.view(Sq, H, 128)
    assert torch.equal(o3[flagged], c3[flagged])
    assert (o3[~flagged].float() - c3[~flagged].float()).abs().max().item() < 2e-2
    assert torch.isfinite(out.float()).all()


def test_attention_strided_views(attn_mfma, K):
    # q/k/v as column slices of a fused [M, 3D] buffer (row stride 3D)
    B, S, H = 1, 200, 2
    D = H * 128
    qkv = rnd(B * S, 3 * D, seed=40)
    ref = O.attention(qkv[:, :D].reshape(B, S, D), qkv[:, D:2 * D].reshape(B, S, D), qkv[:, 2 * D:].reshape(B, S, D), H)
    d = qkv.cuda()
    out = torch.empty(B * S, D, dtype=BF16, device="cuda")
    K.attention(d[:, :D], d[:, D:2 * D], d[:, 2 * D:], out, H, B)
    assert err(out.view(B, S, D), ref)[1] < 1e-2


@pytest.mark.parametrize("D", [1536, 5120, 6144, 8192])    # > 5120: the 8-chunk wide-row instantiation
def test_layernorm_modulate(K, D):
    B, S = 2, 37
    x = rnd(B * S, D, scale=2.0, seed=50)
    mod = rnd(B, 6, D, scale=0.3, seed=51)
    ref = torch.cat([O.modulate(O.layer_norm(x[b * S:(b + 1) * S]), mod[b, 0], mod[b, 1]) for b in range(B)])
    out = torch.empty(B * S, D, dtype=BF16, device="cuda")
    md = mod.cuda()
    K.layernorm_modulate(x.cuda(), out, 1e-6, shift=md[:, 0], scale=md[:, 1], mod_bstride=6 * D, rows_per_batch=S)
    mx, _ = err(out, ref)
    assert mx <= 2 ** -5 * max(1.0, ref.float().abs().max().item()), mx
    w, b = rnd(D, scale=0.1, seed=52) + 1, rnd(D, scale=0.1, seed=53)
    ref = O.layer_norm(x, 1e-6, w, b)
    K.layernorm_modulate(x.cuda(), out, 1e-6, weight=w.cuda(), bias=b.cuda())
    assert err(out, ref)[0] <= 2 ** -5 * max(1.0, ref.float().abs().max().item())


@pytest.mark.parametrize("mode", ["gate_res", "gate_res_hint", "res"])
def test_residual_layernorm_matches_two_passes(K, mode):
    """vs_residual_layernorm == vs_gemm's residual epilogue on a staged y, then vs_layernorm_modulate."""
    B, S, D = 2, 37, 1536
    M = B * S
    y, x0 = rnd(M, D, scale=0.5, seed=60).cuda(), rnd(M, D, scale=2.0, seed=61).cuda()
    mod = rnd(B, 6, D, scale=0.3, seed=62).cuda()
    hint = rnd(M, D, seed=63).cuda()
    w, b = (rnd(D, scale=0.1, seed=64) + 1).cuda(), rnd(D, scale=0.1, seed=65).cuda()
    eye = torch.eye(D, dtype=BF16, device="cuda")       # y = y . I^T exactly: the epilogue runs on y
    x1, h1 = x0.clone(), torch.empty(M, D, dtype=BF16, device="cuda")
    x2, h2 = x0.clone(), torch.empty(M, D, dtype=BF16, device="cuda")
    if mode == "res":
        K.gemm(y, eye, x1, epilogue=K.VS_EPI_RES, residual=x1, alpha=0.75)
        K.layernorm_modulate(x1, h1, 1e-6, shift=mod[:, 3], scale=mod[:, 4], mod_bstride=6 * D, rows_per_batch=S)
        K.residual_layernorm(y, x2, h2, 1e-6, epilogue=K.VS_EPI_RES, alpha=0.75, shift=mod[:, 3], scale=mod[:, 4],
                             mod_bstride=6 * D, rows_per_batch=S)
    else:
        hk = dict(hint=hint, hint_scale=0.5) if mode == "gate_res_hint" else {}
        K.gemm(y, eye, x1, epilogue=K.VS_EPI_GATE_RES, residual=x1, gate=mod[:, 2], gate_bstride=6 * D,
               rows_per_batch=S, **hk)
        K.layernorm_modulate(x1, h1, 1e-6, weight=w, bias=b)
        K.residual_layernorm(y, x2, h2, 1e-6, epilogue=K.VS_EPI_GATE_RES, gate=mod[:, 2], gate_bstride=6 * D,
                             gate_rows=S, weight=w, bias=b, **hk)
    assert torch.equal(x1, x2)
    assert torch.equal(h1, h2)


@pytest.mark.parametrize("H", [2, 48])     # D = 256; 6144 runs on the 8-chunk wide-row instantiation
def test_rmsnorm_rope(K, H):
    B, grid = 2, (3, 4, 5)
    S, D = 60, 128 * H
    x = rnd(B * S, D, scale=3.0, seed=60)
    w = (1 + 0.1 * torch.randn(D, generator=torch.Generator().manual_seed(61))).to(BF16)
    freqs = O.rope_freqs(*grid)
    ref = O.rope_apply(O.rms_norm(x.view(B, S, D), w), freqs, H).reshape(B * S, D)
    from vstyler.models import rope_table
    xd = x.cuda()
    K.rmsnorm_rope(xd, w.cuda(), 1e-6, rope=rope_table(device="cuda"), grid=grid, rows_per_batch=S)
    mx, rl = err(xd, ref)
    assert mx <= 2 ** -6 * 4 and rl < 2e-3, (mx, rl)
    # no rope (cross-attention q/k) is exact to the rounding of the two bf16 products
    xd = x.cuda()
    K.rmsnorm_rope(xd, w.cuda(), 1e-6)
    assert err(xd, O.rms_norm(x, w))[0] <= 2 ** -6 * 4
    # SP shard: rows are the tokens [20, 40) of the grid
    xs = x.view(B, S, D)[:, 20:40].reshape(B * 20, D).contiguous().cuda()
    K.rmsnorm_rope(xs, w.cuda(), 1e-6, rope=rope_table(device="cuda"), grid=grid, rows_per_batch=20, token_offset=20)
    assert err(xs.view(B, 20, D), ref.view(B, S, D)[:, 20:40])[1] < 2e-3


def test_patchify_unpatchify_time_modadd_cfg(K):
    lat = rnd(2, 16, 3, 8, 12, seed=70)
    D = 64
    cols = torch.empty(2 * 3 * 4 * 6, 64, dtype=BF16, device="cuda")
    K.patchify(lat.cuda(), cols)
    eye = torch.eye(D).reshape(D, 16, 1, 2, 2).to(BF16)
    ref, grid = O.patchify(lat, eye, torch.zeros(D, dtype=BF16))
    assert torch.equal(cols.cpu().view_as(ref), ref)
    tok = rnd(2 * 3 * 4 * 6, 64, seed=71)
    back = torch.empty(2, 16, 3, 8, 12, dtype=BF16, device="cuda")
    K.unpatchify(tok.cuda(), back)
    assert torch.equal(back.cpu(), O.unpatchify(tok.view(2, -1, 64), grid, 16))
    t = torch.tensor([1000.0, 833.3333]).to(BF16)
    s = torch.empty(2, 256, dtype=BF16, device="cuda")
    K.time_sinusoid(t.cuda(), s)
    assert torch.equal(s.cpu(), O.sinusoidal_embedding_1d(256, t))
    p, tv = rnd(1, 6, 64, seed=72), rnd(2, 6, 64, seed=73)
    out = torch.empty(2, 6, 64, dtype=BF16, device="cuda")
    K.mod_add(p.cuda().view(6, 64), tv.cuda(), out, 6 * 64, 64)
    assert torch.equal(out.cpu(), O.bf(p.float() + tv.float()))
    vp, vn, x = rnd(1, 16, 2, 16, 16, seed=74), rnd(1, 16, 2, 16, 16, seed=75), rnd(1, 16, 2, 16, 16, seed=76)
    sig, _ = O.set_timesteps(2)
    ds = O.euler_delta(sig, 0)
    ref = O.cfg_euler(vp, vn, x, 5.0, ds)
    xd = x.cuda()
    K.cfg_euler(vp.cuda(), vn.cuda(), xd, 5.0, float(ds))
    assert torch.equal(xd.cpu(), ref)


def test_ulysses_permute_roundtrip(K):
    B, Sl, P, cpr = 2, 24, 4, 128
    D = P * cpr
    local = rnd(B * Sl, D, seed=80).cuda()
    packed = torch.empty(P * B * Sl * cpr, dtype=BF16, device="cuda")
    K.ulysses_permute(local, packed, B, Sl, P, cpr, D, B * Sl * cpr, 0)
    ref = local.view(B, Sl, P, cpr).permute(2, 0, 1, 3).reshape(-1)
    assert torch.equal(packed, ref)
    back = torch.empty_like(local)
    K.ulysses_permute(packed, back, B, Sl, P, cpr, D, B * Sl * cpr, 1)
    assert torch.equal(back, local)
    full = torch.empty(B * P * Sl, cpr, dtype=BF16, device="cuda")
    K.ulysses_permute(packed, full, B, Sl, P, cpr, D, B * Sl * cpr, 2)
    assert torch.equal(full.view(B, P, Sl, cpr), packed.view(P, B, Sl, cpr).permute(1, 0, 2, 3))
    packed2 = torch.empty_like(packed)
    K.ulysses_permute(full, packed2, B, Sl, P, cpr, D, B * Sl * cpr, 3)
    assert torch.equal(packed2, packed)


def test_ulysses_permute_interleaved_rows(K):
    """One sample's q|k|v packed as [rank j][token t][q | k | v] (packed_ld = 3 cpr): chunk j, read
    as rows, is rank j's heads of q|k|v for every local token, so the concatenated chunks are the
    whole sequence's q|k|v rows in token order (the layout usp.attend reads in place)."""
    Sl, P, cpr = 40, 4, 128
    D = P * cpr
    src = [rnd(Sl, 3 * D, seed=81 + i).cuda()[:, i * D:(i + 1) * D] for i in range(3)]   # fused q|k|v slices
    send = torch.empty(P * 3 * Sl * cpr, dtype=BF16, device="cuda")
    for i, t in enumerate(src):
        K.ulysses_permute(t, send[i * cpr:], 1, Sl, P, cpr, t.stride(0), 3 * Sl * cpr, 0, packed_ld=3 * cpr)
    rows = send.view(P, Sl, 3, cpr)
    for i, t in enumerate(src):
        assert torch.equal(rows[:, :, i], t.reshape(Sl, P, cpr).permute(1, 0, 2))


@pytest.mark.parametrize("B,Sq,Skv,H", [(2, 7700, 7700, 10), (2, 29640, 29640, 5), (1, 12000, 4200, 24)])
def test_attention_item_queue_matches_static_lists(K, opt, B, Sq, Skv, H):
    """attn_fwd_w4's persistent blocks fed by the XCD item queues (default) vs the static per-block
    item lists (option queue=0): every item is computed the same way whichever block takes it, so
    the outputs are bit-identical; the queue words are zero again after every launch (the last block
    zeroes them), so repeated launches agree too.  (2, 29640, 29640, 5): the Ulysses SP = 8 rank shape."""
    D = H * 128
    g = torch.Generator(device="cuda").manual_seed(77)
    q = torch.randn(B * Sq, D, device="cuda", generator=g).to(BF16)
    k = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    v = torch.randn(B * Skv, D, device="cuda", generator=g).to(BF16)
    outs = []
    for qopt in (1, 1, 0):
        opt(queue=qopt)
        o = torch.empty_like(q)
        K.attention(q, k, v, o, H, B)
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    bufs = [b for (kind, _, _), b in K._SPLIT_WS.items() if kind == 5]
    assert bufs and all(int(b.count_nonzero()) == 0 for b in bufs)
