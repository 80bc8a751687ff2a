"""Typed wrappers over the C ABI: torch tensors in, launches on the current HIP stream.

PyTorch is used only for device memory and streams; every computation below is a kernel of
libvstyler.so.  Wrappers validate dtype/device/layout and raise ValueError before launching.
"""
import os
import ctypes

import torch

from . import _lib
from ._lib import VS_EPI_BIAS, VS_EPI_GELU, VS_EPI_SILU, VS_EPI_GATE_RES, VS_EPI_RES, VsEpilogue

BF16 = torch.bfloat16


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def set_option(name, value):
    """Select a path of libvstyler (include/vstyler.h VS_OPT_*, e.g. set_option("queue", 0));
    returns the previous value.  The defaults are the product configuration; tests and A/B probes
    use the others."""
    prev = _lib.load().vs_set_option(_lib.OPTIONS[name], int(value))
    if prev < 0:
        raise ValueError(f"vs_set_option: bad option {name}={value}")
    return prev


def get_option(name):
    return _lib.load().vs_get_option(_lib.OPTIONS[name])


class options:
    """Context manager: options(gemm_kernel=8, gemm_split=0) for the duration of a with-block."""

    def __init__(self, **kw):
        self.kw, self.saved = kw, {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.saved[k] = set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_option(k, v)
        return False


def apply_env_options():
    """VSTYLER_OPTS="queue=0,sp_comm=native": the one environment hook, read by the Python host
    (never by the library) so that A/B scripts can select paths of a whole run: host option names
    (vstyler.options) set the host's table, every other name a library option."""
    from .options import apply_spec
    apply_spec(os.environ.get("VSTYLER_OPTS", ""), set_option)


_SPLIT_WS = {}


def _split_ws(kind, t, nbytes=None):
    """Bind library scratch of `kind` (0 attention split tail, 1 GEMM split tail, 2 / 3 unused since
    r6 (the removed vendor-library route), 4 attention item flags, 5 GEMM tile and attention item
    queues) for the current stream of t's device from the torch
    allocator (vs_split_workspace_bind: the library never allocates).  Re-bound larger when a
    bigger one is needed; never inside a graph capture (the library then takes its fallback)."""
    stream = _stream(t)
    key = (kind, t.device.index, stream)
    have = _SPLIT_WS.get(key)
    if nbytes is None:
        if have is not None:
            return
        nbytes = _lib.load().vs_split_workspace_bytes(kind)
        if nbytes <= 0:             # a kind this build does not use (2, 3)
            return
    elif have is not None and have.numel() >= nbytes:
        return
    if torch.cuda.is_current_stream_capturing():
        return
    # kinds 4 (attention item flags) and 5 (GEMM tile queues) must be zero when bound; the library
    # keeps them zero
    buf = (torch.zeros if kind in (4, 5) else torch.empty)(nbytes, dtype=torch.uint8, device=t.device)
    _lib.check(_lib.load().vs_split_workspace_bind(kind, buf.data_ptr(), nbytes, stream))
    _SPLIT_WS[key] = buf


def _req(t, name):
    if t.dtype != BF16:
        raise ValueError(f"{name}: expected bfloat16, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device (cuda/hip) tensor")
    return t


def _rows(t, name):
    """(rows, cols, row_stride) of a 2-D view whose last dim is contiguous."""
    _req(t, name)
    if t.dim() < 2:
        raise ValueError(f"{name}: expected >=2-D tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"{name}: last dim must be contiguous")
    if t.dim() > 2:
        # all leading dims must collapse into one row index
        rows = 1
        for i in range(t.dim() - 1):
            rows *= t.shape[i]
        for i in range(t.dim() - 2):
            if t.stride(i) != t.stride(i + 1) * t.shape[i + 1]:
                raise ValueError(f"{name}: leading dims not collapsible")
        return rows, t.shape[-1], t.stride(-2)
    return t.shape[0], t.shape[1], t.stride(0)


def _ptr(t):
    return None if t is None else t.data_ptr()


def _epilogue(bias, residual, gate, gate_bstride, hint, hint_scale, alpha, rows_per_batch):
    ep = VsEpilogue()
    ep.bias = _ptr(bias)
    ep.hint_scale = float(hint_scale)
    ep.alpha = float(alpha)
    ep.rows_per_batch = int(rows_per_batch)
    if residual is not None:
        _, _, ldr = _rows(residual, "residual")
        ep.residual, ep.ld_res = residual.data_ptr(), ldr
    if gate is not None:
        ep.gate, ep.gate_bstride = gate.data_ptr(), int(gate_bstride)
    if hint is not None:
        _, _, ldh = _rows(hint, "hint")
        ep.hint, ep.ld_hint = hint.data_ptr(), ldh
    return ep


def gemm(a, w, out, epilogue=VS_EPI_BIAS, bias=None, residual=None, gate=None, gate_bstride=0,
         hint=None, hint_scale=1.0, alpha=1.0, rows_per_batch=0, a2=None, w2=None):
    """out[M,N] = epilogue(a[M,K] @ w[N,K]^T (+ a2 @ w2^T)) (see include/vstyler.h vs_gemm)."""
    M, K, lda = _rows(a, "a")
    N, Kw, ldw = _rows(w, "w")
    Mo, No, ldc = _rows(out, "out")
    if Kw != K or Mo != M or No != N:
        raise ValueError(f"gemm shape mismatch a={tuple(a.shape)} w={tuple(w.shape)} out={tuple(out.shape)}")
    ep = _epilogue(bias, residual, gate, gate_bstride, hint, hint_scale, alpha, rows_per_batch)
    k2, lda2, ldw2 = 0, 0, 0
    if a2 is not None:
        _, k2, lda2 = _rows(a2, "a2")
        _, _, ldw2 = _rows(w2, "w2")
    if k2 == 0:
        _split_ws(1, a)
        _split_ws(5, a)
        if gemm_route(M, N, K, epilogue=epilogue):   # the A/B build's library route only
            _split_ws(2, a)
            if epilogue in (VS_EPI_GATE_RES, VS_EPI_RES):
                _split_ws(3, a, M * N * 2)
    _lib.check(_lib.load().vs_gemm(a.data_ptr(), lda, w.data_ptr(), ldw, out.data_ptr(), ldc, M, N, K,
                                   int(epilogue), ep, _ptr(a2), lda2, _ptr(w2), ldw2, k2, _stream(a)))
    return out


def _rows_u8(t, name):
    if t.dtype != torch.uint8 or not t.is_cuda or t.dim() != 2 or t.stride(-1) != 1:
        raise ValueError(f"{name}: expected a 2-D row-major uint8 (e4m3 bits) device tensor")
    return t.shape[0], t.shape[1], t.stride(0)


def quant_fp8_rows(x, x8, scale):
    """x8 (uint8 e4m3 bits) and per-row fp32 scale of x, as fp8_linear (layers.py:124-137)."""
    M, K, ldx = _rows(x, "x")
    M8, K8, ld8 = _rows_u8(x8, "x8")
    if (M8, K8) != (M, K) or scale.dtype != torch.float32 or scale.numel() < M:
        raise ValueError("quant_fp8_rows: shape mismatch")
    _lib.check(_lib.load().vs_quant_fp8_rows(x.data_ptr(), ldx, x8.data_ptr(), ld8, scale.data_ptr(), M, K,
                                             _stream(x)))
    return x8, scale


def gemm_fp8(a8, scale_a, w8, out, epilogue=VS_EPI_BIAS, bias=None, residual=None, gate=None, gate_bstride=0,
             hint=None, hint_scale=1.0, alpha=1.0, rows_per_batch=0):
    """out = epilogue(scale_a[m] * (a8 @ w8^T)) with e4m3 operands (see vs_gemm_fp8)."""
    M, K, lda = _rows_u8(a8, "a8")
    N, Kw, ldw = _rows_u8(w8, "w8")
    Mo, No, ldc = _rows(out, "out")
    if Kw != K or Mo != M or No != N or scale_a.dtype != torch.float32:
        raise ValueError(f"gemm_fp8 shape mismatch a8={tuple(a8.shape)} w8={tuple(w8.shape)} out={tuple(out.shape)}")
    ep = _epilogue(bias, residual, gate, gate_bstride, hint, hint_scale, alpha, rows_per_batch)
    _split_ws(1, a8)                                                    # split tail of the MFMA kernel
    _split_ws(5, a8)                                                    # its tile queues
    if gemm_route(M, N, K, epilogue=epilogue, fp8=True):                # the A/B build's library route only
        _split_ws(2, a8)
        if epilogue in (VS_EPI_GATE_RES, VS_EPI_RES):
            _split_ws(3, a8, M * N * 2)
    _lib.check(_lib.load().vs_gemm_fp8(a8.data_ptr(), lda, scale_a.data_ptr(), w8.data_ptr(), ldw, out.data_ptr(),
                                       ldc, M, N, K, int(epilogue), ep, _stream(a8)))
    return out


def attention(q, k, v, out, num_heads, batch, scale=None):
    """q/out: [batch*Sq, >=H*128] rows, k/v: [batch*Skv, ...] (views with row strides allowed)."""
    Mq, _, ldq = _rows(q, "q")
    Mk, _, ldk = _rows(k, "k")
    Mv, _, ldv = _rows(v, "v")
    Mo, _, ldo = _rows(out, "out")
    if Mq % batch or Mk % batch or Mk != Mv or Mo != Mq:
        raise ValueError("attention: row counts do not match batch")
    sq, skv = Mq // batch, Mk // batch
    hd = 128
    if scale is None:
        scale = hd ** -0.5
    _split_ws(0, q)
    _split_ws(4, q)
    _split_ws(5, q)             # the persistent grid's XCD item queues (zero-filled words)
    _lib.check(_lib.load().vs_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), batch, sq,
                                       skv, num_heads, hd, ldq, ldk, ldv, ldo, sq * ldq, skv * ldk,
                                       skv * ldv, sq * ldo, float(scale), _stream(q)))
    return out


def attention_split_plan(batch, sq, skv, heads, cus):
    """(whole-item workgroups, split tail items, pieces per item, tiles per piece) of vs_attn_fwd."""
    out = (ctypes.c_int * 4)()
    _lib.check(_lib.load().vs_attn_split_plan(batch, sq, skv, heads, cus, out))
    return tuple(out)


def gemm_split_plan(m, n, k, cus):
    """(whole-tile workgroups, split tail tiles, K pieces per tile, K per piece) of vs_gemm (256 schedule)."""
    out = (ctypes.c_int * 4)()
    _lib.check(_lib.load().vs_gemm_split_plan(m, n, k, cus, out))
    return tuple(out)


def layernorm_modulate(x, out, eps=1e-6, shift=None, scale=None, mod_bstride=0, rows_per_batch=0,
                       weight=None, bias=None):
    M, D, ldx = _rows(x, "x")
    Mo, Do, ldo = _rows(out, "out")
    if Mo != M or Do != D:
        raise ValueError("layernorm_modulate: shape mismatch")
    _lib.check(_lib.load().vs_layernorm_modulate(x.data_ptr(), ldx, out.data_ptr(), ldo, M, D, int(rows_per_batch),
                                                 _ptr(shift), _ptr(scale), int(mod_bstride), _ptr(weight),
                                                 _ptr(bias), float(eps), _stream(x)))
    return out


def layernorm_modulate_fp8(x, x8, qscale, eps=1e-6, shift=None, scale=None, mod_bstride=0, rows_per_batch=0,
                           weight=None, bias=None):
    """layernorm_modulate straight into fp8_linear's activation quantisation: x8 [M, D] uint8 (e4m3fn
    bytes), qscale [M] fp32 -- equal to quant_fp8_rows of layernorm_modulate's bf16 output."""
    M, D, ldx = _rows(x, "x")
    if x8.dtype != torch.uint8 or x8.dim() != 2 or x8.shape[0] != M or x8.shape[1] < D or x8.stride(1) != 1:
        raise ValueError("layernorm_modulate_fp8: x8 must be uint8 [M, >=D] with unit column stride")
    if qscale.dtype != torch.float32 or qscale.numel() < M or not qscale.is_contiguous():
        raise ValueError("layernorm_modulate_fp8: qscale must be contiguous float32 [M]")
    _lib.check(_lib.load().vs_layernorm_modulate_fp8(x.data_ptr(), ldx, x8.data_ptr(), x8.stride(0), qscale.data_ptr(),
                                                     M, D, int(rows_per_batch), _ptr(shift), _ptr(scale),
                                                     int(mod_bstride), _ptr(weight), _ptr(bias), float(eps),
                                                     _stream(x)))
    return x8, qscale


def residual_layernorm(y, x, out, eps=1e-6, epilogue=VS_EPI_GATE_RES, gate=None, gate_bstride=0, gate_rows=0,
                       alpha=1.0, hint=None, hint_scale=1.0, shift=None, scale=None, mod_bstride=0,
                       rows_per_batch=0, weight=None, bias=None):
    """x = epilogue(y, x) (gate-residual / residual of a staged projection y), then
    out = layernorm_modulate(x) -- one pass (vs_residual_layernorm)."""
    M, D, ldy = _rows(y, "y")
    Mx, Dx, ldx = _rows(x, "x")
    Mo, Do, ldo = _rows(out, "out")
    if (Mx, Dx) != (M, D) or (Mo, Do) != (M, D):
        raise ValueError("residual_layernorm: shape mismatch")
    ep = _epilogue(None, None, gate, gate_bstride, hint, hint_scale, alpha, gate_rows)
    _lib.check(_lib.load().vs_residual_layernorm(y.data_ptr(), ldy, x.data_ptr(), ldx, out.data_ptr(), ldo, M, D,
                                                 int(epilogue), ep, int(rows_per_batch), _ptr(shift), _ptr(scale),
                                                 int(mod_bstride), _ptr(weight), _ptr(bias), float(eps), _stream(x)))
    return out


def gemm_route(M, N, K, epilogue=None, fp8=False):
    """True if vs_gemm (vs_gemm_fp8 with fp8=True) runs an (M, N, K) GEMM without LoRA phase and with
    `epilogue` as a staged product + a separate epilogue pass (vs_gemm_route / vs_gemm_route_epi):
    never in the product library (every GEMM fuses its epilogue), the vendor-library route of the
    A/B build (make ab)."""
    if epilogue is None and not fp8:
        return _lib.load().vs_gemm_route(int(M), int(N), int(K)) == 1
    ep = VS_EPI_BIAS if epilogue is None else int(epilogue)
    return _lib.load().vs_gemm_route_epi(int(M), int(N), int(K), ep, 1 if fp8 else 0) == 1


def rmsnorm_rope(x, weight, eps=1e-6, rope=None, grid=(1, 1, 1), rows_per_batch=0, token_offset=0, head_dim=128):
    M, D, ldx = _rows(x, "x")
    rlen = 0 if rope is None else rope.shape[0]
    if rope is not None and (rope.dtype != torch.float32 or rope.shape[1] != head_dim // 2 or rope.shape[2] != 2):
        raise ValueError("rope table must be float32 [len, head_dim/2, 2]")
    gf, gh, gw = grid
    _lib.check(_lib.load().vs_rmsnorm_rope(x.data_ptr(), ldx, M, D, head_dim, weight.data_ptr(), float(eps),
                                           _ptr(rope), rlen, gf, gh, gw, int(rows_per_batch), int(token_offset),
                                           _stream(x)))
    return x


def patchify(lat, out):
    _req(lat, "lat")
    B, C, T, H, W = lat.shape
    if not lat.is_contiguous() or not out.is_contiguous() or out.numel() != lat.numel():
        raise ValueError("patchify: contiguous tensors of equal numel required")
    _lib.check(_lib.load().vs_patchify(lat.data_ptr(), out.data_ptr(), B, C, T, H, W, _stream(lat)))
    return out


def unpatchify(tokens, out):
    _req(out, "out")
    B, C, T, H, W = out.shape
    if not tokens.is_contiguous() or not out.is_contiguous() or out.numel() != tokens.numel():
        raise ValueError("unpatchify: contiguous tensors of equal numel required")
    _lib.check(_lib.load().vs_unpatchify(tokens.data_ptr(), out.data_ptr(), B, C, T, H, W, _stream(out)))
    return out


def cfg_euler(v_pos, v_neg, x, cfg_scale, dsigma):
    for t, n in ((v_pos, "v_pos"), (x, "x")):
        _req(t, n)
        if not t.is_contiguous():
            raise ValueError(f"{n} must be contiguous")
    use_cfg = v_neg is not None
    _lib.check(_lib.load().vs_cfg_euler(v_pos.data_ptr(), _ptr(v_neg), x.data_ptr(), x.numel(), float(cfg_scale),
                                        float(dsigma), int(use_cfg), _stream(x)))
    return x


def cfg_euler_dev(v_pos, v_neg, x, cfg_scale, dsigma_dev):
    """cfg_euler with dsigma read from a one-element fp32 device tensor (graph-replayable)."""
    for t, n in ((v_pos, "v_pos"), (x, "x")):
        _req(t, n)
        if not t.is_contiguous():
            raise ValueError(f"{n} must be contiguous")
    if dsigma_dev.dtype != torch.float32 or not dsigma_dev.is_cuda:
        raise ValueError("dsigma_dev must be a float32 device tensor")
    _lib.check(_lib.load().vs_cfg_euler_dev(v_pos.data_ptr(), _ptr(v_neg), x.data_ptr(), x.numel(), float(cfg_scale),
                                            dsigma_dev.data_ptr(), int(v_neg is not None), _stream(x)))
    return x


def time_sinusoid(t, out):
    _lib.check(_lib.load().vs_time_sinusoid(t.data_ptr(), out.data_ptr(), t.numel(), out.shape[-1], _stream(t)))
    return out


def mod_add(param, tv, out, tv_bstride, tv_rstride):
    """out[b][r][d] = bf16(param[r][d] + tv[b*bs + r*rs + d]); out is [B, R, D] contiguous."""
    B, R, D = out.shape
    _lib.check(_lib.load().vs_mod_add(param.data_ptr(), tv.data_ptr(), out.data_ptr(), B, R, D, int(tv_bstride),
                                      int(tv_rstride), _stream(out)))
    return out


def axpy(x, y, scale):
    _lib.check(_lib.load().vs_axpy(x.data_ptr(), y.data_ptr(), float(scale), x.numel(), _stream(x)))
    return x


def ulysses_permute(src, dst, batch, s_local, world, cols_per_rank, ld_local, jstride, mode, packed_ld=None):
    """Row permutation between token-sharded / all_to_all-packed / head-sharded layouts (packed rows
    packed_ld elements apart, default cols_per_rank)."""
    pld = cols_per_rank if packed_ld is None else packed_ld
    _lib.check(_lib.load().vs_ulysses_permute_rows(src.data_ptr(), dst.data_ptr(), int(batch), int(s_local),
                                                   int(world), int(cols_per_rank), int(ld_local), int(jstride),
                                                   int(pld), int(mode), _stream(src)))
    return dst


__all__ = ["set_option", "get_option", "options", "ulysses_permute", "gemm", "attention", "layernorm_modulate", "rmsnorm_rope", "patchify", "unpatchify", "cfg_euler",
           "time_sinusoid", "mod_add", "axpy", "VS_EPI_BIAS", "VS_EPI_GELU", "VS_EPI_SILU", "VS_EPI_GATE_RES",
           "VS_EPI_RES"]
