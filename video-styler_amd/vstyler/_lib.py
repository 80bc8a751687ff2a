"""ctypes binding of libvstyler.so (the C ABI declared in include/vstyler.h).

The product path has no CPU fallback: if the library is missing every op raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VSTYLER_LIB", os.path.join(_HERE, "lib", "libvstyler.so"))

VS_EPI_BIAS, VS_EPI_GELU, VS_EPI_SILU, VS_EPI_GATE_RES, VS_EPI_RES = range(5)

# path-selection options (include/vstyler.h VS_OPT_*): name -> id
OPTIONS = {"gemm_tile": 0, "gemm_kernel": 1, "gemm_split": 2, "queue": 3, "attn_impl": 4, "attn_mfma": 5,
           "attn_nc": 6, "attn_split": 7, "attn_persist": 8, "vae_pxb": 9, "vae_pre": 10,
           "vae_halo": 11, "piece_queue": 12}


class VsEpilogue(ctypes.Structure):
    _fields_ = [
        ("bias", ctypes.c_void_p),
        ("residual", ctypes.c_void_p),
        ("ld_res", ctypes.c_longlong),
        ("gate", ctypes.c_void_p),
        ("gate_bstride", ctypes.c_longlong),
        ("hint", ctypes.c_void_p),
        ("ld_hint", ctypes.c_longlong),
        ("hint_scale", ctypes.c_float),
        ("alpha", ctypes.c_float),
        ("rows_per_batch", ctypes.c_int),
        ("reserved", ctypes.c_int),
    ]


_P, _LL, _I, _F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float


class VsConv3d(ctypes.Structure):
    """struct vs_conv3d of include/vstyler.h (implicit-GEMM VAE convolution)."""
    _fields_ = [
        ("x", _P), ("x_zs", _LL), ("x_ns", _LL), ("ldx", _LL),
        ("n", _I), ("t_in", _I), ("h_in", _I), ("w_in", _I), ("cin", _I),
        ("kt", _I), ("kh", _I), ("kw", _I), ("st", _I), ("sh", _I), ("sw", _I),
        ("pt", _I), ("ph", _I), ("pw", _I), ("up2", _I), ("t_lo", _I),
        ("t_out", _I), ("h_out", _I), ("w_out", _I),
        ("w", _P), ("w_zs", _LL), ("ldw", _LL),
        ("bias", _P),
        ("cout", _I),
        ("y", _P), ("y_zs", _LL), ("y_ns", _LL), ("ldy", _LL),
        ("t_mul", _I), ("t_add", _I), ("split", _I), ("out_f32", _I),
        ("alpha", _F),
        ("res", _P),
        ("nz", _I),
    ]

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "vs_abi_version": [],
    "vs_strerror": [_I],
    "vs_gemm": [_P, _LL, _P, _LL, _P, _LL, _I, _I, _I, _I, ctypes.POINTER(VsEpilogue),
                _P, _LL, _P, _LL, _I, _P],
    "vs_quant_fp8_rows": [_P, _LL, _P, _LL, _P, _I, _I, _P],
    "vs_gemm_fp8": [_P, _LL, _P, _P, _LL, _P, _LL, _I, _I, _I, _I, ctypes.POINTER(VsEpilogue), _P],
    "vs_attn_fwd": [_P, _P, _P, _P, _I, _I, _I, _I, _I, _LL, _LL, _LL, _LL, _LL, _LL, _LL, _LL,
                    _F, _P],
    "vs_attn_split_plan": [_I, _I, _I, _I, _I, _P],
    "vs_gemm_split_plan": [_I, _I, _I, _I, _P],
    "vs_gemm_route": [_I, _I, _I],
    "vs_gemm_route_epi": [_I, _I, _I, _I, _I],
    "vs_split_workspace_bytes": [_I],
    "vs_set_option": [_I, _I],
    "vs_get_option": [_I],
    "vs_split_workspace_bind": [_I, _P, _LL, _P],
    "vs_layernorm_modulate": [_P, _LL, _P, _LL, _I, _I, _I, _P, _P, _LL, _P, _P, _F, _P],
    "vs_layernorm_modulate_fp8": [_P, _LL, _P, _LL, _P, _I, _I, _I, _P, _P, _LL, _P, _P, _F, _P],
    "vs_residual_layernorm": [_P, _LL, _P, _LL, _P, _LL, _I, _I, _I, ctypes.POINTER(VsEpilogue), _I, _P, _P, _LL,
                              _P, _P, _F, _P],
    "vs_rmsnorm_rope": [_P, _LL, _I, _I, _I, _P, _F, _P, _I, _I, _I, _I, _I, _I, _P],
    "vs_patchify": [_P, _P, _I, _I, _I, _I, _I, _P],
    "vs_unpatchify": [_P, _P, _I, _I, _I, _I, _I, _P],
    "vs_cfg_euler": [_P, _P, _P, _LL, _F, _F, _I, _P],
    "vs_cfg_euler_dev": [_P, _P, _P, _LL, _F, _P, _I, _P],
    "vs_time_sinusoid": [_P, _P, _I, _I, _P],
    "vs_mod_add": [_P, _P, _P, _I, _I, _I, _LL, _LL, _P],
    "vs_axpy": [_P, _P, _F, _LL, _P],
    "vs_ulysses_permute": [_P, _P, _I, _I, _I, _I, _LL, _LL, _I, _P],
    "vs_ulysses_permute_rows": [_P, _P, _I, _I, _I, _I, _LL, _LL, _LL, _I, _P],
    "vs_embed_rows": [_P, _P, _LL, _LL, _P, _LL, _LL, _I, _P],
    "vs_t5_bias_softmax": [_P, _LL, _LL, _P, _LL, _LL, _P, _P, _I, _I, _P, _I, _I, _P],
    "vs_t5_gelu_mul": [_P, _P, _P, _LL, _P],
    "vs_vae_conv": [ctypes.POINTER(VsConv3d), _P],
    "vs_vae_rmsnorm": [_P, _LL, _P, _LL, _P, _LL, _I, _I, _P],
    "vs_vae_softmax": [_P, _LL, _P, _LL, _LL, _I, _P],
    "vs_vae_transpose": [_P, _LL, _LL, _P, _LL, _LL, _I, _I, _I, _P],
    "vs_vae_attention": [_P, _LL, _LL, _P, _LL, _LL, _I, _I, _I, _P],
    "vs_vae_tile_gather": [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P],
    "vs_vae_to_u8": [_P, _P, _I, _I, _I, _P],
    "vs_unipc_update": [_P, _P, _P, _P, _P, _LL, _I, ctypes.POINTER(ctypes.c_float), _P],
    "vs_cast": [_P, _P, _LL, _I, _P],
    "vs_vace_prepare": [_P, _P, _P, _P, _P, _I, _I, _I, _P],
    "vs_vace_mask_latents": [_P, _P, _I, _I, _I, _I, _P],
    "vs_vae_tile_blend": [_P, _LL, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P],
    "vs_vae_blend_finish": [_P, _P, _P, _I, _LL, _I, _P],
    "vs_vae_copy_frames": [_P, _LL, _P, _LL, _I, _LL, _P],
    "vs_sp_unique_id": [_P],
    "vs_sp_init": [_I, _I, _P, _I, ctypes.POINTER(_P)],
    "vs_sp_all_to_all": [_P, _P, _P, _LL, _P],
    "vs_sp_all_gather": [_P, _P, _P, _LL, _P],
    "vs_sp_comm_destroy": [_P],
    "vs_sp_last_error": [],
}
_RESTYPES = {"vs_strerror": ctypes.c_char_p, "vs_split_workspace_bytes": ctypes.c_longlong,
             "vs_sp_last_error": ctypes.c_char_p}

_lib = None


def load():
    """Load libvstyler.so once; raise (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libvstyler.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C video-styler_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = lib
    return _lib


def check(code):
    if code != 0:
        msg = load().vs_strerror(code).decode()
        raise RuntimeError(f"vstyler kernel error {code}: {msg}")
