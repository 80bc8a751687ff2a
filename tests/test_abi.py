"""The C-ABI library: loads, exports every symbol include/vstyler.h declares, validates arguments
before launching (no GPU needed: invalid calls return VS_E_INVALID/VS_E_UNSUPPORTED up front)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "vstyler.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int)\s+(vs_\w+)\s*\(", src, re.M)))


def test_header_declares_abi():
    syms = header_symbols()
    assert "vs_gemm" in syms and "vs_attn_fwd" in syms and len(syms) >= 13


def test_library_exports_every_header_symbol():
    from vstyler import _lib
    lib = _lib.load()
    for s in header_symbols():
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert lib.vs_abi_version() == 2


def test_error_codes_and_messages():
    from vstyler import _lib
    lib = _lib.load()
    assert lib.vs_strerror(0) == b"VS_OK"
    assert lib.vs_strerror(1).startswith(b"VS_E_INVALID")
    assert lib.vs_strerror(3).startswith(b"VS_E_UNSUPPORTED")


def test_invalid_arguments_rejected_before_launch():
    from vstyler import _lib
    lib = _lib.load()
    ep = _lib.VsEpilogue()
    # null pointers
    assert lib.vs_gemm(None, 64, None, 64, None, 64, 8, 8, 64, 0, ep, None, 0, None, 0, 0, None) == 1
    fake = 1 << 20   # aligned non-null (never dereferenced: validation fails first)
    # fp8: K must be a multiple of 128 (the MFMA kernel's K-tile; K = 192 rejected up front), and 256
    # passes validation only to fail on the null scale vector
    assert lib.vs_gemm_fp8(fake, 192, fake, fake, 192, fake, 8, 8, 8, 192, 0, ep, None) == 1
    assert lib.vs_gemm_fp8(fake, 256, None, fake, 256, fake, 8, 8, 8, 256, 0, ep, None) == 1
    # K not a multiple of 64
    assert lib.vs_gemm(fake, 48, fake, 48, fake, 8, 8, 8, 48, 0, ep, None, 0, None, 0, 0, None) == 1
    # bad epilogue id
    assert lib.vs_gemm(fake, 64, fake, 64, fake, 8, 8, 8, 64, 9, ep, None, 0, None, 0, 0, None) == 1
    # gate-residual without residual
    assert lib.vs_gemm(fake, 64, fake, 64, fake, 8, 8, 8, 64, 3, ep, None, 0, None, 0, 0, None) == 1
    # head_dim != 128 is unsupported, misaligned stride invalid
    assert lib.vs_attn_fwd(fake, fake, fake, fake, 1, 16, 16, 1, 64, 64, 64, 64, 64, 0, 0, 0, 0, 1.0, None) == 3
    assert lib.vs_attn_fwd(fake, fake, fake, fake, 1, 16, 16, 1, 128, 130, 128, 128, 128, 0, 0, 0, 0, 1.0, None) == 1
    # rmsnorm dim too large / not multiple of 8
    assert lib.vs_rmsnorm_rope(fake, 8200, 4, 8200, 128, fake, 1e-6, None, 0, 1, 1, 1, 0, 0, None) == 1
    assert lib.vs_layernorm_modulate(fake, 12, fake, 12, 4, 12, 0, None, None, 0, None, None, 1e-6, None) == 1
    # RoPE token range beyond the grid
    assert lib.vs_rmsnorm_rope(fake, 256, 4, 256, 128, fake, 1e-6, fake, 1024, 1, 1, 2, 4, 0, None) == 1
    # VAE flash attention: c a multiple of 128 up to 384, qkv rows >= 3c, 16-B aligned qkv
    assert lib.vs_vae_attention(fake, 64 * 576, 576, fake, 64 * 192, 192, 1, 64, 192, None) == 1
    assert lib.vs_vae_attention(fake, 64 * 1536, 1536, fake, 64 * 512, 512, 1, 64, 512, None) == 1
    assert lib.vs_vae_attention(fake, 64 * 300, 300, fake, 64 * 128, 128, 1, 64, 128, None) == 1
    assert lib.vs_vae_attention(fake + 8, 64 * 384, 384, fake, 64 * 128, 128, 1, 64, 128, None) == 1
    assert lib.vs_vae_attention(fake, 63 * 384, 384, fake, 64 * 128, 128, 1, 64, 128, None) == 1
    # Ulysses permute: columns not a multiple of 8
    assert lib.vs_ulysses_permute(fake, fake, 1, 4, 2, 12, 24, 48, 0, None) == 1
    # SP collectives: argument checks come before RCCL is opened or a device is touched
    out = ctypes.c_void_p()
    assert lib.vs_sp_unique_id(None) == 1
    assert lib.vs_sp_init(0, 0, fake, 0, ctypes.byref(out)) == 1          # world < 1
    assert lib.vs_sp_init(2, 2, fake, 0, ctypes.byref(out)) == 1          # rank >= world
    assert lib.vs_sp_init(0, 1, None, 0, ctypes.byref(out)) == 1          # no unique id
    assert lib.vs_sp_all_to_all(None, fake, fake, 16, None) == 1
    assert lib.vs_sp_all_gather(None, fake, fake, 16, None) == 1
    assert lib.vs_sp_comm_destroy(None) == 1
    assert lib.vs_strerror(4).startswith(b"VS_E_COMM")
    assert lib.vs_sp_last_error() == b""


def test_wrappers_raise_on_bad_dtype():
    import torch
    from vstyler import kernels as K
    with pytest.raises(ValueError):
        K.gemm(torch.zeros(4, 64), torch.zeros(4, 64), torch.zeros(4, 4))


def test_lora_key_layouts():
    """GeneralLoRALoader.get_name_dict (lora/__init__.py:11-25) naming, plus the kohya layout
    (lora_down/lora_up/alpha) of CausVid-style LoRAs normalised onto it."""
    import torch
    from vstyler.lora import get_name_dict, normalize_lora_keys
    sd = {"diffusion_model.blocks.0.self_attn.q.lora_B.default.weight": torch.ones(8, 4),
          "diffusion_model.blocks.0.self_attn.q.lora_A.default.weight": torch.ones(4, 8),
          "vace_blocks.1.ffn.0.lora_B.weight": torch.ones(8, 4),
          "vace_blocks.1.ffn.0.lora_A.weight": torch.ones(4, 8)}
    names = get_name_dict(sd)
    assert set(names) == {"blocks.0.self_attn.q", "vace_blocks.1.ffn.0"}
    kohya = {"diffusion_model.blocks.3.cross_attn.o.lora_down.weight": torch.ones(32, 16),
             "diffusion_model.blocks.3.cross_attn.o.lora_up.weight": torch.full((16, 32), 2.0),
             "diffusion_model.blocks.3.cross_attn.o.alpha": torch.tensor(16.0)}
    norm = normalize_lora_keys(kohya)
    names = get_name_dict(norm)
    assert list(names) == ["blocks.3.cross_attn.o"]
    b, a = norm[names["blocks.3.cross_attn.o"][0]], norm[names["blocks.3.cross_attn.o"][1]]
    assert a.shape == (32, 16) and torch.allclose(b, torch.full((16, 32), 1.0))   # 2 * 16/32


def test_attention_split_plan_host_only():
    """vs_attn_split_plan is host arithmetic (no device call): the 14B 832x480x73 self-attention
    grid (9280 items) on 256 CUs splits its last 64 items 4 ways; SP=8 (5 heads per rank) splits
    136 items 7 ways; cross-attention (8 key tiles) and exact multiples are never split."""
    from vstyler import _lib
    lib = _lib.load()
    out = (ctypes.c_int * 4)()
    cases = [((2, 29640, 29640, 40, 256), (9216, 64, 4, 116)),
             ((2, 29640, 29640, 5, 256), (1024, 136, 7, 67)),
             ((2, 29640, 512, 40, 256), (9280, 0, 1, 0)),
             ((1, 256 * 256, 4096, 1, 256), (256, 0, 1, 0)),
             ((2, 29640, 29640, 40, 0), (9280, 0, 1, 0))]
    for args, want in cases:
        assert lib.vs_attn_split_plan(*args, out) == 0
        assert tuple(out) == want, (args, tuple(out))
        nmain, ntail, nsplit, tiles = want
        if ntail:
            nkv = (args[2] + 63) // 64
            assert (nsplit - 1) * tiles < nkv <= nsplit * tiles
    assert lib.vs_attn_split_plan(0, 1, 1, 1, 256, out) == 1


def test_gemm_split_plan_host_only():
    """vs_gemm_split_plan (host arithmetic, measured cost model): the 14B N=5120 GEMMs (4640 tiles)
    split their last 32 tiles 8 ways along K; under SP=8 (7410 rows) 580 tiles -> 68 split 3 ways;
    FFN-up (12528 tiles, tail 240), a 136-tile tail at K=5120 (where the partial-tile traffic
    costs more than it saves) and grids below one round are not split."""
    from vstyler import _lib
    lib = _lib.load()
    out = (ctypes.c_int * 4)()
    cases = [((59280, 5120, 5120, 256), (4608, 32, 8, 640)),
             ((59280, 5120, 13824, 256), (4608, 32, 8, 1728)),
             ((7410, 5120, 5120, 256), (512, 68, 3, 1728)),
             ((59280, 13824, 5120, 256), (12528, 0, 1, 0)),
             ((14820, 5120, 5120, 256), (1160, 0, 1, 0)),
             ((1024, 1024, 4096, 256), (16, 0, 1, 0)),
             ((59280, 5120, 5120, 0), (4640, 0, 1, 0))]
    for args, want in cases:
        assert lib.vs_gemm_split_plan(*args, out) == 0
        assert tuple(out) == want, (args, tuple(out))
        nmain, ntail, ks, pk = want
        if ntail:
            assert pk % 32 == 0 and (ks - 1) * pk < args[2] <= ks * pk
    assert lib.vs_gemm_split_plan(64, 64, 100, 256, out) == 1


def test_gemm_route_is_fused_everywhere():
    """r5: every GEMM of the product library runs on the MFMA kernels with its epilogue fused
    (gemm.hip 'Routing (r5)'): vs_gemm_route / vs_gemm_route_epi answer 0 for every shape, epilogue
    and dtype, and reject bad arguments; the library needs no vendor-library workspace (kinds 2, 3:
    0 bytes) and reads no environment variable."""
    from vstyler import _lib
    lib = _lib.load()
    for m, n, k in ((59280, 15360, 5120), (59280, 13824, 5120), (59280, 5120, 13824), (7410, 15360, 5120),
                    (1024, 10240, 4096), (2, 30720, 5120), (64, 64, 64)):
        assert lib.vs_gemm_route(m, n, k) == 0
        for epi in range(5):
            assert lib.vs_gemm_route_epi(m, n, k, epi, 0) == 0
            assert lib.vs_gemm_route_epi(m, n, k, epi, 1) == 0
    assert lib.vs_gemm_route(0, 1, 1) < 0 or lib.vs_gemm_route(0, 1, 1) == 1
    assert lib.vs_gemm_route_epi(59280, 5120, 5120, 9, 0) < 0
    assert lib.vs_split_workspace_bytes(2) == 0 and lib.vs_split_workspace_bytes(3) == 0
    assert lib.vs_split_workspace_bytes(5) >= 1280
    so = open(_lib.LIB_PATH, "rb").read()
    assert b"libhipblaslt" not in so and b"VS_GEMM_BACKEND" not in so and b"getenv" not in so


def test_options_table():
    """vs_set_option / vs_get_option (include/vstyler.h): product defaults, range checks, the previous
    value returned, and kernels.options() restoring the table."""
    from vstyler import _lib, kernels as K
    lib = _lib.load()
    defaults = {"gemm_tile": 0, "gemm_kernel": 4, "gemm_split": 1, "queue": 1, "attn_impl": 0,
                "attn_mfma": 16, "attn_nc": 1, "attn_split": 1, "attn_persist": 1, "vae_pxb": 2, "vae_pre": 3,
                "vae_halo": 1, "piece_queue": 1}
    assert set(defaults) == set(_lib.OPTIONS)
    for name, v in defaults.items():
        assert K.get_option(name) == v, name
    with K.options(gemm_kernel=8, queue=0, attn_mfma=32):
        assert (K.get_option("gemm_kernel"), K.get_option("queue"), K.get_option("attn_mfma")) == (8, 0, 32)
    assert (K.get_option("gemm_kernel"), K.get_option("queue"), K.get_option("attn_mfma")) == (4, 1, 16)
    for name, bad in (("gemm_tile", 64), ("gemm_kernel", 5), ("attn_mfma", 8), ("vae_pre", 4), ("gemm_split", 2),
                      ("piece_queue", 3)):
        with pytest.raises(ValueError):
            K.set_option(name, bad)
    assert lib.vs_set_option(99, 0) < 0 and lib.vs_get_option(-1) < 0


def test_built_library_passes_isa_guards():
    """the accumulator-copy guard of scripts/check_isa.py (run by `make` on gemm.o)
    holds for the gfx950 code objects inside the shipped libvstyler.so: every 4-wave GEMM
    instantiation reads its accumulators only through acc_rd (no v_accvgpr_write / mov), 512 reads,
    no scratch, one returning tile-queue atomic."""
    import subprocess
    import sys
    from vstyler import _lib
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py"), _lib.LIB_PATH],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "13 gemm_*_4w kernels OK" in r.stdout
