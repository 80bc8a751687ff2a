"""The oracle against the reference's own known-answer constants.

The reference has no golden vectors; these KATs pin the oracle's structure: the md5 key-layout
hashes from diffsynth/configs/model_config.py:142-179 (+ wan_video_dit.py:509,523,
wan_video_vace.py:100) and the closed-form flow-matching schedule (schedulers/flow_match.py:34-58).
"""
import math

import torch

from oracle import wan_oracle as O


def test_dit_key_layout_hashes_match_reference():
    assert O.hash_state_dict_keys(O.dit_param_shapes(O.WAN_CONFIGS["1.3B"])) == "9269f8db9040a9d860eaca435be61814"
    assert O.hash_state_dict_keys(O.dit_param_shapes(O.WAN_CONFIGS["14B"])) == "aafcfd9672c3a2456dc46e1cb6e52c70"


def test_vace_key_layout_hashes_match_reference():
    assert O.hash_state_dict_keys(O.vace_param_shapes(O.WAN_CONFIGS["14B"])) == "3b2726384e4f64837bdf216eea3f310d"
    # combined DiT+VACE single-file hashes registered for (WanModel, VaceWanModel) (model_config.py:157-158)
    registered = {"a61453409b67cd3246cf0c3bebad47ba", "7a513e1f257a861512b1afd387a8ecd9"}
    for name in ("1.3B", "14B"):
        c = O.WAN_CONFIGS[name]
        both = dict(O.dit_param_shapes(c))
        both.update(O.vace_param_shapes(c))
        assert O.hash_state_dict_keys(both) in registered


def test_product_model_keys_equal_oracle_layout():
    from vstyler.models import VaceWanModel, WanModel
    c = dict(O.WAN_CONFIGS["1.3B"])
    dit = WanModel(dim=c["dim"], in_dim=16, ffn_dim=c["ffn_dim"], out_dim=16, text_dim=4096, freq_dim=256, eps=1e-6,
                   patch_size=(1, 2, 2), num_heads=c["num_heads"], num_layers=c["num_layers"], device="meta")
    shapes = {k: tuple(v.shape) for k, v in dit.state_dict().items()}
    assert O.hash_state_dict_keys(shapes) == "9269f8db9040a9d860eaca435be61814"
    vace = VaceWanModel(vace_layers=c["vace_layers"], dim=c["dim"], num_heads=c["num_heads"], ffn_dim=c["ffn_dim"],
                        device="meta")
    vs = {k: tuple(v.shape) for k, v in vace.state_dict().items()}
    both = dict(shapes)
    both.update(vs)
    assert O.hash_state_dict_keys(both) == "a61453409b67cd3246cf0c3bebad47ba"


def test_sigma_schedule_closed_form():
    for n in (2, 4, 50):
        sig, ts = O.set_timesteps(n, shift=5.0)
        for i in range(n):
            s = 1.0 - i / n
            assert math.isclose(float(sig[i]), 5 * s / (1 + 4 * s), rel_tol=0, abs_tol=2e-7)
        assert torch.allclose(ts, sig * 1000)
        assert float(O.euler_delta(sig, n - 1)) == -float(sig[-1])


def test_sinusoid_and_rope_tables():
    t = torch.tensor([1000.0]).to(torch.bfloat16)
    e = O.sinusoidal_embedding_1d(256, t)
    assert e.shape == (1, 256) and e.dtype == torch.bfloat16
    assert float(e[0, 0]) == 1.0 or abs(float(e[0, 0]) - math.cos(1000.0)) < 1e-2
    tf, th, tw = O.rope_tables(128)
    assert tf.shape == (1024, 22) and th.shape == (1024, 21) and tw.shape == (1024, 21)
    f = O.rope_freqs(2, 3, 4)
    assert f.shape == (24, 1, 64)
    # token (f=1,h=2,w=3) -> pairs 0..21 use position 1, 22..42 position 2, 43..63 position 3
    tok = 1 * 12 + 2 * 4 + 3
    assert torch.allclose(f[tok, 0, :22], tf[1]) and torch.allclose(f[tok, 0, 22:43], th[2])
    assert torch.allclose(f[tok, 0, 43:], tw[3])


def test_unpatchify_inverts_patchify_layout():
    lat = torch.randn(2, 16, 3, 8, 6).to(torch.bfloat16)
    D = 64
    eye = torch.eye(D).reshape(D, 16, 1, 2, 2).to(torch.bfloat16)   # identity conv: token = im2col
    tok, grid = O.patchify(lat, eye, torch.zeros(D, dtype=torch.bfloat16))
    # im2col column order c*4+kh*2+kw; head/unpatchify order (y*2+z)*16+c
    perm = torch.tensor([c * 4 + y * 2 + z for y in range(2) for z in range(2) for c in range(16)])
    back = O.unpatchify(tok[..., perm], grid, 16)
    assert torch.equal(back, lat)


def test_t5_key_layout_matches_reference_registry():
    """configs/model_config.py:161: the Wan UMT5-XXL text encoder file's md5 key hash."""
    from oracle import t5_oracle as T
    assert O.hash_state_dict_keys(T.t5_param_shapes()) == "9c8818c2cbea55eca56c7b447df170da"


def test_t5_relative_position_buckets():
    from oracle import t5_oracle as T
    b = T.relative_position_bucket(512, 512)
    assert b.min() == 0 and b.max() == 31
    assert b[0, 0] == 0 and b[0, 1] == 17 and b[1, 0] == 1 and b[0, 7] == 23 and b[7, 0] == 7
    assert b[0, 511] == 31 and b[511, 0] == 15


def test_loader_normalizes_comfyui_kijai_layouts():
    """loader.normalize_keys: 'model.diffusion_model.' / 'diffusion_model.' prefixes stripped, fp8
    weights with '.scale_weight' folded (exact upcast, then the scale), so the reference's md5
    key-layout hash of the stripped file equals the plain layout's."""
    import torch
    from vstyler.loader import hash_state_dict_keys, normalize_keys
    w8 = torch.tensor([[1.5, -2.0], [0.25, 448.0]]).to(torch.float8_e4m3fn)
    plain = {"blocks.0.self_attn.q.weight": torch.zeros(2, 2), "head.head.bias": torch.zeros(2)}
    comfy = {"model.diffusion_model.blocks.0.self_attn.q.weight": w8,
             "model.diffusion_model.blocks.0.self_attn.q.scale_weight": torch.tensor(0.5),
             "model.diffusion_model.head.head.bias": torch.zeros(2), "scaled_fp8": torch.zeros(1)}
    n = normalize_keys(comfy)
    assert set(n) == set(plain)
    assert hash_state_dict_keys(n) == hash_state_dict_keys(plain)
    assert torch.equal(n["blocks.0.self_attn.q.weight"].float(), w8.float() * 0.5)
    assert set(normalize_keys({"diffusion_model.x.weight": torch.zeros(1)})) == {"x.weight"}


def test_loader_configs_from_shapes_and_shards(tmp_path):
    """loader.dit/vace_config_from_shapes (the extension for key hashes outside the reference's
    table) reproduce the published configs from the 1.3B / 14B layouts, and a tiny checkpoint split
    over two safetensors shards reads back as one state dict with the tiny config."""
    from safetensors.torch import save_file
    from vstyler.loader import (WAN_DIT_CONFIGS, dit_config_from_shapes, load_state_dict,
                                vace_config_from_shapes)

    def meta(shapes):
        return {k: torch.empty(s, device="meta") for k, s in shapes.items()}
    for name in ("1.3B", "14B", "tiny"):
        cfg = O.WAN_CONFIGS[name]
        d = dit_config_from_shapes(meta(O.dit_param_shapes(cfg)))
        for k in ("dim", "ffn_dim", "num_heads", "num_layers", "in_dim", "out_dim", "text_dim", "freq_dim"):
            assert d[k] == cfg[k], (name, k)
        v = vace_config_from_shapes(meta(O.vace_param_shapes(cfg)), cfg["num_layers"])
        assert v["vace_layers"] == tuple(cfg["vace_layers"]) and v["dim"] == cfg["dim"], name
        assert v["ffn_dim"] == cfg["ffn_dim"] and v["vace_in_dim"] == cfg["vace_in_dim"], name
    assert dit_config_from_shapes({"head.head.weight": torch.zeros(64, 8)}) is None
    assert len(WAN_DIT_CONFIGS) == 2
    W = O.random_weights(O.WAN_CONFIGS["tiny"], seed=3)
    keys = sorted(W)
    save_file({k: W[k] for k in keys[0::2]}, str(tmp_path / "a-00001-of-00002.safetensors"))
    save_file({k: W[k] for k in keys[1::2]}, str(tmp_path / "a-00002-of-00002.safetensors"))
    sd = load_state_dict([str(tmp_path / "a-00001-of-00002.safetensors"),
                          str(tmp_path / "a-00002-of-00002.safetensors")])
    assert set(sd) == set(W) and all(torch.equal(sd[k], W[k]) for k in W)


def test_model_fn_rows_matches_full_model_fn():
    """O.model_fn_rows (the C4 GPU test's oracle: a one-block pair evaluated at sampled token rows,
    keys / values from every row) equals O.model_fn at those rows, tiny config on the CPU (up to the
    GEMM's row-blocking order: a bf16 ulp here and there)."""
    cfg = dict(O.WAN_CONFIGS["tiny"], num_layers=1, vace_layers=(0,))
    W = O.random_weights(cfg, seed=9)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 9, 64, 96)
    t = torch.tensor([600.0, 600.0]).to(torch.bfloat16)
    ctx = torch.cat([cp, cn])
    full = O.patchify_output(O.model_fn(W, cfg, torch.cat([lat, lat]), t, ctx, torch.cat([vc, vc]), vace_scale=0.9))
    S = full.shape[1]
    rows = torch.tensor([0, 5, 47, 48, S // 2, S - 1])
    got = O.model_fn_rows(W, cfg, torch.cat([lat, lat]), t, ctx, torch.cat([vc, vc]), rows, vace_scale=0.9)
    ref = full[:, rows]
    d = (got.float() - ref.float())
    assert got.shape == ref.shape
    assert (d.norm() / ref.float().norm()).item() < 2e-3 and d.abs().max().item() < 2e-2
    # patchify_output inverts unpatchify
    x = torch.randn(2, 3 * 4 * 16).view(2, 3, 64).to(torch.bfloat16)
    assert torch.equal(O.patchify_output(O.unpatchify(x.view(2, 3, 64), (3, 1, 1))), x)
