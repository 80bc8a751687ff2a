"""CPU tests of the VAE oracle and of the whole-sequence formulation the product runs."""
import pytest
import torch

from oracle import wan_oracle as O
from oracle import wan_vae_oracle as V
from vae_util import TINY_VAE, decode_whole, encode_whole, synthetic_video


def test_vae_key_layout_matches_reference_registry():
    # configs/model_config.py:164 -- the Wan2.1 VAE file's md5 state-dict key hash
    assert O.hash_state_dict_keys(V.vae_param_shapes()) == "ccc42284ea13e1ad04693284c7a09be6"
    assert len(V.vae_param_shapes()) == 194


def test_vae_latent_constants():
    assert len(V.VAE_MEAN) == len(V.VAE_STD) == 16
    assert V.VAE_MEAN[0] == -0.7571 and V.VAE_STD[-1] == 1.9160


def test_tile_tasks_832x480():
    # 832x480 latent 60x104 with the pipeline defaults (30, 52)/(15, 26): a 3x3 grid of full tiles
    tasks = V.tile_tasks(60, 104, (30, 52), (15, 26))
    assert tasks == [(h, h + 30, w, w + 52) for h in (0, 15, 30) for w in (0, 26, 52)]


@pytest.fixture
def fp64_acc():
    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    yield
    O.ACC_DTYPE = old


@pytest.mark.parametrize("frames", [1, 5, 9])
def test_whole_sequence_encode_equals_chunked(fp64_acc, frames):
    W = V.random_vae_weights(TINY_VAE, seed=11)
    x = synthetic_video(frames, 32, 32)
    ref = V.vae_encode(x, W, TINY_VAE)
    got = encode_whole(x, W, TINY_VAE)
    assert ref.shape == got.shape == (1, 16, 1 + (frames - 1) // 4, 4, 4)
    assert torch.equal(ref, got)


@pytest.mark.parametrize("frames", [1, 2, 3])
def test_whole_sequence_decode_equals_chunked(fp64_acc, frames):
    W = V.random_vae_weights(TINY_VAE, seed=12)
    g = torch.Generator().manual_seed(3)
    z = torch.randn((1, 16, frames, 4, 4), generator=g).to(torch.bfloat16)
    ref = V.vae_decode(z, W, TINY_VAE)
    got = decode_whole(z, W, TINY_VAE)
    assert ref.shape == got.shape == (1, 3, 4 * frames - 3, 32, 32)
    assert torch.equal(ref, got)


def test_blend_mask_ramps():
    m = V.build_mask(6, 8, (True, False, False, True), (3, 4))[0, 0, 0]
    assert torch.allclose(m[0], torch.tensor([0.25, 0.5, 0.75, 1, 1, 1, 1, 1]))
    assert torch.allclose(m[:, 7], torch.tensor([1, 1, 1, 1, 2 / 3, 1 / 3]), atol=1e-6)
    assert m[-1].max() <= 1 / 3 + 1e-6


def test_output_to_u8_rounding():
    v = torch.tensor([-1.0, -0.99, 0.0, 0.5, 1.0]).to(torch.bfloat16).view(1, 1, 1, 1, 5).expand(1, 3, 1, 1, 5)
    u = V.vae_output_to_u8(v)
    assert u.shape == (1, 1, 5, 3)
    assert u[0, 0, :, 0].tolist() == [0, 1, 127, 191, 255]


def test_product_vae_layout_matches_oracle():
    """The product's own state-dict layout (used for synthetic weights) is the reference file's."""
    import vstyler.vae as PV
    m = PV.WanVideoVAE.__new__(PV.WanVideoVAE)
    m.z_dim, m.dim, m.dim_mult, m.nrb = 16, 96, (1, 2, 4, 4), 2
    m.temperal_downsample = (False, True, True)
    m.enc_layers, m.enc_dims = m._encoder_layers()
    m.dec_layers, m.dec_dims = m._decoder_layers()
    assert m.state_dict_shapes() == V.vae_param_shapes()
