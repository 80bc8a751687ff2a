"""The oracle reproduces the committed golden fixtures (tests/golden/make_golden.py)."""
import os

import numpy as np
import torch

from oracle import wan_oracle as O

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bf(a):
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


def test_ops_fixture():
    z = np.load(os.path.join(HERE, "ops.npz"))
    q, k, v = bf(z["q"]), bf(z["k"]), bf(z["v"])
    o = O.attention(q, k, v, 2)
    assert (o.float() - bf(z["attn"]).float()).abs().max() <= 2 ** -7
    x, w = bf(z["x"]), bf(z["w"])
    rn = O.rope_apply(O.rms_norm(x.view(2, 300, 256), w), O.rope_freqs(3, 10, 10), 2)
    assert (rn.float() - bf(z["rmsnorm_rope"]).float()).abs().max() <= 2 ** -6


def test_tiny_denoise_fixture():
    z = np.load(os.path.join(HERE, "tiny_2step.npz"))
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    lat, cp, cn, vc = O.synthetic_inputs(cfg, 5, 128, 128)
    assert torch.equal(lat, bf(z["latents_in"]).view(lat.shape))
    out = O.denoise(W, cfg, lat, cp, cn, vc, num_inference_steps=2)
    ref = bf(z["latents_out"]).view(out.shape)
    assert (out.float() - ref.float()).abs().max() <= 2 ** -5
