"""GPU parity of the UMT5 text encoder (vstyler/t5.py + csrc/t5.hip) against the oracle restatement
(oracle/t5_oracle.py) at a scaled-down shape (head_dim 64 like UMT5-XXL), within 1.5x the oracle's
own fp32-vs-fp64 noise floor; padded rows must be exactly zero as in WanPrompter.encode_prompt."""
import pytest
import torch

from gpu_util import err
from oracle import t5_oracle as T
from oracle import wan_oracle as O

pytestmark = pytest.mark.gpu
TINY_T5 = dict(vocab=1000, dim=256, dim_attn=256, dim_ffn=512, num_heads=4, num_layers=2, num_buckets=32)


def _inputs(lengths, L=64, seed=3):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, TINY_T5["vocab"], (len(lengths), L), generator=g)
    mask = torch.zeros(len(lengths), L, dtype=torch.long)
    for b, n in enumerate(lengths):
        mask[b, :n] = 1
        ids[b, n:] = 0
    return ids, mask


@pytest.mark.parametrize("lengths", [(40,), (64,), (17, 51)])
def test_t5_encode_tiny_vs_oracle(lengths):
    from vstyler.t5 import WanPrompter, WanTextEncoder
    W = T.random_t5_weights(TINY_T5, seed=9)
    ids, mask = _inputs(lengths)
    ref = T.t5_encode(ids, mask, W, TINY_T5)
    old = O.ACC_DTYPE
    try:
        O.ACC_DTYPE = torch.float64
        ref64 = T.t5_encode(ids, mask, W, TINY_T5)
    finally:
        O.ACC_DTYPE = old
    enc = WanTextEncoder(**TINY_T5, device="cuda").load_state_dict(W)
    pr = WanPrompter()
    pr.fetch_models(enc)
    got = pr.encode_ids(ids, mask)
    assert got.shape == ref.shape
    n = min(lengths)
    assert not got[:, n:].any()
    fmx, frl = err(ref64, ref)
    mx, rl = err(got, ref)
    print(f"T5 tiny {lengths}: max-abs {mx:.4g} rel-L2 {rl:.4g} (floor {fmx:.4g} / {frl:.4g})")
    assert rl <= 1.5 * frl + 2e-3 and mx <= 1.5 * fmx + 3e-2
