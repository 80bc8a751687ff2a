"""GPU parity of the UMT5 text encoder (vstyler/t5.py + csrc/t5.hip) against the oracle restatement
(oracle/t5_oracle.py) at a scaled-down shape (head_dim 64 like UMT5-XXL) and at the UMT5-XXL layer
dims (D 4096, 64 heads, FFN 10 240, L 512), within 1.5x the oracle's own fp32-vs-fp64 noise floor;
padded rows must be exactly zero as in WanPrompter.encode_prompt."""
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


# UMT5-XXL dims (wan_video_text_encoder.py:209-219: dim 4096, 64 heads of 64, FFN 10 240, 32 buckets)
# at the prompter's text_len 512, two layers; the vocabulary is cut to 4096 rows (the embedding is a
# row gather, its size changes no arithmetic) so the random weights stay small
XXL_T5 = dict(vocab=4096, dim=4096, dim_attn=4096, dim_ffn=10240, num_heads=64, num_layers=2, num_buckets=32)


@pytest.mark.parametrize("lengths", [(48, 300), (512,)])
def test_t5_encode_xxl_dims_vs_oracle(lengths):
    """UMT5-XXL layer dims at L = 512 (the bucket table, the -inf mask of padded keys over 512
    positions, the 64-head softmax, the gated-GELU FFN) against the oracle within 1.5x its own
    fp32-vs-fp64 floor; the padded rows of each prompt exactly zero (wan_prompter.py:98-109)."""
    from vstyler.t5 import WanPrompter, WanTextEncoder
    torch.set_num_threads(16)
    W = T.random_t5_weights(XXL_T5, seed=11)
    g = torch.Generator().manual_seed(5)
    L = 512
    ids = torch.randint(1, XXL_T5["vocab"], (len(lengths), L), generator=g)
    mask = torch.zeros(len(lengths), L, dtype=torch.long)
    for b, n in enumerate(lengths):
        mask[b, :n] = 1
        ids[b, n:] = 0
    enc = WanTextEncoder(**XXL_T5, device="cuda").load_state_dict(W)
    pr = WanPrompter()
    pr.fetch_models(enc)
    got = pr.encode_ids(ids, mask).cpu()
    ref = T.t5_encode(ids, mask, W, XXL_T5)
    old = O.ACC_DTYPE
    try:
        O.ACC_DTYPE = torch.float64
        ref64 = T.t5_encode(ids, mask, W, XXL_T5)
    finally:
        O.ACC_DTYPE = old
    assert got.shape == ref.shape == (len(lengths), L, 4096)
    n = min(lengths)
    assert not got[:, n:].any()
    fmx, frl = err(ref64, ref)
    mx, rl = err(got, ref)
    print(f"T5 XXL dims {lengths}: max-abs {mx:.4g} rel-L2 {rl:.4g} (floor {fmx:.4g} / {frl:.4g})")
    assert rl <= 1.5 * frl + 2e-3 and mx <= 1.5 * fmx + 3e-2
