"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
anything from this package, and only as the checker / CPU baseline.  The product path
(`video-styler_amd/vstyler`) never imports it and fails loudly without its HIP library.

Parity status: numerics are **parity unpinned** -- the reference ships no golden vectors
 and importing/running the reference Python was refused by the
environment (binding).  The restatement is pinned structurally by the
reference's own known-answer constants: the md5 state-dict key-layout hashes
(configs/model_config.py:142-179), the closed-form sigma table (schedulers/flow_match.py:34-69)
and the VAE latent mean/std (models/wan_video_vae.py:1063-1070); see tests/test_oracle_kat.py.
"""
