"""GPU parity of the VACE conditioning unit (WanVideoUnit_VACE, wan_video_new.py:861-920) and of the
whole Ditto call (VACE encode -> CFG denoise -> tiled decode -> uint8 frames) against the oracle chain.

Bit-exact: preprocessing + inactive/reactive split and the mask latents (pure bf16 elementwise /
index work).  Encoded latents: within 1.5x the oracle's fp32-vs-fp64 noise floor.  End-to-end
uint8 frames: the two bf16 pipelines (40+ rounding layers) agree to a few code values; bounds in
the test."""
import numpy as np
import pytest
import torch

from gpu_util import err
from oracle import wan_oracle as O
from oracle import wan_vae_oracle as V
from test_model_gpu import build
from vae_util import TINY_VAE

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16
TS, ST = (4, 6), (2, 3)


def _frames(t, h, w, seed, binary=False):
    g = torch.Generator().manual_seed(seed)
    if binary:
        f = (torch.rand((t, h, w, 1), generator=g) > 0.5).to(torch.uint8) * 255
        return f.expand(t, h, w, 3).contiguous()
    return torch.randint(0, 256, (t, h, w, 3), generator=g, dtype=torch.uint8)


def _vae_model(W):
    from vstyler import vae
    return vae.WanVideoVAE(z_dim=16, dim=TINY_VAE["dim"], device="cuda").load_state_dict(W)


def test_vace_prepare_and_mask_latents_bit_exact():
    from vstyler import _lib
    T, H, W = 9, 64, 96
    video, mask = _frames(T, H, W, 1), _frames(T, H, W, 2)
    v = V.preprocess_video(video)
    m = V.preprocess_video(mask, 0, 1)
    ref_in = v * (1 - m) + 0 * m
    ref_re = v * m + 0 * (1 - m)
    inact = torch.empty((1, 3, T, H, W), dtype=BF16, device="cuda")
    react = torch.empty_like(inact)
    mask0 = torch.empty((T, H, W), dtype=BF16, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    lib = _lib.load()
    vd, md = video.cuda(), mask.cuda()
    _lib.check(lib.vs_vace_prepare(vd.data_ptr(), md.data_ptr(), inact.data_ptr(), react.data_ptr(),
                                   mask0.data_ptr(), T, H, W, st))
    assert torch.equal(inact.cpu(), ref_in) and torch.equal(react.cpu(), ref_re)
    assert torch.equal(mask0.cpu(), m[0, 0])
    t_lat = (T + 3) // 4
    out = torch.empty((64, t_lat, H // 8, W // 8), dtype=BF16, device="cuda")
    _lib.check(lib.vs_vace_mask_latents(mask0.data_ptr(), out.data_ptr(), T, H, W, t_lat, st))
    mm = m[0, 0].reshape(T, H // 8, 8, W // 8, 8).permute(2, 4, 0, 1, 3).reshape(1, 64, T, H // 8, W // 8)
    mref = torch.nn.functional.interpolate(mm, size=(t_lat, H // 8, W // 8), mode="nearest-exact")
    assert torch.equal(out.cpu(), mref[0])
    # defaults: no video -> zeros, no mask -> ones
    _lib.check(lib.vs_vace_prepare(None, None, inact.data_ptr(), react.data_ptr(), mask0.data_ptr(), T, H, W, st))
    assert not inact.any() and not react.any() and bool((mask0 == 1).all())


@pytest.mark.parametrize("with_mask", [False, True])
def test_vace_context_vs_oracle(with_mask):
    from vstyler.vae import vace_context
    Wv = V.random_vae_weights(TINY_VAE, seed=31)
    T, H, W = 9, 64, 96
    video = _frames(T, H, W, 3)
    mask = _frames(T, H, W, 4, binary=True) if with_mask else None
    vin = V.preprocess_video(video)
    min_ = None if mask is None else V.preprocess_video(mask, 0, 1)

    def ref_fn():
        return V.vace_context(Wv, vin, min_, tiled=True, tile_size=TS, tile_stride=ST, cfg=TINY_VAE)

    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    r64 = ref_fn()
    O.ACC_DTYPE = old
    ref = ref_fn()
    got = vace_context(_vae_model(Wv), video, mask, tiled=True, tile_size=TS, tile_stride=ST)
    assert got.shape == ref.shape == (1, 96, 3, 8, 12)
    assert torch.equal(got[:, 32:].cpu(), ref[:, 32:])
    fmx, frel = err(r64[:, :32], ref[:, :32])
    mx, rel = err(got[:, :32], ref[:, :32])
    print(f"vace_context latents: max-abs {mx:.4g} rel-L2 {rel:.4g} (floor {fmx:.4g} / {frel:.4g})")
    assert rel <= 1.5 * frel + 1e-3 and mx <= 1.5 * fmx + 1e-2


@pytest.mark.parametrize("nref", [1, 2])
def test_vace_context_reference_images_vs_oracle(nref):
    """WanVideoUnit_VACE.process with vace_reference_image (wan_video_new.py:896-912): each reference
    frame encoded as its own video -- the second one with the reference's compounded x8 tile size
    (wan_video_vae.py:1224-1225) -- and prepended along time; mask latents get zero frames."""
    from vstyler.vae import vace_context
    Wv = V.random_vae_weights(TINY_VAE, seed=33)
    T, H, W = 5, 64, 96
    video = _frames(T, H, W, 6)
    refs = _frames(nref, H, W, 7)
    vin = V.preprocess_video(video)
    rin = V.preprocess_video(refs)

    def ref_fn():
        return V.vace_context(Wv, vin, None, tiled=True, tile_size=TS, tile_stride=ST, cfg=TINY_VAE,
                              vace_reference_image=rin)

    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    r64 = ref_fn()
    O.ACC_DTYPE = old
    ref = ref_fn()
    got = vace_context(_vae_model(Wv), video, None, tiled=True, tile_size=TS, tile_stride=ST,
                       vace_reference_image=[f.numpy() for f in refs])
    assert got.shape == ref.shape == (1, 96, nref + 2, 8, 12)
    assert torch.equal(got[:, 16:32, :nref].cpu(), ref[:, 16:32, :nref]) and not got[:, 16:32, :nref].any()
    assert torch.equal(got[:, 32:].cpu(), ref[:, 32:])
    fmx, frel = err(r64[:, :32], ref[:, :32])
    mx, rel = err(got[:, :32], ref[:, :32])
    print(f"vace_context + {nref} ref: max-abs {mx:.4g} rel-L2 {rel:.4g} (floor {fmx:.4g} / {frel:.4g})")
    assert rel <= 1.5 * frel + 1e-3 and mx <= 1.5 * fmx + 1e-2


def test_pipeline_reference_image_latents():
    """__call__ with vace_reference_image: rolled noise over T'+1 latent frames, the reference frame
    dropped after denoising (wan_video_new.py:545-550, 578-587)."""
    from vstyler import WanVideoPipeline
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    Wv = V.random_vae_weights(TINY_VAE, seed=34)
    T, H, Wd = 5, 64, 96
    video, refimg = _frames(T, H, Wd, 8), _frames(1, H, Wd, 9)
    _, cp, cn, _ = O.synthetic_inputs(cfg, T, H, Wd)
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = build(cfg, W)
    pipe.vae = _vae_model(Wv)
    got = pipe(prompt_emb=cp, negative_prompt_emb=cn, vace_video=list(video.numpy()),
               vace_reference_image=refimg[0].numpy(), seed=3, height=H, width=Wd, num_frames=T,
               num_inference_steps=2, tile_size=TS, tile_stride=ST, output_type="latents")
    t_lat = (T - 1) // 4 + 1
    assert got.shape == (1, 16, t_lat, H // 8, Wd // 8)

    def chain():
        vc = V.vace_context(Wv, V.preprocess_video(video), None, tiled=True, tile_size=TS, tile_stride=ST,
                            cfg=TINY_VAE, vace_reference_image=V.preprocess_video(refimg))
        lat = O.generate_noise((1, 16, t_lat + 1, H // 8, Wd // 8), 3)
        lat = torch.cat((lat[:, :, -1:], lat[:, :, :-1]), dim=2)
        return O.denoise(W, cfg, lat, cp, cn, vc, num_inference_steps=2)[:, :, 1:]

    ref = chain()
    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    ref64 = chain()
    O.ACC_DTYPE = old
    fmx, frel = err(ref64, ref)
    mx, rel = err(got, ref)
    print(f"ref-image latents: max-abs {mx:.4g} rel-L2 {rel:.4g} (floor {fmx:.4g} / {frel:.4g})")
    assert rel <= 1.5 * frel + 2e-3 and mx <= 1.5 * fmx + 2e-2


def test_pipeline_end_to_end_tiny():
    """WanVideoPipeline.__call__(vace_video=PIL frames, ...) -> PIL frames, vs the oracle chain."""
    from PIL import Image

    from vstyler import WanVideoPipeline
    cfg = O.WAN_CONFIGS["tiny"]
    W = O.random_weights(cfg, seed=5)
    Wv = V.random_vae_weights(TINY_VAE, seed=32)
    T, H, Wd = 9, 64, 96
    video = _frames(T, H, Wd, 5)
    _, cp, cn, _ = O.synthetic_inputs(cfg, T, H, Wd)
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = build(cfg, W)
    pipe.vae = _vae_model(Wv)
    frames = pipe(prompt_emb=cp, negative_prompt_emb=cn, vace_video=[Image.fromarray(f.numpy()) for f in video],
                  seed=1, height=H, width=Wd, num_frames=T, num_inference_steps=2, tile_size=TS, tile_stride=ST)
    assert len(frames) == T and frames[0].size == (Wd, H)
    got = torch.from_numpy(np.stack([np.asarray(f) for f in frames]))
    def chain():  # the oracle chain
        vc = V.vace_context(Wv, V.preprocess_video(video), None, tiled=True, tile_size=TS, tile_stride=ST,
                            cfg=TINY_VAE)
        lat = O.generate_noise((1, 16, (T - 1) // 4 + 1, H // 8, Wd // 8), 1)
        lat = O.denoise(W, cfg, lat, cp, cn, vc, num_inference_steps=2)
        return V.vae_output_to_u8(V.tiled_decode(lat, Wv, TS, ST, TINY_VAE))

    ref = chain()
    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    ref64 = chain()
    O.ACC_DTYPE = old
    d = (got.int() - ref.int()).abs().float()
    f = (ref64.int() - ref.int()).abs().float()
    print(f"e2e uint8: mean |d| {d.mean().item():.3f} max {d.max().item():.0f}; oracle fp32-vs-fp64 floor: "
          f"mean {f.mean().item():.3f} max {f.max().item():.0f}")
    assert d.mean().item() <= 1.5 * f.mean().item() + 0.1 and d.max().item() <= 2 * f.max().item() + 4


def test_teacache_decisions_and_latents_vs_oracle():
    """TeaCache (wan_video_new.py:1154-1203): same skip decisions as the restated reference cache and
    latents within the fp32/fp64 noise floor.  The tiny random model's t_mod changes ~50 % per step
    (real checkpoints: a few %); a +0.25 shift of the time_projection bias brings the relative L1 to
    ~1.5-1.9 % per step, where the T2V-1.3B polynomial gives ~0.07 per step, and th = 0.2 then
    computes every third step: [T, F, F, T, F, F, T, T] with >= 0.016 margin at every decision."""
    from vstyler import WanVideoPipeline
    from vstyler.teacache import TeaCache
    cfg = O.WAN_CONFIGS["tiny"]
    W = dict(O.random_weights(cfg, seed=5))
    W["time_projection.1.bias"] = (W["time_projection.1.bias"].float() + 0.25).to(BF16)
    T, H, Wd = 5, 64, 96
    lat0, cp, cn, vc = O.synthetic_inputs(cfg, T, H, Wd)
    n, th, mid = 8, 0.2, "Wan2.1-T2V-1.3B"

    def oracle():
        caches = (O.TeaCacheOracle(n, th, mid), O.TeaCacheOracle(n, th, mid))
        out = O.denoise(W, cfg, lat0.clone(), cp, cn, vc, num_inference_steps=n, tea_caches=caches)
        assert caches[0].decisions == caches[1].decisions
        return out, caches[0].decisions

    ref, dec = oracle()
    assert dec == [True, False, False, True, False, False, True, True], dec
    pipe = WanVideoPipeline(device="cuda")
    pipe.dit, pipe.vace = build(cfg, W)
    tc = TeaCache(n, th, mid)
    got = pipe.denoise(lat0.cuda(), cp.cuda(), cn.cuda(), vc.cuda(), num_inference_steps=n, tea_cache=tc)
    assert tc.decisions == dec, (tc.decisions, dec)
    old = O.ACC_DTYPE
    O.ACC_DTYPE = torch.float64
    ref64, _ = oracle()
    O.ACC_DTYPE = old
    fmx, frel = err(ref64, ref)
    mx, rel = err(got, ref)
    print(f"teacache th={th} decisions {dec}: max-abs {mx:.4g} rel-L2 {rel:.4g} (floor {fmx:.4g} / {frel:.4g})")
    assert rel <= 1.5 * frel + 2e-3 and mx <= 1.5 * fmx + 2e-2
