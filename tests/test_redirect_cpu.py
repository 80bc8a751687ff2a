"""from_pretrained over a ./models tree laid out the way the reference's downloads leave it
(VERDICT r3 next-step 1).  infer_ditto.py:15-19 asks for the T5 and VAE files under
model_id "Wan-AI/Wan2.1-VACE-14B", and WanVideoPipeline.from_pretrained rewrites those two
model_ids to "Wan-AI/Wan2.1-T2V-1.3B" before resolving files (redirect_common_files=True,
wan_video_new.py:352-363), where ModelScope put them.  Tiny-width tensors in the reference key
layouts; everything stays on the CPU (loading only, no kernels run)."""
import pytest
import torch

from oracle import wan_oracle as O

BF16 = torch.bfloat16
VACE_ID, COMMON_ID = "Wan-AI/Wan2.1-VACE-14B", "Wan-AI/Wan2.1-T2V-1.3B"


def infer_ditto_configs(ModelConfig):
    """inference/infer_ditto.py:15-19, verbatim."""
    return [
        ModelConfig(model_id="Wan-AI/Wan2.1-VACE-14B", origin_file_pattern="diffusion_pytorch_model*.safetensors", offload_device="cpu"),
        ModelConfig(model_id="Wan-AI/Wan2.1-VACE-14B", origin_file_pattern="models_t5_umt5-xxl-enc-bf16.pth", offload_device="cpu"),
        ModelConfig(model_id="Wan-AI/Wan2.1-VACE-14B", origin_file_pattern="Wan2.1_VAE.pth", offload_device="cpu"),
    ]


def tiny_t5_state_dict(seed=3):
    from vstyler.t5 import WanTextEncoder
    te = WanTextEncoder(vocab=512, dim=128, dim_attn=128, dim_ffn=256, num_heads=2, num_layers=2, device="cpu")
    g = torch.Generator().manual_seed(seed)
    return {k: (0.02 * torch.randn(shape, generator=g)).to(BF16) for k, shape in te.state_dict_shapes().items()}


def tiny_vae_state_dict(seed=4):
    from vstyler.vae import WanVideoVAE
    vae = WanVideoVAE(z_dim=16, dim=32, device="cpu")
    g = torch.Generator().manual_seed(seed)
    return {k: (0.02 * torch.randn(shape, generator=g)).to(BF16) for k, shape in vae.state_dict_shapes().items()}


def write_tree(root, common_id=COMMON_ID):
    from safetensors.torch import save_file
    W = O.random_weights(O.WAN_CONFIGS["tiny"], seed=21)
    keys = sorted(W)
    d = root / "models" / VACE_ID
    d.mkdir(parents=True)
    for i in range(2):
        save_file({k: W[k].contiguous() for k in keys[i::2]},
                  str(d / f"diffusion_pytorch_model-0000{i + 1}-of-00002.safetensors"))
    c = root / "models" / common_id
    c.mkdir(parents=True, exist_ok=True)
    torch.save(tiny_t5_state_dict(), str(c / "models_t5_umt5-xxl-enc-bf16.pth"))
    torch.save(tiny_vae_state_dict(), str(c / "Wan2.1_VAE.pth"))
    return W


def test_redirect_loads_reference_download_layout(tmp_path, monkeypatch, capsys):
    from vstyler import ModelConfig, WanVideoPipeline
    W = write_tree(tmp_path)
    monkeypatch.chdir(tmp_path)          # ModelConfig's default local_model_path is "./models"
    pipe = WanVideoPipeline.from_pretrained(torch_dtype=BF16, device="cpu",
                                            model_configs=infer_ditto_configs(ModelConfig))
    out = capsys.readouterr().out
    for f in ("models_t5_umt5-xxl-enc-bf16.pth", "Wan2.1_VAE.pth"):
        assert f"({VACE_ID}, {f}) is redirected to ({COMMON_ID}, {f})" in out
    assert pipe.dit is not None and pipe.vace is not None
    assert pipe.vae is not None and pipe.text_encoder is not None
    assert len(pipe.dit.blocks) == O.WAN_CONFIGS["tiny"]["num_layers"]
    assert torch.equal(pipe.dit.blocks[0].ffn[0].weight.detach().cpu(), W["blocks.0.ffn.0.weight"].to(BF16))
    assert pipe.text_encoder.num_layers == 2 and pipe.text_encoder.dim == 128
    assert pipe.vae.dim == 32 and pipe.vae.z_dim == 16


def test_redirect_rewrites_only_the_common_files():
    from vstyler import ModelConfig
    from vstyler.pipeline import redirect_model_configs
    cfgs = infer_ditto_configs(ModelConfig) + [
        ModelConfig(path="x.safetensors"),
        ModelConfig(model_id="Wan-AI/Wan2.1-T2V-1.3B", origin_file_pattern="Wan2.1_VAE.pth"),
        ModelConfig(model_id="Some/Other", origin_file_pattern=["Wan2.1_VAE.pth"]),
    ]
    redirect_model_configs(cfgs)
    assert [c.model_id for c in cfgs] == [VACE_ID, COMMON_ID, COMMON_ID, None, COMMON_ID, "Some/Other"]


def test_no_redirect_resolves_unredirected_paths(tmp_path, monkeypatch, capsys):
    from vstyler import ModelConfig, WanVideoPipeline
    write_tree(tmp_path, common_id=VACE_ID)      # every file under the VACE model_id
    monkeypatch.chdir(tmp_path)
    pipe = WanVideoPipeline.from_pretrained(torch_dtype=BF16, device="cpu", redirect_common_files=False,
                                            model_configs=infer_ditto_configs(ModelConfig))
    assert "redirected" not in capsys.readouterr().out
    assert pipe.vae is not None and pipe.text_encoder is not None and pipe.dit is not None
    # the same tree with redirection on looks for T5/VAE under the common model_id and finds nothing
    with pytest.raises(FileNotFoundError):
        WanVideoPipeline.from_pretrained(torch_dtype=BF16, device="cpu",
                                         model_configs=infer_ditto_configs(ModelConfig))
