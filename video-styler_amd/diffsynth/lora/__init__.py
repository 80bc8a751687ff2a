"""diffsynth.lora: GeneralLoRALoader with the reference signature, merging on the GPU GEMM."""
import torch

from vstyler.lora import get_name_dict, merge_lora


class GeneralLoRALoader:
    def __init__(self, device="cpu", torch_dtype=torch.float32):
        self.device = device
        self.torch_dtype = torch_dtype

    def get_name_dict(self, lora_state_dict):
        return get_name_dict(lora_state_dict)

    def load(self, model, state_dict_lora, alpha=1.0):
        return merge_lora(model, state_dict_lora, alpha)
