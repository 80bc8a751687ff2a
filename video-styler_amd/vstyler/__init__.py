"""vstyler: MI355X-native (gfx950) engine for the Ditto / Wan2.1-VACE denoising path.

Public surface mirrors diffsynth.pipelines.wan_video_new (WanVideoPipeline, ModelConfig,
model_fn_wan_video); kernels live in lib/libvstyler.so (C ABI: include/vstyler.h).
"""
from .flow_match import FlowMatchScheduler
from .models import VaceWanModel, WanModel, init_random_
from .pipeline import ModelConfig, WanVideoPipeline, model_fn_wan_video

__all__ = ["WanVideoPipeline", "ModelConfig", "model_fn_wan_video", "FlowMatchScheduler", "WanModel",
           "VaceWanModel", "init_random_"]
