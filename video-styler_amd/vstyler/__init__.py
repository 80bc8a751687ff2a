"""vstyler: MI355X-native (gfx950) engine for the Ditto / Wan2.1-VACE denoising path.

Public surface mirrors diffsynth.pipelines.wan_video_new (WanVideoPipeline, ModelConfig,
model_fn_wan_video); kernels live in lib/libvstyler.so (C ABI: include/vstyler.h).
"""
import os

from .flow_match import FlowMatchScheduler
from .models import VaceWanModel, WanModel, init_random_
from .pipeline import ModelConfig, WanVideoPipeline, model_fn_wan_video

if os.environ.get("VSTYLER_OPTS"):     # path selection for a whole A/B run (kernels.apply_env_options;
    # host option names: vstyler.options, the rest libvstyler's VS_OPT_*)
    from .kernels import apply_env_options
    apply_env_options()

__all__ = ["WanVideoPipeline", "ModelConfig", "model_fn_wan_video", "FlowMatchScheduler", "WanModel",
           "VaceWanModel", "init_random_"]
