"""diffsynth.pipelines.wan_video_new -> vstyler (MI355X kernels)."""
from vstyler.pipeline import ModelConfig, WanVideoPipeline, model_fn_wan_video  # noqa: F401
from vstyler.flow_match import FlowMatchScheduler  # noqa: F401
