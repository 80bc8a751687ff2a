"""Drop-in facade with the reference's module paths (`diffsynth.pipelines.wan_video_new`, ...).
Put `video-styler_amd/` on PYTHONPATH and `inference/infer_ditto.py`-style code imports this build
(`from diffsynth import save_video, VideoData`, `diffsynth/__init__.py` -> `data/`).
Only the Ditto / Wan2.1-VACE path is provided; everything else is out of scope."""
from vstyler import ModelConfig, WanVideoPipeline  # noqa: F401
from .data import VideoData, save_frames, save_video  # noqa: F401
