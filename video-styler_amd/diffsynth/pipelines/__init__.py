from vstyler.pipeline import WanVideoPipeline  # noqa: F401
