from vstyler.models import DiTBlock, Head, WanModel  # noqa: F401
