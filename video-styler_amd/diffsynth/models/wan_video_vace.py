from vstyler.models import VaceWanAttentionBlock, VaceWanModel  # noqa: F401
