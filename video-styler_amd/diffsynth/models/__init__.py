from vstyler.loader import load_state_dict  # noqa: F401
