from .video import VideoData, crop_and_resize, save_frames, save_video  # noqa: F401
