"""diffsynth.data.video (VideoData / save_frames / crop_and_resize, reference diffsynth/data/video.py)
on CPU: natural file order, centre crop + resize semantics, round trip through save_frames."""
import os

import numpy as np
import pytest
from PIL import Image


def _img(h, w, seed):
    return Image.fromarray(np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8))


def test_image_folder_natural_order(tmp_path):
    from diffsynth import VideoData
    names = ["f10.png", "f2.png", "f1.png", "f100.jpg", "notes.txt"]
    for i, n in enumerate(names[:-1]):
        _img(8, 12, i).save(tmp_path / n)
    (tmp_path / names[-1]).write_text("x")
    vd = VideoData(image_folder=str(tmp_path))
    assert len(vd) == 4
    assert [os.path.basename(f) for f in vd.data.files] == ["f1.png", "f2.png", "f10.png", "f100.jpg"]
    vd.set_length(2)
    assert len(vd) == 2 and vd.shape() == (8, 12)


@pytest.mark.parametrize("h,w", [(64, 96), (96, 64), (48, 48)])
def test_crop_and_resize_semantics(h, w):
    """Same centre crop arithmetic as video.py:67-80 followed by PIL's resize."""
    from diffsynth.data.video import crop_and_resize
    src = _img(120, 200, 7)
    a = np.asarray(src)
    ih, iw = a.shape[:2]
    if ih / iw < h / w:
        cw = int(ih / h * w)
        ref = a[:, (iw - cw) // 2:(iw - cw) // 2 + cw]
    else:
        ch = int(iw / w * h)
        ref = a[(ih - ch) // 2:(ih - ch) // 2 + ch]
    ref = Image.fromarray(np.ascontiguousarray(ref)).resize((w, h))
    got = crop_and_resize(src, h, w)
    assert got.size == (w, h) and np.array_equal(np.asarray(got), np.asarray(ref))


def test_videodata_resizes_and_save_frames_roundtrip(tmp_path):
    from diffsynth import VideoData, save_frames
    frames = [_img(30, 40, s) for s in range(3)]
    save_frames(frames, str(tmp_path / "out"))
    vd = VideoData(image_folder=str(tmp_path / "out"))
    assert [np.array_equal(np.asarray(vd[i]), np.asarray(frames[i])) for i in range(3)] == [True] * 3
    vd2 = VideoData(image_folder=str(tmp_path / "out"), height=16, width=32)
    assert vd2[0].size == (32, 16)


def test_video_file_without_codec_is_a_clear_error(tmp_path):
    import shutil
    from diffsynth import VideoData
    try:
        import imageio  # noqa: F401
        pytest.skip("imageio present")
    except ImportError:
        pass
    if shutil.which("ffmpeg"):
        pytest.skip("ffmpeg present")
    with pytest.raises(ImportError, match="imageio"):
        VideoData(str(tmp_path / "missing.mp4"))
