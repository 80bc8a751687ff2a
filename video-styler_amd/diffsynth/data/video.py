"""diffsynth.data.video: the reference's video I/O surface (diffsynth/data/video.py:9-145) --
VideoData (a video file or an image folder, frames centre-cropped to the target aspect and
resized), save_video and save_frames.  Host-side I/O, not the hot path: the frames these return
go to WanVideoPipeline(vace_video=...), whose VACE unit moves them to the GPU as uint8.

Container decode/encode needs a codec library.  The reference uses imageio(-ffmpeg); this build
uses imageio when it is importable, else the `ffmpeg` executable when it is on PATH, else raises
an ImportError naming both (image folders and save_frames need only PIL)."""
import os
import re
import shutil
import subprocess

import numpy as np
from PIL import Image

__all__ = ["VideoData", "save_video", "save_frames", "crop_and_resize", "search_for_images"]


def _natural_key(name):
    """split_file_name (video.py:24-40): digit runs compare as integers, everything else per
    character.  Tagged so that names the reference cannot compare (int vs str at one position)
    still sort; names it can compare keep its order."""
    return tuple((0, int(tok), "") if tok.isdigit() else (1, 0, tok)
                 for tok in re.findall(r"\d+|\D", name))


def search_for_images(folder):
    """search_for_images (video.py:43-48): *.jpg / *.png in natural order."""
    names = [n for n in os.listdir(folder) if n.endswith(".jpg") or n.endswith(".png")]
    return [os.path.join(folder, n) for n in sorted(names, key=_natural_key)]


def crop_and_resize(image, height, width):
    """crop_and_resize (video.py:67-80): centre crop to height:width, then PIL resize (default
    resampling filter, as the reference calls it)."""
    a = np.asarray(image)
    ih, iw = a.shape[0], a.shape[1]
    if ih / iw < height / width:
        cw = int(ih / height * width)
        x0 = (iw - cw) // 2
        a = a[:, x0:x0 + cw]
    else:
        ch = int(iw / width * height)
        y0 = (ih - ch) // 2
        a = a[y0:y0 + ch, :]
    return Image.fromarray(np.ascontiguousarray(a)).resize((width, height))


class _ImageFolder:
    def __init__(self, folder, file_list=None):
        self.files = search_for_images(folder) if file_list is None else [os.path.join(folder, f) for f in file_list]

    def __len__(self):
        return len(self.files)

    def __getitem__(self, i):
        return Image.open(self.files[i]).convert("RGB")


def _ffmpeg():
    exe = shutil.which("ffmpeg")
    if exe is None:
        raise ImportError("video files need imageio (with its ffmpeg plugin) or an `ffmpeg` executable on PATH; "
                          "neither is available -- pass an image folder (VideoData(image_folder=...)) instead")
    return exe


class _VideoFile:
    """Frame-indexed video reader (LowMemoryVideo, video.py:9-21)."""

    def __init__(self, path):
        self.path = path
        self.reader = None
        self.frames = None
        try:
            import imageio
            self.reader = imageio.get_reader(path)
        except ImportError:
            self._decode_ffmpeg()

    def _decode_ffmpeg(self):
        exe = _ffmpeg()
        probe = subprocess.run([exe, "-i", self.path], capture_output=True, text=True)
        m = re.search(r"Stream.*Video.*?, (\d+)x(\d+)", probe.stderr)
        if not m:
            raise RuntimeError(f"cannot read a video stream from {self.path}")
        w, h = int(m.group(1)), int(m.group(2))
        raw = subprocess.run([exe, "-v", "error", "-i", self.path, "-f", "rawvideo", "-pix_fmt", "rgb24", "-"],
                             capture_output=True, check=True).stdout
        self.frames = np.frombuffer(raw, dtype=np.uint8).reshape(-1, h, w, 3)

    def __len__(self):
        return self.reader.count_frames() if self.reader is not None else len(self.frames)

    def __getitem__(self, i):
        a = self.reader.get_data(i) if self.reader is not None else self.frames[i]
        return Image.fromarray(np.array(a)).convert("RGB")

    def __del__(self):
        if getattr(self, "reader", None) is not None:
            self.reader.close()


class VideoData:
    """VideoData (video.py:83-136): VideoData(video_file, height=..., width=...) or
    VideoData(image_folder=...); frames are PIL RGB images, centre-cropped/resized to (height,
    width) when those are set and differ from the frame size."""

    def __init__(self, video_file=None, image_folder=None, height=None, width=None, **kwargs):
        if video_file is not None:
            self.data_type = "video"
            self.data = _VideoFile(video_file, **kwargs)
        elif image_folder is not None:
            self.data_type = "images"
            self.data = _ImageFolder(image_folder, **kwargs)
        else:
            raise ValueError("Cannot open video or image folder")
        self.length = None
        self.set_shape(height, width)

    def raw_data(self):
        return [self[i] for i in range(len(self))]

    def set_length(self, length):
        self.length = length

    def set_shape(self, height, width):
        self.height, self.width = height, width

    def __len__(self):
        return len(self.data) if self.length is None else self.length

    def shape(self):
        if self.height is not None and self.width is not None:
            return self.height, self.width
        w, h = self[0].size
        return h, w

    def __getitem__(self, i):
        frame = self.data[i]
        w, h = frame.size
        if self.height is not None and self.width is not None and (self.height != h or self.width != w):
            frame = crop_and_resize(frame, self.height, self.width)
        return frame

    def save_images(self, folder):
        save_frames([self[i] for i in range(len(self))], folder)


def save_video(frames, save_path, fps, quality=9, ffmpeg_params=None):
    """save_video (video.py:139-144): frames (PIL images or HxWx3 uint8 arrays) -> a video file."""
    arrs = [np.asarray(f, dtype=np.uint8) for f in frames]
    try:
        import imageio
    except ImportError:
        imageio = None
    if imageio is not None:
        writer = imageio.get_writer(save_path, fps=fps, quality=quality, ffmpeg_params=ffmpeg_params)
        for a in arrs:
            writer.append_data(a)
        writer.close()
        return
    exe = _ffmpeg()
    h, w = arrs[0].shape[:2]
    # imageio-ffmpeg's quality q (0-10) maps to libx264 -crf ~ 51 * (1 - q / 10)
    crf = str(int(round(51 * (1 - min(max(quality, 0), 10) / 10))))
    cmd = [exe, "-y", "-v", "error", "-f", "rawvideo", "-pix_fmt", "rgb24", "-s", f"{w}x{h}", "-r", str(fps), "-i", "-",
           "-c:v", "libx264", "-pix_fmt", "yuv420p", "-crf", crf] + list(ffmpeg_params or []) + [save_path]
    subprocess.run(cmd, input=b"".join(a.tobytes() for a in arrs), check=True)


def save_frames(frames, save_path):
    """save_frames (video.py:146-149): frame i -> save_path/i.png."""
    os.makedirs(save_path, exist_ok=True)
    for i, f in enumerate(frames):
        (f if isinstance(f, Image.Image) else Image.fromarray(np.asarray(f, dtype=np.uint8))).save(
            os.path.join(save_path, f"{i}.png"))
