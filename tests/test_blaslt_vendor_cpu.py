"""The private copy of the image's ROCm hipBLASLt (scripts/vendor_blaslt.py, csrc/blaslt.hip): the
copies carry renamed SONAMEs / NEEDED entries and are otherwise byte-identical, and libvstyler opens
them (vs_blaslt_library names the copy) next to the hipBLASLt torch loaded.  CPU-only: dlopen and
symbol resolution need no GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import vendor_blaslt  # noqa: E402

ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH") or "/opt/rocm", "lib")
HAVE = all(os.path.exists(os.path.join(ROCM_LIB, f)) for f in vendor_blaslt.FILES)


def _dynamic(path, tag):
    out = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    return [ln.split("[")[1].rstrip("]") for ln in out.splitlines() if f"({tag})" in ln]


@pytest.mark.skipif(not HAVE, reason="no ROCm hipBLASLt in this image")
def test_vendored_copies_renamed_only(tmp_path):
    vendor_blaslt.main([str(tmp_path), ROCM_LIB])
    lt = str(tmp_path / "libvsblaslt7.so.1")
    rr = str(tmp_path / "libvsroller7.so.1")
    assert _dynamic(lt, "SONAME") == ["libvsblaslt7.so.1"]
    assert _dynamic(rr, "SONAME") == ["libvsroller7.so.1"]
    needed = _dynamic(lt, "NEEDED")
    assert "libvsroller7.so.1" in needed and "librocroller.so.1" not in needed
    assert "libamdhip64.so.7" in needed          # shares the process's HIP runtime by SONAME
    # nothing but the renamed .dynstr names differs from the originals
    for src, dst in vendor_blaslt.FILES.items():
        a = open(os.path.realpath(os.path.join(ROCM_LIB, src)), "rb").read()
        b = open(tmp_path / dst, "rb").read()
        assert len(a) == len(b)
        diff = [i for i in range(0, len(a), 1 << 16) if a[i:i + (1 << 16)] != b[i:i + (1 << 16)]]
        assert 1 <= len(diff) <= 2, diff
        off, size = vendor_blaslt.dynstr_range(a)
        nd = sum(x != y for x, y in zip(a[off:off + size], b[off:off + size]))
        assert nd > 0 and nd == sum(x != y for x, y in zip(a, b))


@pytest.mark.skipif(not HAVE, reason="no ROCm hipBLASLt in this image")
def test_library_opens_private_copy_beside_torch():
    code = ("import sys, torch; sys.path.insert(0, 'video-styler_amd'); from vstyler import _lib; "
            "print(_lib.load().vs_blaslt_library().decode())")
    env = {k: v for k, v in os.environ.items() if k != "VS_LT_LIB"}
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, env=env,
                         check=True).stdout.strip().splitlines()[-1]
    assert out.endswith("lt72/libvsblaslt7.so.1"), out
    env["VS_LT_LIB"] = "linked"
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, env=env,
                         check=True).stdout.strip().splitlines()[-1]
    assert out == "linked"
