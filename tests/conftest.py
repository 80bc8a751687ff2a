import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "video-styler_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def _heartbeat(request):
    """A line on the real stderr every 60 s while the GPU suite runs: some tests (the 14B production-
    shape oracle checks, the RCCL world-1 worker) compute for minutes without output, and a GPU box
    watchdog takes 3 silent minutes for a hang.  fd-level capture redirects fd 2 during a test, so
    the line goes to the descriptor the capture manager saved (the session's original stderr)."""
    import threading
    import time
    import torch
    stop = threading.Event()
    fd = 2
    capman = request.config.pluginmanager.getplugin("capturemanager")
    try:
        fd = capman._global_capturing.err.targetfd_save
    except AttributeError:        # capture disabled (-s) or a pytest without the fd capture internals
        pass
    if torch.cuda.is_available():
        t0 = time.time()

        def beat():
            while not stop.wait(60):
                try:
                    os.write(fd, f"[heartbeat {time.time() - t0:.0f} s]\n".encode())
                except OSError:
                    return
        threading.Thread(target=beat, daemon=True).start()
    yield
    stop.set()
