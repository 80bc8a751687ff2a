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
def _heartbeat():
    """A line on stderr every 60 s while the GPU suite runs: some tests (the 14B production-shape
    oracle checks, the RCCL world-1 worker) compute for minutes without output, and a GPU box
    watchdog takes 3 silent minutes for a hang."""
    import threading
    import time
    import torch
    stop = threading.Event()
    if torch.cuda.is_available():
        t0 = time.time()

        def beat():
            while not stop.wait(60):
                print(f"[heartbeat {time.time() - t0:.0f} s]", file=sys.__stderr__, flush=True)
        threading.Thread(target=beat, daemon=True).start()
    yield
    stop.set()
