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
    config.addinivalue_line("markers", "gpu_long: MI355X test whose oracle takes minutes (C4 block pair, "
                                       "480x832 VAE): outside the round-end -m gpu tier, run by scripts/ab/r4_parity.sh")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords or "gpu_long" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def opt():
    """opt(gemm_kernel=8, gemm_split=0, ...): libvstyler path-selection options (kernels.set_option,
    include/vstyler.h VS_OPT_*) for one test, restored afterwards."""
    from vstyler import kernels as K
    saved = {}

    def set_(**kw):
        for k, v in kw.items():
            prev = K.set_option(k, v)
            saved.setdefault(k, prev)
    yield set_
    for k, v in saved.items():
        K.set_option(k, v)


_PROGRESS = {"fd": 2, "t0": None}


def _progress(msg):
    if _PROGRESS.get("on") is None:
        import torch
        _PROGRESS["on"] = torch.cuda.is_available()     # the GPU suite only (CPU runs stay quiet)
    if not _PROGRESS["on"]:
        return
    try:
        os.write(_PROGRESS["fd"], (msg + "\n").encode())
    except OSError:
        pass


def pytest_runtest_logstart(nodeid, location):
    import time
    _PROGRESS["t0"] = time.time()
    _progress(f"[start] {nodeid}")


def pytest_runtest_logfinish(nodeid, location):
    import time
    t0 = _PROGRESS["t0"]
    _progress(f"[done {time.time() - t0:.1f} s] {nodeid}" if t0 else f"[done] {nodeid}")


@pytest.fixture(scope="session", autouse=True)
def _progress_lines(request):
    """Progress on the session's real stderr (fd-level capture redirects fd 2 during a test, so the
    lines go to the descriptor the capture manager saved): one line when each test starts and ends,
    and while a GPU-suite test runs, a line every 60 s ONLY if the main thread moved on since the
    previous sample (its innermost Python frame or bytecode offset changed).  A long oracle check
    that keeps computing stays visible; a test stuck in one GPU call (a hung kernel blocks the main
    thread inside a synchronising call) goes silent, so the GPU box's 3-minute silence watchdog
    still ends it."""
    import sys
    import threading
    import time
    import torch
    capman = request.config.pluginmanager.getplugin("capturemanager")
    try:
        _PROGRESS["fd"] = capman._global_capturing.err.targetfd_save
    except AttributeError:        # capture disabled (-s) or a pytest without the fd capture internals
        pass
    stop = threading.Event()
    if torch.cuda.is_available():
        main_id = threading.main_thread().ident
        t0 = time.time()

        def where():
            f = sys._current_frames().get(main_id)
            return None if f is None else (f.f_code.co_filename, f.f_lineno, f.f_lasti, id(f))

        def beat():
            last = where()
            while not stop.wait(60):
                now = where()
                if now != last:
                    _progress(f"[alive {time.time() - t0:.0f} s] {now[0]}:{now[1]}" if now else "[alive]")
                last = now
        threading.Thread(target=beat, daemon=True).start()
    yield
    stop.set()
