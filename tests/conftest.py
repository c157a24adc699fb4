import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402  (torch's HIP runtime must load before our extensions)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running (multi-process clusters)")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def hipk():
    from drtc_amd.ops._ext import hipk as _h

    return _h()


def pytest_sessionfinish(session, exitstatus):
    """Leave no thread running into interpreter finalization: a daemon thread that is inside
    native code (HIP / torch / gRPC) when CPython finalizes is ended with pthread_exit, whose
    forced unwind through C++ frames aborts the process ("terminate called without an active
    exception") after every test passed.  Join what the tests left (engine loops, server
    handlers still returning) and drain the GPU while the runtime is intact."""
    import gc
    import os
    import threading
    import time

    if os.environ.get("DRTC_TEST_JOIN", "1") == "0":
        # product behaviour only: EngineLoops stop themselves at exit (engine/engine.py
        # _stop_live_loops) - used to check that no join here is needed for a clean exit
        return
    main = threading.main_thread()
    deadline = time.time() + 30
    for t in threading.enumerate():
        if t is not main and t.is_alive():
            t.join(timeout=max(0.1, deadline - time.time()))
    gc.collect()
    try:
        import torch

        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:
        pass


def pytest_unconfigure(config):
    """DRTC_TEST_THREADS=1: list the threads still alive when the session ends (a native
    thread left running is what aborts an interpreter at exit)."""
    import os
    import sys
    import threading

    if os.environ.get("DRTC_TEST_THREADS") == "1":
        for t in threading.enumerate():
            print(f"[threads at exit] {t.name} daemon={t.daemon} alive={t.is_alive()}",
                  file=sys.stderr, flush=True)
