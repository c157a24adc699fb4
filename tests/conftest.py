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
    """Drain the GPU while the runtime is intact.  No thread joins: the product stops its own
    engine loops at interpreter exit (engine/engine.py ``_stop_live_loops``), and the GPU suite
    exits cleanly without any help from here (profiles/r6b: DRTC_TEST_THREADS=1 lists only the
    main thread at the end)."""
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
