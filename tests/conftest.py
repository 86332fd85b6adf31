import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_sessionstart(session):
    # IMAGENT_SEGV_BT=1: print native frames on SIGSEGV / SIGABRT (scripts/segv_bt.c), chained in front of
    # pytest's faulthandler -- host-side diagnostics for crashes inside the HIP runtime (graph capture)
    if os.environ.get("IMAGENT_SEGV_BT") == "1":
        lib = os.path.join(ROOT, "scripts", "bin", "libsegv_bt.so")
        if os.path.exists(lib):
            import ctypes
            ctypes.CDLL(lib).install()
