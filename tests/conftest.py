import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _test_sync():
    """SPA_TEST_SYNC=1: drain the device after every test, so asynchronous work of one test can
    never land in the next one's (stream-ordered, reused) allocations."""
    yield
    if os.environ.get("SPA_TEST_SYNC") == "1":
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()


@pytest.fixture(autouse=True)
def _device_bounds_guards():
    """In a debug-bounds build (SPA_EXT_SO=ab/_C_dbg.so with SPA_DEBUG_SYNC=1, see
    tests/test_debug_bounds_gpu.py) fail any test after which a device guard recorded a violation,
    including ones reached through torch.ops.spa directly (not via the checked ops() wrapper)."""
    yield
    if os.environ.get("SPA_DEBUG_SYNC") != "1" or not os.environ.get("SPA_EXT_SO"):
        return
    from solvingpapers_amd.ops import _ext
    if _ext.debug_bounds_enabled():
        rep = _ext.debug_bounds_report(True)
        assert rep == "", f"device bounds guard fired:\n{rep}"
