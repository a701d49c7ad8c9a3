import os
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tts.cpp_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    """The step coalescer's tests (test_coalesce_gpu.py) run after the parity suite: they drive many backends
    from many threads at once, and a failure there must not stop (-x) the kernels' parity tests from
    running."""
    items.sort(key=lambda it: it.nodeid.startswith("tests/test_coalesce_gpu.py") or "test_coalesce_gpu.py::" in it.nodeid)


@pytest.fixture(scope="session")
def hip():
    import ttship
    be = ttship.HipBackend(0)
    yield be
    be.close()
