import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
# tests compile their kernels afresh (the engine's on-disk code-object cache is off unless a
# test turns it on for a child process: test_jit_disk_cache.py)
os.environ.setdefault("MYTHGPU_JIT_DISK_CACHE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libmythgpu.so")


@pytest.fixture(scope="session")
def engine():
    """The GPU engine.  On a GPU box the HIP path must load: no silent skip."""
    from mythril_amd import build, native

    build.build()
    return native.Engine.get()
