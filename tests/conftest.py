"""pytest configuration: the `gpu` marker, import paths, shared fixtures.

-m "not gpu": oracle vs the reference's known answers, host logic, ABI surface (no compute calls).
-m gpu      : parity of the HIP engine (through the C ABI) against the oracle.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "janus-crdt_amd", ROOT / "tests", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


# torch (device buffers, collectives in the shard tests) loads before libjanusgpu so the process holds
# ONE HIP runtime instance, as in bench.py
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libjanusgpu.so")


@pytest.fixture(scope="session")
def ctx():
    import janus_gpu as jg
    c = jg.Context(int(os.environ.get("JANUS_GPU_DEVICE", "0")))
    yield c
    c.close()
