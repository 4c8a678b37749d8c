"""GPU parity of the committed-batch apply loop (SafeCRDTManager.HandleAfterConsensusUpdates,
SURVEY.md §8a A13) through the C++ host mirror (janus-crdt_amd/host/) against the oracle's
SafeCRDTManager on a simulated 4-node cluster (see janus-crdt_amd/host/test_host.cpp)."""
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

BIN = Path(__file__).resolve().parent.parent / "janus-crdt_amd" / "build" / "test_host"


def test_committed_waves_match_oracle():
    out = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=110)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count("PASS case") == 4
