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
    assert "FAIL" not in out.stdout
    assert out.stdout.count("PASS case") == 5
    for check in ("codec cross-check", "bad-payload wave", "unknown uid"):
        assert check in out.stdout


BENCH = BIN.parent / "bench_apply"


def test_sharded_apply_covers_the_wave_once():
    """Key-space sharding of the apply loop (GpuStableStore::ShardOf): two shards of the same waves,
    run one after the other on device 0, own disjoint accounts that cover the keyspace, and between
    them apply every message of every wave exactly once."""
    import json
    res = []
    for r in range(2):
        out = subprocess.run([str(BENCH), "--accounts", "20000", "--msgs", "50000", "--waves", "2", "--cpu-msgs", "0",
                              "--rank", str(r), "--world", "2"], capture_output=True, text=True, timeout=110)
        assert out.returncode == 0, out.stderr
        res.append(json.loads(out.stdout.strip().splitlines()[-1]))
    assert res[0]["owned_accounts"] + res[1]["owned_accounts"] == 20000
    assert min(x["owned_accounts"] for x in res) > 9000  # balanced hash split
    assert res[0]["applied_msgs_per_wave"] + res[1]["applied_msgs_per_wave"] == 50000
