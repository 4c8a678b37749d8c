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


def test_committed_waves_match_oracle_chunked():
    """The same 4-node parity run with waves cut into 5-message chunks and every phase on the worker
    pool (JANUS_WAVE_CHUNK / JANUS_HOST_PAR_MIN): many chunks per wave, the dealt classify / gather tasks,
    chunk appends overlapped with the next chunk's classify, the split-off tail chunk, the parallel
    completion list, and the rejected-payload cut landing inside a multi-chunk wave."""
    import os
    env = dict(os.environ, JANUS_WAVE_CHUNK="5", JANUS_HOST_PAR_MIN="1")
    out = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=110, env=env)
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
        out = subprocess.run([str(BENCH), "--accounts", "20000", "--ops", "50000", "--waves", "2", "--cpu-msgs", "0",
                              "--rank", str(r), "--world", "2"], capture_output=True, text=True, timeout=110)
        assert out.returncode == 0, out.stderr
        res.append(json.loads(out.stdout.strip().splitlines()[-1]))
    assert res[0]["owned_accounts"] + res[1]["owned_accounts"] == 20000
    assert min(x["owned_accounts"] for x in res) > 9000  # balanced hash split
    assert res[0]["state_msgs_per_wave"] == res[1]["state_msgs_per_wave"]  # both ranks saw the same waves
    assert res[0]["applied_msgs_per_wave"] + res[1]["applied_msgs_per_wave"] == res[0]["state_msgs_per_wave"]


@pytest.mark.parametrize("args", [
    ["--accounts", "1000000", "--ops", "1000000", "--waves", "1"],             # C5: one 1M-op wave, 1M accounts
    ["--accounts", "100", "--ops", "200000", "--waves", "2", "--normal"],     # the paper's 100 accounts, N(n/2, n/6)
    ["--accounts", "5000", "--ops", "100000", "--waves", "2", "--rank", "1", "--world", "3"],  # one key-space shard
    ["--accounts", "200000", "--ops", "400000", "--waves", "2", "--direct"],  # payloads in page-locked memory, uploaded in place
    ["--accounts", "200000", "--ops", "400000", "--waves", "2", "--arena-stream", "--part-msgs", "30000"],  # streamed parts (jg_apply_stream_*)
])
def test_banking_replay_matches_oracle(args):
    """C5 parity (BankingWorload.cs ops through the node batchers): after every committed wave, every owned
    account's stable Get and the safe-update completions in commit order equal the oracle's
    HandleAfterConsensusUpdates over the same wave."""
    import json
    out = subprocess.run([str(BENCH), "--parity"] + args, capture_output=True, text=True, timeout=280)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["parity"], (res, out.stderr[-2000:])
    assert res["safe_per_wave"] > 0 and res["completed_per_wave"] > 0


def test_c1_replay_matches_oracle():
    """BASELINE configs[0] (C1: PNCWorkload, 100 keys, opsRatio [0.25, 0.25, 0.5], safeRatio 0.5) through the
    node batchers: every key's stable Get equals the oracle's after the committed waves."""
    import json
    out = subprocess.run([str(BIN.parent / "bench_c1"), "--ops", "300000", "--waves", "2"], capture_output=True, text=True, timeout=200)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["parity_vs_oracle"] is True, res


_BIG_PNC = ["--workload", "pnc", "--keys", "100000", "--ops", "1000", "--cpu-ops", "300000", "--waves", "1"]


@pytest.mark.parametrize("args,env", [
    (["--workload", "pnc", "--keys", "2000", "--ops", "20000", "--cpu-ops", "20000", "--waves", "1"], {}),  # many repeats per key
    (["--workload", "pnc", "--keys", "200000", "--ops", "50000", "--cpu-ops", "50000", "--waves", "1"], {}),
    (["--workload", "orset", "--keys", "300", "--ops", "20000", "--cpu-ops", "6000", "--waves", "1"], {}),  # Clears at 50 elements
    # >= 2^18 ops in one call: the PN-Counter batch in 4 encode-and-apply chunks, messages built per chunk
    (_BIG_PNC, {}),
    # the same with the states' size underguessed: a later chunk refused for room goes to a block of its own ...
    (_BIG_PNC, {"JANUS_PNC_STATE_GUESS": "200"}),
    # ... and the first chunk refused grows the buffer (nothing applied by a refused call)
    (_BIG_PNC, {"JANUS_PNC_STATE_GUESS": "20"}),
    # an invalid method in the last chunk: the chunks already on the device are taken back, the call raises with
    # nothing applied or queued; then the same call, valid, matches the oracle (the restored state included)
    (_BIG_PNC + ["--bad-at", "290000"], {"JANUS_SUBMIT_LOCKSTEP": "1"}),
    (_BIG_PNC + ["--bad-at", "10"], {}),
])
def test_producer_path_matches_oracle(args, env):
    """The producer path (SafeCRDT.Update + full-state Encode + ActualPropagateSyncMsg + ComputeDigest,
    GpuStableStore::SubmitClientUpdates) on the C5 banking and ORSetWorkload op streams: op results, every
    submitted UpdateMessage (order, identities, payload bytes) and its digest equal the oracle's
    (host/bench_submit.cpp's parity sample, one call over the whole sample)."""
    import json
    import os
    out = subprocess.run([str(BIN.parent / "bench_submit")] + args, capture_output=True, text=True, timeout=110, env={**os.environ, **env})
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert out.returncode == 0 and res["parity_vs_oracle"] is True, (res, out.stderr[-2000:])
    assert res["submitted_msgs_per_wave"] > 0
