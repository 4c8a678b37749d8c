"""CPU-only: the N>1 path of bench.py with world size 2..5 over gloo — keyspace shards are disjoint
and cover N x the per-GPU shard (weak scaling) or exactly configs[3]'s 200M keys (strong scaling),
the barrier completes, the timing reduction is the max over ranks and the key count the sum (the
driver launches bench.py with torch.distributed.run, one rank per GPU)."""
import os
import socket
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, str(ROOT))
    import bench
    w, r, local = bench.dist_env()
    sync = bench.Sync(w, local, backend="gloo")
    sync.barrier()
    key0, n, _ = bench.pnc_shard("c4", "weak", r, w)
    worst = sync.max(1.0 + r)  # rank r "took" 1 + r seconds
    s0, sn, sR = bench.pnc_shard("c4", "strong", r, w)
    total = sync.sum_int(sn)
    sync.barrier()
    sync.close()
    q.put((r, key0, n, worst, s0, sn, sR, total))


@pytest.mark.parametrize("world", [2, 3, 5])
def test_weak_scaling_shards_and_max_over_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spans = [(k0, k0 + n) for _, k0, n, *_ in res]
    assert all(n == 25_000_000 for _, _, n, *_ in res)  # fixed per-GPU work: one C4 shard
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0  # disjoint, contiguous
    assert spans[0][0] == 0 and spans[-1][1] == world * res[0][2]
    assert all(x[3] == float(world) for x in res)  # max over ranks reached every rank
    # strong scaling: contiguous, disjoint, together exactly configs[3]'s 200M keys, 128 replicas
    strong = [(s0, s0 + sn) for *_, s0, sn, _, _ in res]
    assert strong[0][0] == 0 and strong[-1][1] == 200_000_000
    assert all(a1 == b0 for (_, a1), (b0, _) in zip(strong, strong[1:]))
    assert all(x[6] == 128 and x[7] == 200_000_000 for x in res)  # every rank saw the summed key count


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
def test_orset_strong_split_is_whole_sets_of_c3_times_8(world):
    """--scaling strong for the OR-Set leg: the C3 shape x 8 shards (80M (set, elem) groups) split into
    whole sets over the ranks, together exactly the total; weak keeps one C3 shard per rank."""
    sys.path.insert(0, str(ROOT))
    import bench
    parts = [bench.orset_groups("strong", r, world) for r in range(world)]
    assert sum(parts) == bench.ORSET_STRONG_SHARDS * bench.ORSET_GROUPS
    assert all(p % bench.ORSET_E == 0 for p in parts) and max(parts) - min(parts) <= bench.ORSET_E
    assert all(bench.orset_groups("weak", r, world) == bench.ORSET_GROUPS for r in range(world))
