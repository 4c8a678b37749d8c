"""CPU-only: the cross-shard exchange protocol of janus_gpu/shard.py over gloo at world size 2 and 3.

Each rank receives a batch of states addressed by GLOBAL keys, routes it with the host restatement of
the route rule (tests/shard_ref.py, the checker of csrc/route.hip), exchanges the runs with
shard.Exchange (the same all-to-all code that runs over RCCL on the GPU box), and merges what it
receives into its own shard with the oracle.  Every rank's shard must equal its slice of the oracle
merge of the whole keyspace with every rank's batch (PNCounter.Merge, ORSet.Merge are per key).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent
K_LOCAL, R, ROWS = 37, 6, 90


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pnc_inputs(world):
    from gen import random_pnc
    rng = np.random.default_rng(99)
    G = K_LOCAL * world
    AP = random_pnc(rng, G, R, 8, absent=False, lo=0, hi=1 << 40)
    AN = random_pnc(rng, G, R, 8, absent=False, lo=0, hi=1 << 40)
    batches = []
    for r in range(world):
        keys = rng.integers(0, G, ROWS).astype(np.uint32)
        batches.append((keys, random_pnc(rng, ROWS, R, 8, lo=0, hi=1 << 40), random_pnc(rng, ROWS, R, 8, lo=0, hi=1 << 40)))
    return AP, AN, batches


def _orset_inputs(world):
    from gen import random_orset_pair
    rng = np.random.default_rng(7)
    La, Lr, _, _ = random_orset_pair(rng, n_sets=5 * world, n_elems=4, pool=8)
    recv = [random_orset_pair(rng, n_sets=5 * world, n_elems=4, pool=8)[2:] for _ in range(world)]
    return La, Lr, recv


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    for p in (ROOT / "janus-crdt_amd", ROOT / "tests"):
        sys.path.insert(0, str(p))
    import torch
    import torch.distributed as dist
    import oracle_ref as orc
    import shard_ref as ref
    from janus_gpu.shard import Exchange
    dist.init_process_group("gloo")
    try:
        ex = Exchange(torch.device("cpu"))
        assert ex.staged and ex.world == world and ex.rank == rank
        # ---- PN-Counter ----
        AP, AN, batches = _pnc_inputs(world)
        keys, BP, BN = batches[rank]
        sent, lk, sP, sN = ref.route_rows(keys, BP, BN, world)
        got = ex.counts(sent)
        rk = ex.runs(torch.from_numpy(lk.astype(np.int32)), sent, got).numpy().astype(np.uint32)
        rP = ex.runs(torch.from_numpy(sP), sent, got).numpy()
        rN = ex.runs(torch.from_numpy(sN), sent, got).numpy()
        myP, myN = orc.pnc_merge(ref.shard_rows(AP, world, rank), ref.shard_rows(AN, world, rank), rP, rN, rk)
        eP, eN = AP, AN
        for k, bp, bn in batches:
            eP, eN = orc.pnc_merge(eP, eN, bp, bn, k)
        ok_pnc = np.array_equal(myP, ref.shard_rows(eP, world, rank)) and np.array_equal(myN, ref.shard_rows(eN, world, rank))
        # every source's run arrives, in source-rank order
        ok_counts = int(got.sum()) == sum(int(np.sum(b[0] % world == rank)) for b in batches)
        # ---- OR-Set ----
        La, Lr, recv = _orset_inputs(world)
        Ra, Rr = recv[rank]
        sa, ra_ = ref.route_records(Ra, world)
        sr, rr_ = ref.route_records(Rr, world)
        ga, gr = ex.counts(sa), ex.counts(sr)
        view = lambda x: torch.from_numpy(x.view(np.int64).reshape(-1, 4))
        ia = ex.runs(view(ra_), sa, ga).numpy().reshape(-1).view(orc.REC_DTYPE)
        ir = ex.runs(view(rr_), sr, gr).numpy().reshape(-1).view(orc.REC_DTYPE)
        ma, mr = ref.shard_records(La, world, rank), ref.shard_records(Lr, world, rank)
        for i in range(world):  # merge run after run, like jg_orset_merge_device
            a0, a1 = int(ga[:i].sum()), int(ga[: i + 1].sum())
            r0, r1 = int(gr[:i].sum()), int(gr[: i + 1].sum())
            ma, mr = orc.orset_merge(ma, mr, ia[a0:a1], ir[r0:r1])
        ea, er = La, Lr
        for a, r in recv:
            ea, er = orc.orset_merge(ea, er, a, r)
        ok_orset = orc.same_orset(ma, mr, ref.shard_records(ea, world, rank), ref.shard_records(er, world, rank))
        q.put((rank, ok_pnc, ok_counts, ok_orset, ""))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, False, False, False, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_over_gloo_matches_global_merge(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_pnc, ok_counts, ok_orset, err in res:
        assert not err, f"rank {rank}: {err}"
        assert ok_pnc and ok_counts and ok_orset, (rank, ok_pnc, ok_counts, ok_orset)


def test_route_rule_is_a_stable_partition():
    import shard_ref as ref
    from gen import random_orset_pair
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 1000, 500).astype(np.uint32)
    P = np.arange(500 * 2, dtype=np.int64).reshape(500, 2)
    counts, lk, rP, _ = ref.route_rows(keys, P, P, 4)
    at = 0
    for d in range(4):
        seg = rP[at: at + int(counts[d]), 0] // 2
        assert np.all(np.diff(seg) > 0)               # batch order kept
        assert np.all(keys[seg] % 4 == d) and np.array_equal(lk[at: at + int(counts[d])], keys[seg] // 4)
        at += int(counts[d])
    La, _, _, _ = random_orset_pair(rng, n_sets=30, n_elems=5, pool=6)
    c, out = ref.route_records(La, 3)
    at = 0
    for d in range(3):
        run = out[at: at + int(c[d])]
        assert np.array_equal(np.unique(run), run)    # each owner's run stays strictly increasing
        at += int(c[d])


@pytest.mark.parametrize("world", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("k,skip_own", [(1, True), (1, False), (2, False)])
def test_exchange_plan_matches_all_to_all_layout(world, k, skip_own):
    """jg_exchange_plan (csrc/comm.hip, the plan every exchange call follows: RCCL or host transport) against
    janus_gpu/shard.py's all_to_all_single layout on the same counts, then the whole exchange simulated: every
    rank's runs copied where the plan says must land exactly the records routed to each rank, in source-rank
    order (the order the OR-Set union keeps for arrival ordinals).  Pure host arithmetic: runs on CPU."""
    sys.path.insert(0, str(ROOT / "janus-crdt_amd"))
    import janus_gpu as jg
    from janus_gpu.shard import all_to_all_plan
    rng = np.random.default_rng(world * 10 + k)
    counts = rng.integers(0, 50, (world, world, k)).astype(np.uint64)
    counts[rng.random((world, world, k)) < 0.25] = 0  # empty runs, incl. own ones
    counts[0] = 0  # a rank that sends nothing
    plans = [jg.exchange_plan(r, world, counts, skip_own) for r in range(world)]
    for r in range(world):
        for a, b in zip(plans[r], all_to_all_plan(counts, r, skip_own)):
            assert np.array_equal(a, b)
    for j in range(k):
        # send buffer of src: (src, dst, idx) records grouped by dst in rank order
        send = [[(s_, d, i) for d in range(world) for i in range(int(counts[s_, d, j]))] for s_ in range(world)]
        for d in range(world):
            so, sn, ro, rn = (x[:, j] for x in plans[d])
            recv = [None] * int(rn.sum())
            for s_ in range(world):
                s_off, s_n = plans[s_][0][d, j], plans[s_][1][d, j]
                assert s_n == rn[s_], "what src sends dst must equal what dst receives from src"
                if s_ == d and skip_own:
                    assert s_n == 0
                    continue
                recv[int(ro[s_]):int(ro[s_] + rn[s_])] = send[s_][int(s_off):int(s_off + s_n)]
            exp = [(s_, d, i) for s_ in range(world) if not (skip_own and s_ == d) for i in range(int(counts[s_, d, j]))]
            assert recv == exp
            if skip_own:  # the own run stays in the send buffer where the merge reads it
                own = send[d][int(so[d]):int(so[d] + counts[d, d, j])]
                assert own == [(d, d, i) for i in range(int(counts[d, d, j]))]


def test_global_key_follows_shard_of():
    """The one owner rule: a key registered by its owner jg_shard_of(uid, world) with local
    index l has the global key l * world + owner, which the exchange routes to rank global % world as local
    key global // world (csrc/jg_internal.hpp owner_of_key).  Pure host: runs on CPU."""
    sys.path.insert(0, str(ROOT / "janus-crdt_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    import janus_gpu as jg
    import shard_ref as ref
    rng = np.random.default_rng(5)
    uids = [(int(a), int(b)) for a, b in rng.integers(1, 2**63, (300, 2), dtype=np.int64)]
    for world in range(1, 9):
        nxt = [0] * world
        for lo, hi in uids:
            owner = jg.shard_of(lo, hi, world)
            g = jg.global_key(lo, hi, world, nxt[owner])
            assert g % world == owner and g // world == nxt[owner]
            assert ref.owner_of_key(g, world) == owner and ref.local_of_key(g, world) == nxt[owner]
            nxt[owner] += 1
        assert sum(nxt) == len(uids)
