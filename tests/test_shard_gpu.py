"""GPU parity of the cross-shard exchange (csrc/route.hip, janus_gpu/shard.py) against the host route
rule (tests/shard_ref.py) and the oracle's PNCounter.Merge / ORSet.Merge.

* route kernels: bit-exact stable partitions (counts, local keys, rows / records) for world 1..8,
  int32 / int64 rows, 16-B-vector and ragged row widths, identity and indexed batches, tile edges;
* merge from device memory: equal to jg_pnc_merge_rows / the oracle, all or nothing on bad keys;
* a keyspace sharded over W "ranks" in one process (routing without a collective): every owner's
  shard equals its slice of the oracle merge of the whole keyspace;
* two processes sharing device 0 over gloo (host-staged all-to-all): the full exchange path with the
  real kernels (the RCCL transport itself runs in bench.py on the 8-GPU node).
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

import janus_gpu as jg
import oracle_ref as orc
import shard_ref as ref
from gen import random_orset_pair, random_pnc
from janus_gpu import shard

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _dev(ctx):
    return torch.device("cuda", ctx.device)


def _route_rows(ctx, keys, P, N, world, eb):
    n, R = P.shape
    rows = jg.Rows(ctx, n, R, eb)
    rows.upload(P, N, keys)
    dt = torch.int64 if eb == 8 else torch.int32
    k = torch.empty(n, dtype=torch.int32, device=_dev(ctx))
    dP = torch.empty((n, R), dtype=dt, device=_dev(ctx))
    dN = torch.empty((n, R), dtype=dt, device=_dev(ctx))
    counts = rows.route(world, k.data_ptr(), dP.data_ptr(), dN.data_ptr())
    rows.close()
    return counts, k.cpu().numpy().astype(np.uint32), dP.cpu().numpy(), dN.cpu().numpy()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("eb,R", [(8, 64), (4, 64), (8, 5), (4, 3)])
@pytest.mark.parametrize("n", [1, 1023, 1024, 1025, 20_000])
def test_rows_route_matches_host_rule(ctx, world, eb, R, n):
    rng = np.random.default_rng(world * 1000 + n + R)
    keys = rng.integers(0, 5 * n + 7, n).astype(np.uint32)
    P, N = random_pnc(rng, n, R, eb), random_pnc(rng, n, R, eb)
    got = _route_rows(ctx, keys, P, N, world, eb)
    exp = ref.route_rows(keys, P, N, world)
    for g, e in zip(got, exp):
        assert np.array_equal(g, e)


def test_identity_rows_route(ctx):
    rng = np.random.default_rng(5)
    n, R, world = 3000, 8, 4
    P, N = random_pnc(rng, n, R, 8), random_pnc(rng, n, R, 8)
    rows = jg.Rows(ctx, n, R, 8)
    rows.upload(P, N)  # no key_idx: row i is key i
    k = torch.empty(n, dtype=torch.int32, device=_dev(ctx))
    dP = torch.empty((n, R), dtype=torch.int64, device=_dev(ctx))
    dN = torch.empty_like(dP)
    counts = rows.route(world, k.data_ptr(), dP.data_ptr(), dN.data_ptr())
    rows.close()
    exp = ref.route_rows(np.arange(n, dtype=np.uint32), P, N, world)
    assert np.array_equal(counts, exp[0]) and np.array_equal(k.cpu().numpy(), exp[1])
    assert np.array_equal(dP.cpu().numpy(), exp[2]) and np.array_equal(dN.cpu().numpy(), exp[3])


def test_route_rejects_bad_buffers(ctx):
    rows = jg.Rows(ctx, 100, 4, 8)
    rows.upload(np.zeros((100, 4), np.int64), np.zeros((100, 4), np.int64), np.arange(100, dtype=np.uint32))
    small = torch.empty(10, dtype=torch.int64, device=_dev(ctx))
    big = torch.empty((100, 4), dtype=torch.int64, device=_dev(ctx))
    host = np.zeros((100, 4), np.int64)
    with pytest.raises(jg.JanusError) as e:
        rows.route(2, big.data_ptr(), big.data_ptr(), host.ctypes.data)  # host memory
    assert e.value.code == jg.JG_EINVAL
    with pytest.raises(jg.JanusError):
        rows.route(0, big.data_ptr(), big.data_ptr(), big.data_ptr())    # world 0
    with pytest.raises(jg.JanusError):
        rows.route(2, big.data_ptr(), big.data_ptr(), big.data_ptr(), cap_rows=99)
    del small
    rows.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_merge_device_matches_oracle_and_is_all_or_nothing(ctx, eb):
    rng = np.random.default_rng(11 + eb)
    K, R, n = 300, 16, 5000
    AP, AN = random_pnc(rng, K, R, eb, absent=False), random_pnc(rng, K, R, eb, absent=False)
    BP, BN = random_pnc(rng, n, R, eb), random_pnc(rng, n, R, eb)
    keys = rng.integers(0, K, n).astype(np.uint32)
    s = jg.PNCStore(ctx, K, R, eb)
    s.write_rows(AP, AN)
    dev = _dev(ctx)
    dk = torch.from_numpy(keys.astype(np.int32)).to(dev)
    dP, dN = torch.from_numpy(BP).to(dev), torch.from_numpy(BN).to(dev)
    torch.cuda.synchronize(dev)
    s.merge_device(n, dk.data_ptr(), dP.data_ptr(), dN.data_ptr())
    eP, eN = orc.pnc_merge(AP, AN, BP, BN, keys)
    P, N = s.read_rows()
    assert np.array_equal(P, eP) and np.array_equal(N, eN)
    bad = dk.clone()
    bad[n // 2] = K  # one key outside the store: nothing merges
    torch.cuda.synchronize(dev)
    with pytest.raises(jg.JanusError) as e:
        s.merge_device(n, bad.data_ptr(), dP.data_ptr(), dN.data_ptr())
    assert e.value.code == jg.JG_EINVAL
    P2, N2 = s.read_rows()
    assert np.array_equal(P2, eP) and np.array_equal(N2, eN)
    s.close()


@pytest.mark.parametrize("world", [2, 4, 7])
def test_pnc_sharded_keyspace_in_one_process(ctx, world):
    """W ranks simulated in one process: each routes its batch; each owner merges every source's run
    (source order) from device memory; owner shards = slices of the oracle's global merge."""
    rng = np.random.default_rng(40 + world)
    K_local, R, n = 257, 64, 4000
    G = K_local * world
    AP, AN = random_pnc(rng, G, R, 8, absent=False, lo=0), random_pnc(rng, G, R, 8, absent=False, lo=0)
    batches = [(rng.integers(0, G, n).astype(np.uint32), random_pnc(rng, n, R, 8), random_pnc(rng, n, R, 8)) for _ in range(world)]
    routed = [_route_rows(ctx, k, P, N, world, 8) for k, P, N in batches]
    eP, eN = AP, AN
    for k, P, N in batches:
        eP, eN = orc.pnc_merge(eP, eN, P, N, k)
    dev = _dev(ctx)
    for d in range(world):
        s = jg.PNCStore(ctx, K_local, R, 8)
        s.write_rows(ref.shard_rows(AP, world, d), ref.shard_rows(AN, world, d))
        parts = []
        for counts, k, P, N in routed:
            lo = int(counts[:d].sum())
            hi = lo + int(counts[d])
            parts.append((k[lo:hi], P[lo:hi], N[lo:hi]))
        k = torch.from_numpy(np.concatenate([p[0] for p in parts]).astype(np.int32)).to(dev)
        P = torch.from_numpy(np.concatenate([p[1] for p in parts])).to(dev)
        N = torch.from_numpy(np.concatenate([p[2] for p in parts])).to(dev)
        torch.cuda.synchronize(dev)
        s.merge_device(k.numel(), k.data_ptr(), P.data_ptr(), N.data_ptr())
        gP, gN = s.read_rows()
        s.close()
        assert np.array_equal(gP, ref.shard_rows(eP, world, d)) and np.array_equal(gN, ref.shard_rows(eN, world, d))


def _route_store(ctx, add, rem, world):
    src = jg.ORSetStore(ctx, len(add), len(rem))
    src.load(add, rem)
    dev = _dev(ctx)
    na, nr = len(add), len(rem)
    ak, rk = torch.empty(na, dtype=torch.int64, device=dev), torch.empty(nr, dtype=torch.int64, device=dev)
    at, rt = torch.empty((na, 2), dtype=torch.int64, device=dev), torch.empty((nr, 2), dtype=torch.int64, device=dev)
    ao, ro = torch.empty(na, dtype=torch.int32, device=dev), torch.empty(nr, dtype=torch.int32, device=dev)
    ca, cr = src.route(world, ak.data_ptr(), at.data_ptr(), ao.data_ptr(), na, rk.data_ptr(), rt.data_ptr(), ro.data_ptr(), nr)
    src.close()

    def recs(k, t, o):
        r = np.empty(k.shape[0], jg.REC_DTYPE)
        r["key"] = k.cpu().numpy().view(np.uint64)
        tt = t.cpu().numpy().view(np.uint64).reshape(-1, 2)
        r["tag_lo"], r["tag_hi"] = tt[:, 0], tt[:, 1]
        r["ord"] = o.cpu().numpy().view(np.uint32)
        return r

    return ca, cr, recs(ak, at, ao), recs(rk, rt, ro)


def _dev_recs(recs, dev):
    """A record array as the (key, tag, ord) device buffers jg_orset_merge_device reads."""
    k = torch.from_numpy(recs["key"].view(np.int64).copy()).to(dev)
    t = torch.from_numpy(np.stack([recs["tag_lo"], recs["tag_hi"]], 1).view(np.int64).copy()).to(dev)
    o = torch.from_numpy(recs["ord"].astype(np.uint32).view(np.int32).copy()).to(dev)
    return k, t, o


@pytest.mark.parametrize("world", [1, 3, 8])
@pytest.mark.parametrize("n_sets", [5, 2000])
def test_orset_route_matches_host_rule(ctx, world, n_sets):
    rng = np.random.default_rng(n_sets + world)
    La, Lr, _, _ = random_orset_pair(rng, n_sets=n_sets, n_elems=6, pool=8)
    ca, cr, ga, gr = _route_store(ctx, La, Lr, world)
    ea, er = ref.route_records(La, world), ref.route_records(Lr, world)
    assert np.array_equal(ca, ea[0]) and np.array_equal(ga, ea[1])
    assert np.array_equal(cr, er[0]) and np.array_equal(gr, er[1])


def test_orset_route_of_a_union_output(ctx):
    """Route a chunked (non-dense) stream: the output of a union, whose chunks are partly full."""
    rng = np.random.default_rng(8)
    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=3000, n_elems=5, pool=6)
    a, b = jg.ORSetStore(ctx, len(La), len(Lr)), jg.ORSetStore(ctx, len(Ra), len(Rr))
    a.load(La, Lr)
    b.load(Ra, Rr)
    a.merge_store(b)
    na, nr = a.size()
    dev = _dev(ctx)
    ak, rk = torch.empty(na, dtype=torch.int64, device=dev), torch.empty(nr, dtype=torch.int64, device=dev)
    at, rt = torch.empty((na, 2), dtype=torch.int64, device=dev), torch.empty((nr, 2), dtype=torch.int64, device=dev)
    ao, ro = torch.empty(na, dtype=torch.int32, device=dev), torch.empty(nr, dtype=torch.int32, device=dev)
    ca, cr = a.route(5, ak.data_ptr(), at.data_ptr(), ao.data_ptr(), na, rk.data_ptr(), rt.data_ptr(), ro.data_ptr(), nr)
    ea, er = orc.orset_merge(La, Lr, Ra, Rr)
    assert np.array_equal(ca, ref.route_records(ea, 5)[0]) and np.array_equal(cr, ref.route_records(er, 5)[0])
    assert np.array_equal(ak.cpu().numpy().view(np.uint64), ref.route_records(ea, 5)[1]["key"])
    for h in (a, b):
        h.close()


@pytest.mark.parametrize("world", [2, 5])
def test_orset_sharded_keyspace_in_one_process(ctx, world):
    rng = np.random.default_rng(70 + world)
    n_sets = 60 * world
    La, Lr, _, _ = random_orset_pair(rng, n_sets=n_sets, n_elems=5, pool=10)
    recv = [random_orset_pair(rng, n_sets=n_sets, n_elems=5, pool=10)[2:] for _ in range(world)]
    routed = [_route_store(ctx, a, r, world) for a, r in recv]
    ea, er = La, Lr
    for a, r in recv:
        ea, er = orc.orset_merge(ea, er, a, r)
    dev = _dev(ctx)
    for d in range(world):
        s = jg.ORSetStore(ctx, 0, 0)
        s.load(ref.shard_records(La, world, d), ref.shard_records(Lr, world, d))
        runs_a, runs_r, cnt_a, cnt_r = [], [], [], []
        for ca, cr, ga, gr in routed:
            a0, r0 = int(ca[:d].sum()), int(cr[:d].sum())
            runs_a.append(ga[a0:a0 + int(ca[d])])
            runs_r.append(gr[r0:r0 + int(cr[d])])
            cnt_a.append(int(ca[d]))
            cnt_r.append(int(cr[d]))
        A, Rm = np.concatenate(runs_a), np.concatenate(runs_r)
        ak, at, ao = _dev_recs(A, dev)
        rk, rt, ro = _dev_recs(Rm, dev)
        torch.cuda.synchronize(dev)
        s.merge_device(cnt_a, cnt_r, ak.data_ptr(), at.data_ptr(), ao.data_ptr(), rk.data_ptr(), rt.data_ptr(), ro.data_ptr())
        ga, gr = s.read()
        s.close()
        assert orc.same_orset(ga, gr, ref.shard_records(ea, world, d), ref.shard_records(er, world, d))


def test_orset_merge_device_rejects_unsorted_run(ctx):
    rng = np.random.default_rng(2)
    La, Lr, Ra, _ = random_orset_pair(rng, n_sets=20, n_elems=4, pool=6)
    s = jg.ORSetStore(ctx, len(La), len(Lr))
    s.load(La, Lr)
    bad = Ra[::-1].copy()
    dev = _dev(ctx)
    ak, at, ao = _dev_recs(bad, dev)
    e0 = torch.empty(0, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    with pytest.raises(jg.JanusError) as e:
        s.merge_device([len(bad)], [0], ak.data_ptr(), at.data_ptr(), ao.data_ptr(), e0.data_ptr(), e0.data_ptr(), e0.data_ptr())
    assert e.value.code == jg.JG_ESTATE
    ga, gr = s.read()  # unchanged
    assert np.array_equal(ga, La) and np.array_equal(gr, Lr)
    s.close()


# ---- two processes on device 0, gloo (host-staged) all-to-all through janus_gpu.shard ----
def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _two_rank_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    for p in (ROOT / "janus-crdt_amd", ROOT / "tests"):
        sys.path.insert(0, str(p))
    import torch.distributed as dist
    import janus_gpu as jg_
    import oracle_ref as orc_
    import shard_ref as ref_
    from gen import random_orset_pair as rop, random_pnc as rpnc
    from janus_gpu import shard as sh
    dist.init_process_group("gloo")
    try:
        dev = torch.device("cuda", 0)
        ex = sh.Exchange(dev)
        rng = np.random.default_rng(123)
        K_local, R, n = 500, 64, 3000
        G = K_local * world
        AP, AN = rpnc(rng, G, R, 8, absent=False, lo=0), rpnc(rng, G, R, 8, absent=False, lo=0)
        batches = [(rng.integers(0, G, n).astype(np.uint32), rpnc(rng, n, R, 8), rpnc(rng, n, R, 8)) for _ in range(world)]
        La, Lr, _, _ = rop(rng, n_sets=40 * world, n_elems=5, pool=8)
        recv = [rop(rng, n_sets=40 * world, n_elems=5, pool=8)[2:] for _ in range(world)]
        with jg_.Context(0) as ctx:
            s = jg_.PNCStore(ctx, K_local, R, 8)
            s.write_rows(ref_.shard_rows(AP, world, rank), ref_.shard_rows(AN, world, rank))
            rows = jg_.Rows(ctx, n, R, 8)
            k, P, N = batches[rank]
            rows.upload(P, N, k)
            sh.exchange_pnc(s, rows, ex, dev)
            gP, gN = s.read_rows()
            eP, eN = AP, AN
            for kk, PP, NN in batches:
                eP, eN = orc_.pnc_merge(eP, eN, PP, NN, kk)
            ok_pnc = np.array_equal(gP, ref_.shard_rows(eP, world, rank)) and np.array_equal(gN, ref_.shard_rows(eN, world, rank))
            o = jg_.ORSetStore(ctx, 0, 0)
            o.load(ref_.shard_records(La, world, rank), ref_.shard_records(Lr, world, rank))
            src = jg_.ORSetStore(ctx, 0, 0)
            src.load(*recv[rank])
            sh.exchange_orset(o, src, ex, dev)
            ga, gr = o.read()
            ea, er = La, Lr
            for a, r in recv:
                ea, er = orc_.orset_merge(ea, er, a, r)
            ok_orset = orc_.same_orset(ga, gr, ref_.shard_records(ea, world, rank), ref_.shard_records(er, world, rank))
            for h in (s, rows, o, src):
                h.close()
        q.put((rank, ok_pnc, ok_orset, ""))
    except Exception as e:
        q.put((rank, False, False, repr(e)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_share_device_0_over_gloo():
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=100) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, ok_pnc, ok_orset, err in res:
        assert not err, f"rank {rank}: {err}"
        assert ok_pnc and ok_orset, (rank, ok_pnc, ok_orset)


# ---- the RCCL path (backend "nccl", device buffers handed to all_to_all_single) at world size 1 ----
def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    for p in (ROOT / "janus-crdt_amd", ROOT / "tests"):
        sys.path.insert(0, str(p))
    import torch.distributed as dist
    import janus_gpu as jg_
    import oracle_ref as orc_
    from gen import random_pnc as rpnc
    from janus_gpu import shard as sh
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        ex = sh.Exchange(dev)
        assert not ex.staged
        rng = np.random.default_rng(5)
        K, R, n = 800, 64, 5000
        AP, AN = rpnc(rng, K, R, 8, absent=False, lo=0), rpnc(rng, K, R, 8, absent=False, lo=0)
        k, P, N = rng.integers(0, K, n).astype(np.uint32), rpnc(rng, n, R, 8), rpnc(rng, n, R, 8)
        with jg_.Context(0) as ctx:
            s = jg_.PNCStore(ctx, K, R, 8)
            s.write_rows(AP, AN)
            rows = jg_.Rows(ctx, n, R, 8)
            rows.upload(P, N, k)
            out = sh.exchange_pnc(s, rows, ex, dev)
            gP, gN = s.read_rows()
            eP, eN = orc_.pnc_merge(AP, AN, P, N, k)
            ok = np.array_equal(gP, eP) and np.array_equal(gN, eN) and int(out["received"].sum()) == n
            s.close()
            rows.close()
        q.put((ok, ""))
    except Exception as e:
        q.put((False, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_world1():
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    p = ctxm.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        ok, err = q.get(timeout=100)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert not err, err
    assert ok


# ---- the exchange inside the library (jg_comm over RCCL, csrc/comm.hip) at world size 1 ----
@pytest.mark.parametrize("full", ["0", "1"])
def test_native_exchange_world1(ctx, full, monkeypatch):
    """jg_pnc_exchange / jg_orset_exchange on a one-rank communicator — the in-place merge a single rank takes,
    and (JANUS_TEST_EXCHANGE_FULL=1) the whole multi-rank path: route, RCCL counts all-gather, the rank's own
    run, merge — bit-exact against the oracle's Merge of the whole batch either way."""
    monkeypatch.setenv("JANUS_TEST_EXCHANGE_FULL", full)
    rng = np.random.default_rng(21)
    K, R, n = 700, 64, 4000
    AP, AN = random_pnc(rng, K, R, 8, absent=False, lo=0), random_pnc(rng, K, R, 8, absent=False, lo=0)
    k, P, N = rng.integers(0, K, n).astype(np.uint32), random_pnc(rng, n, R, 8), random_pnc(rng, n, R, 8)
    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=60, n_elems=20, pool=10)
    with jg.Comm(ctx, 0, 1, jg.comm_unique_id()) as cm:
        s = jg.PNCStore(ctx, K, R, 8)
        rows = jg.Rows(ctx, n, R, 8)
        o, src = jg.ORSetStore(ctx, 0, 0), jg.ORSetStore(ctx, 0, 0)
        try:
            s.write_rows(AP, AN)
            rows.upload(P, N, k)
            out = cm.exchange_pnc(s, rows)
            assert out["sent"].tolist() == [n] and out["received"].tolist() == [n]
            st = cm.stats()
            assert st.records_received == n and st.bytes_sent == 0 and st.bytes_received == 0
            gP, gN = s.read_rows()
            eP, eN = orc.pnc_merge(AP, AN, P, N, k)
            assert np.array_equal(gP, eP) and np.array_equal(gN, eN)
            # a batch of another shape is rejected before anything moves
            bad = jg.Rows(ctx, 10, 32, 8)
            try:
                with pytest.raises(jg.JanusError) as ei:
                    cm.exchange_pnc(s, bad)
                assert ei.value.code == jg.JG_EINVAL
            finally:
                bad.close()
            o.load(La, Lr)
            src.load(Ra, Rr)
            out = cm.exchange_orset(o, src)
            assert out["received"][0].tolist() == [len(Ra)] and out["received"][1].tolist() == [len(Rr)]
            ga, gr = o.read()
            ea, er = orc.orset_merge(La, Lr, Ra, Rr)
            assert orc.same_orset(ga, gr, ea, er)
            with pytest.raises(jg.JanusError):
                cm.exchange_orset(o, o)
        finally:
            for h in (s, rows, o, src):
                h.close()


def test_native_exchange_of_empty_batches(ctx):
    with jg.Comm(ctx, 0, 1, jg.comm_unique_id()) as cm:
        s = jg.PNCStore(ctx, 10, 8, 4)
        o, src = jg.ORSetStore(ctx, 0, 0), jg.ORSetStore(ctx, 0, 0)
        try:
            assert cm.exchange_pnc(s, None)["received"].tolist() == [0]  # a rank that received nothing
            assert cm.exchange_orset(o, src)["received"][0].tolist() == [0]
            assert [len(x) for x in o.read()] == [0, 0]
        finally:
            for h in (s, o, src):
                h.close()


def test_comm_init_rejects_bad_ranks(ctx):
    uid = jg.comm_unique_id()
    for rank, world in ((1, 1), (0, 0), (0, 65)):
        with pytest.raises(jg.JanusError) as ei:
            jg.Comm(ctx, rank, world, uid)
        assert ei.value.code == jg.JG_EINVAL


# ---- one owner rule: the apply loop's jg_shard_of and the exchange's route agree ----
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_routes_follow_the_uid_owner(ctx, world):
    """Keys registered by their owner jg_shard_of(uid, world) with global ids from jg_global_key (INTEGRATION.md
    §5): jg_rows_route and jg_orset_route send every row / record of a key to exactly the rank jg_shard_of names
    (the routing safeCRDTsIndexedByuid[u.uid] decides in the reference, SafeCRDTManager.cs:136), as its local id."""
    rng = np.random.default_rng(40 + world)
    uids = [(int(a), int(b)) for a, b in rng.integers(1, 2**63, (600, 2), dtype=np.int64)]
    nxt = [0] * world
    gkey, owner, local = [], [], []
    for lo, hi in uids:
        o = jg.shard_of(lo, hi, world)
        gkey.append(jg.global_key(lo, hi, world, nxt[o]))
        owner.append(o)
        local.append(nxt[o])
        nxt[o] += 1
    gkey, owner, local = np.array(gkey, np.uint32), np.array(owner), np.array(local, np.uint32)
    pick = rng.integers(0, len(uids), 5000)  # a batch of rows of these keys, repeats included
    P, N = random_pnc(rng, len(pick), 64, 8), random_pnc(rng, len(pick), 64, 8)
    counts, k, _, _ = _route_rows(ctx, gkey[pick], P, N, world, 8)
    at = 0
    for d in range(world):
        mine = pick[owner[pick] == d]  # stable: batch order within the destination's run
        assert counts[d] == len(mine)
        assert np.array_equal(k[at:at + len(mine)], local[mine])
        at += len(mine)
    # OR-Set records of these keys (set id = global key), sorted as a store keeps them
    recs = np.zeros(len(uids) * 3, jg.REC_DTYPE)
    recs["key"] = (np.repeat(gkey.astype(np.uint64), 3) << np.uint64(32)) | np.tile(np.arange(3, dtype=np.uint64), len(uids))
    recs["tag_lo"] = rng.integers(1, 2**62, len(recs))
    recs["tag_hi"] = rng.integers(1, 2**62, len(recs))
    recs = np.sort(recs, order=["key", "tag_lo", "tag_hi"])
    recs["ord"] = np.arange(len(recs)) % 3
    ca, _, ga, _ = _route_store(ctx, recs, recs[:0], world)
    sets = (recs["key"] >> np.uint64(32)).astype(np.uint64)
    at = 0
    for d in range(world):
        n_d = int(np.sum(sets % np.uint64(world) == d))
        assert ca[d] == n_d
        got_sets = (ga["key"][at:at + n_d] >> np.uint64(32)).astype(np.uint64)
        exp_sets = sets[sets % np.uint64(world) == d] // np.uint64(world)
        assert np.array_equal(got_sets, exp_sets)
        at += n_d
    idx = {int(g): i for i, g in enumerate(gkey)}
    assert all(owner[idx[int(s)]] == int(s) % world for s in np.unique(sets))


# ---- the RCCL communicator's deadline: a rank that never joins costs a bounded wait, not a hang ----
def test_comm_init_without_peers_times_out():
    """jg_comm_init(world 2, rank 0) with no rank 1: the non-blocking communicator's init polls against
    JANUS_COMM_TIMEOUT_S (5 s here), aborts and returns JG_EHIP (run in a child process with its own limit).
    The child then closes its context and exits cleanly: nothing of the abandoned rendezvous may still run
    when static teardown does (round 4's detached rendezvous thread left a SIGSEGV at exit, rc 139,
    which this test did not see because it never looked at the child's exit status)."""
    import subprocess
    import time
    code = ("import sys, time; sys.path.insert(0, %r); import janus_gpu as jg\n"
            "ctx = jg.Context(0)\nt = time.time()\n"
            "try:\n    jg.Comm(ctx, 0, 2, jg.comm_unique_id())\nexcept jg.JanusError as e:\n"
            "    print('ERR', e.code, round(time.time() - t, 1), flush=True)\nelse:\n    print('JOINED')\n"
            "ctx.close()\n" % str(ROOT / "janus-crdt_amd"))
    env = dict(os.environ, JANUS_COMM_TIMEOUT_S="5")
    t = time.time()
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=90, env=env)
    line = [x for x in out.stdout.splitlines() if x.startswith(("ERR", "JOINED"))]
    assert line and line[0].startswith("ERR"), out.stdout + out.stderr[-3000:]
    _, rc, secs = line[0].split()
    assert int(rc) == jg.JG_EHIP
    assert 4.0 <= float(secs) < 30 and time.time() - t < 90
    assert out.returncode == 0, "child exit status %d after the timed-out rendezvous:\n%s" % (out.returncode, out.stderr[-3000:])


def _stall_worker(rank, uid_q, q):
    """Rank 0 exchanges; rank 1 joins the communicator and then never posts its half (a peer stuck mid-exchange)."""
    os.environ["JANUS_COMM_TIMEOUT_S"] = "5"
    sys.path.insert(0, str(ROOT / "janus-crdt_amd"))
    import time
    import janus_gpu as jg_
    try:
        with jg_.Context(rank) as ctx:
            if rank == 0:
                uid = jg_.comm_unique_id()
                uid_q.put(uid)
            else:
                uid = uid_q.get(timeout=60)
            cm = jg_.Comm(ctx, rank, 2, uid)
            if rank == 1:
                q.put((1, "joined", 0.0))
                time.sleep(40)  # never posts: rank 0's exchange must give up on its own
                cm.close()
                return
            s = jg_.PNCStore(ctx, 1000, 64, 8)
            rows = jg_.Rows(ctx, 500, 64, 8)
            rows.upload(np.zeros((500, 64), np.int64), np.zeros((500, 64), np.int64), np.arange(500, dtype=np.uint32) * 2 + 1)  # odd keys: rank 1's
            t = time.time()
            codes = []
            for _ in range(2):  # the second call finds the communicator aborted and fails at once
                try:
                    cm.exchange_pnc(s, rows)
                    codes.append(0)
                except jg_.JanusError as e:
                    codes.append(e.code)
            q.put((0, codes, time.time() - t))
            cm.close()  # an aborted communicator is released without touching RCCL again
            for h in (s, rows):
                h.close()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc(), 0.0))


def test_rccl_exchange_with_a_stalled_peer_times_out():
    """world 2 over RCCL, one GPU per rank; rank 1 joins and then never posts its sends / receives.
    Rank 0's jg_pnc_exchange polls its non-blocking communicator against JANUS_COMM_TIMEOUT_S (5 s), aborts it
    on its own thread and returns JG_EHIP; a second call returns JG_EHIP at once; destroy does not touch the
    aborted handle.  Needs two GPUs (RCCL refuses two ranks on one device): skipped on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    uid_q, q = ctxm.Queue(), ctxm.Queue()
    procs = [ctxm.Process(target=_stall_worker, args=(r, uid_q, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = {}
        for _ in procs:
            r, what, secs = q.get(timeout=100)
            res[r] = (what, secs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res[1][0] == "joined", res
    codes, secs = res[0]
    assert codes == [jg.JG_EHIP, jg.JG_EHIP], res
    assert 4.0 <= secs < 40, secs


# ---- the library's own exchange at world > 1: the host transport over gloo, ranks sharing device 0 ----
def _host_comm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    for p in (ROOT / "janus-crdt_amd", ROOT / "tests"):
        sys.path.insert(0, str(p))
    import torch as th
    import torch.distributed as dist
    import janus_gpu as jg_
    import oracle_ref as orc_
    import shard_ref as ref_
    from gen import random_orset_pair as rop, random_pnc as rpnc
    dist.init_process_group("gloo")

    def a2a(send, sb, rb):  # the caller's all-to-all-v (gloo over host memory)
        out = th.empty(sum(rb), dtype=th.uint8)
        inp = th.frombuffer(bytearray(send), dtype=th.uint8) if send else th.empty(0, dtype=th.uint8)
        dist.all_to_all_single(out, inp, [int(x) for x in rb], [int(x) for x in sb])
        return out.numpy().tobytes()

    try:
        rng = np.random.default_rng(321)
        K_local, R, n = 400, 64, 2500
        G = K_local * world
        AP, AN = rpnc(rng, G, R, 8, absent=False, lo=0), rpnc(rng, G, R, 8, absent=False, lo=0)
        batches = [(rng.integers(0, G, n).astype(np.uint32), rpnc(rng, n, R, 8), rpnc(rng, n, R, 8)) for _ in range(world)]
        batches[world - 1] = (batches[world - 1][0][:0], batches[world - 1][1][:0], batches[world - 1][2][:0])  # a rank sends nothing
        La, Lr, _, _ = rop(rng, n_sets=30 * world, n_elems=5, pool=8)
        recv = [rop(rng, n_sets=30 * world, n_elems=5, pool=8)[2:] for _ in range(world)]
        with jg_.Context(0) as ctx:
            cm = jg_.Comm(ctx, rank, world, alltoallv=a2a)
            s = jg_.PNCStore(ctx, K_local, R, 8)
            s.write_rows(ref_.shard_rows(AP, world, rank), ref_.shard_rows(AN, world, rank))
            k, P, N = batches[rank]
            rows = None
            if len(k):
                rows = jg_.Rows(ctx, len(k), R, 8)
                rows.upload(P, N, k)
            out = cm.exchange_pnc(s, rows)
            gP, gN = s.read_rows()
            eP, eN = AP, AN
            for kk, PP, NN in batches:
                if len(kk):
                    eP, eN = orc_.pnc_merge(eP, eN, PP, NN, kk)
            ok_pnc = np.array_equal(gP, ref_.shard_rows(eP, world, rank)) and np.array_equal(gN, ref_.shard_rows(eN, world, rank))
            exp_recv = [int(np.sum(b[0] % world == rank)) for b in batches]
            ok_counts = out["received"].tolist() == exp_recv and int(cm.stats().records_received) == sum(exp_recv)
            o = jg_.ORSetStore(ctx, 0, 0)
            o.load(ref_.shard_records(La, world, rank), ref_.shard_records(Lr, world, rank))
            src = jg_.ORSetStore(ctx, 0, 0)
            src.load(*recv[rank])
            cm.exchange_orset(o, src)
            ga, gr = o.read()
            ea, er = La, Lr
            for a, r in recv:  # ORSet.Merge of every rank's state in source-rank order
                ea, er = orc_.orset_merge(ea, er, a, r)
            ok_orset = orc_.same_orset(ga, gr, ref_.shard_records(ea, world, rank), ref_.shard_records(er, world, rank))
            for h in (s, o, src, cm) + ((rows,) if rows is not None else ()):
                h.close()
        q.put((rank, ok_pnc and ok_counts, ok_orset, ""))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, False, False, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_library_exchange_at_world_2_and_3_host_transport(world):
    """jg_pnc_exchange / jg_orset_exchange of csrc/comm.hip at world > 1 — route, counts all-gather, the plan,
    the runs, the merge — with the host transport (RCCL refuses two ranks on one GPU): every rank's shard equals
    its slice of the oracle's Merge of every rank's batch (PNCounter.Merge; ORSet.Merge in source-rank order,
    arrival ordinals included).  Only the transport differs from the RCCL path bench.py --gpus N runs."""
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_host_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=110) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, ok_pnc, ok_orset, err in res:
        assert not err, f"rank {rank}: {err}"
        assert ok_pnc and ok_orset, (rank, ok_pnc, ok_orset)
