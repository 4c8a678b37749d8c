"""GPU parity of the OR-Set path (through the C ABI) against the oracle.

Oracle = dictionary-faithful ORSet<string?> (oracle/oracle.hpp) pinned by the reference's
ORSetTests.cs known answers; comparisons are exact on canonical (sorted) record streams AND on the
reference's enumeration order (HashSet / Dictionary insertion order carried by jg_tagrec.ord:
oracle_ref.same_orset).
"""
from pathlib import Path

import numpy as np
import pytest

import janus_gpu as jg
import oracle_ref as orc
from gen import random_orset_pair, recs

pytestmark = pytest.mark.gpu


def _store(ctx, add, rem):
    s = jg.ORSetStore(ctx, len(add), len(rem))
    s.load(add, rem)
    return s


def _queries(n_sets, n_elems):
    sets = np.repeat(np.arange(n_sets + 1, dtype=np.uint32), n_elems + 2)
    elems = np.tile(np.array(list(range(n_elems + 1)) + [jg.NULL_ELEM], np.uint32), n_sets + 1)
    return sets, elems


@pytest.mark.parametrize("seed,n_sets,n_elems,pool", [(1, 4, 3, 6), (2, 50, 20, 16), (3, 300, 30, 12), (4, 7, 500, 4)])
def test_union_matches_oracle(ctx, seed, n_sets, n_elems, pool):
    rng = np.random.default_rng(seed)
    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=n_sets, n_elems=n_elems, pool=pool)
    ea, er = orc.orset_merge(La, Lr, Ra, Rr)
    a, b = _store(ctx, La, Lr), _store(ctx, Ra, Rr)
    out = jg.ORSetStore(ctx, len(La) + len(Ra), len(Lr) + len(Rr))
    try:
        jg.ORSetStore.union(a, b, out)
        ga, gr = out.read()
        assert orc.same_orset(ga, gr, ea, er)
        s, e = _queries(n_sets, min(n_elems, 40))
        assert np.array_equal(out.contains(s, e), orc.orset_contains(ea, er, s, e))
        # in-place merge of a device store and of host records give the same state
        a.merge_store(b)
        assert orc.same_orset(*a.read(), ea, er)
        # the other direction: R <- L (same records, the other enumeration order)
        fa, fr = orc.orset_merge(Ra, Rr, La, Lr)
        c = _store(ctx, Ra, Rr)
        c.merge(La, Lr)
        assert orc.same_orset(*c.read(), fa, fr)
        c.close()
    finally:
        for h in (a, b, out):
            h.close()


def _interleaved(n, start, step, tag_seed=0):
    k = np.arange(start, start + step * n, step, dtype=np.uint64) // 7
    lo = np.arange(start, start + step * n, step, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    return recs(k, lo, lo ^ np.uint64(tag_seed))


@pytest.mark.parametrize("n", [1, 2047, 2048, 2049, 50_000])
def test_union_duplicates_and_tiles(ctx, n):
    """All-duplicate, disjoint-interleaved and half-overlapping inputs across tile boundaries."""
    A = _interleaved(n, 0, 2)
    B = _interleaved(n, 1, 2)
    empty = np.empty(0, jg.REC_DTYPE)
    mix = np.unique(np.concatenate([A[::2], B[: n // 2]]))
    mix["ord"] = np.random.default_rng(n).permutation(mix.size)
    cases = [(A, A), (A, B), (A, mix), (A, empty), (empty, B)]
    for x, y in cases:
        exp, _ = orc.orset_merge(x, empty, y, empty)
        a, b = _store(ctx, x, empty), _store(ctx, y, empty)
        out = jg.ORSetStore(ctx, len(x) + len(y), 0)
        try:
            jg.ORSetStore.union(a, b, out)
            ga, gr = out.read()
            assert orc.same_stream(ga, exp, False) and gr.size == 0
        finally:
            for h in (a, b, out):
                h.close()


def test_equal_keys_long_runs(ctx):
    """One (set, elem) with 20k tags on each side: runs far longer than a tile; tag order decides."""
    rng = np.random.default_rng(9)
    lo = rng.integers(0, 1 << 62, 40_000, dtype=np.uint64)
    hi = rng.integers(0, 1 << 62, 40_000, dtype=np.uint64)
    key = np.full(40_000, (5 << 32) | 3, np.uint64)
    A = recs(key[:25_000], lo[:25_000], hi[:25_000], rng)
    B = recs(key[15_000:], lo[15_000:], hi[15_000:], rng)
    ea, er = orc.orset_merge(A, A[:100], B, B[:50])
    a, b = _store(ctx, A, A[:100]), _store(ctx, B, B[:50])
    out = jg.ORSetStore(ctx, len(A) + len(B), 150)
    try:
        jg.ORSetStore.union(a, b, out)
        ga, gr = out.read()
        assert orc.same_orset(ga, gr, ea, er)  # one HashSet of 35k tags: its whole enumeration order
        assert out.contains([5], [3])[0] == 1
    finally:
        for h in (a, b, out):
            h.close()


def test_reference_scenarios_on_gpu(ctx):
    """ORSetTests.cs:102-129 (Multiple) and :314-328 (MergeNull) replayed as record states."""
    def rec(s, e, t):
        return ((s << 32) | e, t, 7, 0)

    NUL = jg.NULL_ELEM
    # set1 = {1: t1}, set2 = {2: t2}; set1 <- set2  => 1, 2 present
    s1 = _store(ctx, np.array([rec(0, 1, 1)], jg.REC_DTYPE), np.empty(0, jg.REC_DTYPE))
    s1.merge(np.array([rec(0, 2, 2)], jg.REC_DTYPE), np.empty(0, jg.REC_DTYPE))
    assert list(s1.contains([0, 0], [1, 2])) == [1, 1]
    # set1.Remove(2): tombstone its observed tags
    s1.merge(np.empty(0, jg.REC_DTYPE), np.array([rec(0, 2, 2)], jg.REC_DTYPE))
    assert list(s1.contains([0, 0], [1, 2])) == [1, 0]
    # concurrent Add(2) on set1 vs Remove(2) on set2 -> add wins
    s1.merge(np.array([rec(0, 2, 3)], jg.REC_DTYPE), np.empty(0, jg.REC_DTYPE))
    assert list(s1.contains([0, 0], [1, 2])) == [1, 1]
    s1.close()
    # MergeNull: set1 {hi, null}; set2.Remove(null) was a no-op (empty message)
    s2 = _store(ctx, np.array([rec(0, 4, 9), rec(0, NUL, 10)], jg.REC_DTYPE), np.empty(0, jg.REC_DTYPE))
    s2.merge(np.empty(0, jg.REC_DTYPE), np.empty(0, jg.REC_DTYPE))
    assert list(s2.contains([0, 0, 0], [4, NUL, 5])) == [1, 1, 0]
    # RemoveNull: nullRemove = nullAdd -> null absent
    s2.merge(np.empty(0, jg.REC_DTYPE), np.array([rec(0, NUL, 10)], jg.REC_DTYPE))
    assert list(s2.contains([0], [NUL])) == [0]
    s2.close()


def test_unsorted_or_duplicate_input_rejected(ctx):
    a = np.array([(5, 1, 1, 0), (4, 1, 1, 1)], jg.REC_DTYPE)
    d = np.array([(5, 1, 1, 0), (5, 1, 1, 1)], jg.REC_DTYPE)
    s = jg.ORSetStore(ctx, 4, 4)
    try:
        for bad in (a, d):
            with pytest.raises(jg.JanusError) as e:
                s.load(bad, np.empty(0, jg.REC_DTYPE))
            assert e.value.code == jg.JG_ESTATE
        big = np.array([(5, 1, 1, 1 << 32)], jg.REC_DTYPE)  # ords are 32-bit on the device
        with pytest.raises(jg.JanusError) as e:
            s.load(big, np.empty(0, jg.REC_DTYPE))
        assert e.value.code == jg.JG_EINVAL
        s.load(np.sort(a, order=["key", "tag_lo", "tag_hi"]), np.empty(0, jg.REC_DTYPE))  # the store stays usable
        assert s.size() == (2, 0)
    finally:
        s.close()


def test_golden_fixture(ctx):
    z = np.load(Path(__file__).parent / "golden" / "orset_merge.npz")
    s = _store(ctx, z["La"], z["Lr"])
    try:
        s.merge(z["Ra"], z["Rr"])
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, z["out_add"], z["out_rem"])
        assert np.array_equal(s.contains(z["q_set"], z["q_elem"]), z["contains"])
    finally:
        s.close()


def test_synth_matches_host_generator(ctx):
    s = jg.ORSetStore(ctx, 0, 0)
    try:
        s.synth(77, 1000, 10, 7, 3, 2, 1)
        ga, gr = s.read()
    finally:
        s.close()
    assert np.array_equal(ga, orc.synth_orset(77, 0, 7000, 10, 7, 3))
    assert np.array_equal(gr, orc.synth_orset(77, 0, 2000, 10, 2, 1))


def test_full_size_c3(ctx):
    """BASELINE config C3: 1M sets x 10 elems; L = 100M adds + 20M tombstones, R the same size with
    50 % of its adds (and tombstones) shared.  The union is known in closed form from the generator:
    tags u in [0, 15) per group for adds, [0, 3) for tombstones — compared record for record."""
    seed, G, E = 0x4A414E5553, 10_000_000, 10
    L, R = jg.ORSetStore(ctx, 0, 0), jg.ORSetStore(ctx, 0, 0)
    out = jg.ORSetStore(ctx, 200_000_000, 40_000_000)
    try:
        L.synth(seed, G, E, 10, 0, 2, 0)
        R.synth(seed, G, E, 10, 5, 2, 1)
        jg.ORSetStore.union(L, R, out)
        assert out.size() == (150_000_000, 30_000_000)
        ga, gr = out.read()
        # records in closed form; enumeration order: L's tags (ords kept), then R's new ones (ords after
        # L's), which is ascending u = canonical order within every element
        assert np.array_equal(orc.canon(gr), orc.canon(orc.synth_orset(seed, 0, 30_000_000, E, 3, 0)))
        assert orc.enum_is_canonical(gr, True)
        del gr
        for lo in range(0, 150_000_000, 25_000_000):
            assert np.array_equal(orc.canon(ga[lo:lo + 25_000_000]), orc.canon(orc.synth_orset(seed, lo, 25_000_000, E, 15, 0))), lo
        assert orc.enum_is_canonical(ga, False)
        del ga
        rng = np.random.default_rng(3)
        sets = rng.integers(0, G // E, 100_000).astype(np.uint32)
        elems = rng.integers(0, E + 2, 100_000).astype(np.uint32)
        got = out.contains(sets, elems)
        assert np.array_equal(got, (elems < E).astype(np.uint8))  # 15 adds vs 3 tombstones: present
    finally:
        for h in (L, R, out):
            h.close()


@pytest.mark.parametrize("seed,n_sets,n_elems,n_ops,p_clear", [(1, 3, 4, 60, 0.05), (2, 40, 12, 3000, 0.01), (3, 5, 3, 500, 0.2),
                                                                (4, 300, 20, 20000, 0.002), (5, 50, 8, 30000, 0.02)])
def test_apply_ops_match_oracle(ctx, seed, n_sets, n_elems, n_ops, p_clear):
    """ORSet.Add/Remove/Clear (ORSet.cs:134-198) batched on the device in op order per set,
    interleaved across sets, on top of an existing merged state, vs the oracle op by op."""
    rng = np.random.default_rng(seed)
    La, Lr, _, _ = random_orset_pair(rng, n_sets=n_sets, n_elems=n_elems, pool=6)
    sets = rng.integers(0, n_sets + 1, n_ops).astype(np.uint32)
    elems = rng.integers(0, n_elems + 1, n_ops).astype(np.uint32)
    elems[rng.random(n_ops) < 0.1] = jg.NULL_ELEM
    r = rng.random(n_ops)
    ops = np.where(r < p_clear, 3, np.where(r < 0.55, 1, 2)).astype(np.uint8)
    lo = rng.integers(1, 1 << 63, n_ops, dtype=np.uint64)
    hi = rng.integers(1, 1 << 63, n_ops, dtype=np.uint64)
    ea, er, eres = orc.orset_apply_ops(La, Lr, sets, elems, ops, lo, hi)
    s = _store(ctx, La, Lr)
    try:
        gres = s.apply_ops(sets, elems, ops, lo, hi)
        ga, gr = s.read()
    finally:
        s.close()
    assert np.array_equal(gres, eres)
    assert orc.same_orset(ga, gr, ea, er)


def test_apply_ops_rejects_bad_op(ctx):
    s = jg.ORSetStore(ctx, 0, 0)
    try:
        with pytest.raises(jg.JanusError) as e:
            s.apply_ops([0], [1], [4], [1], [1])  # ORSetWrapper: InvalidOperationException
        assert e.value.code == jg.JG_EINVAL
        assert s.size() == (0, 0)
    finally:
        s.close()


def _rand_recs(rng, n, n_sets, n_elems, tag_pool):
    key = (rng.integers(0, n_sets, n).astype(np.uint64) << np.uint64(32)) | rng.integers(0, n_elems, n).astype(np.uint64)
    t = rng.integers(0, tag_pool, n).astype(np.uint64)
    return recs(key, t * np.uint64(0x9E3779B97F4A7C15), t, rng)


def test_chunked_chain_and_mass_clear(ctx):
    """Chunked stream layout: a store merged 8 times (each union's output — partially filled chunks
    from duplicates — is the next union's input), then a Clear of most sets (runs of EMPTY chunks in
    the middle of the stream), then more unions, Contains and reads; vs numpy set algebra and the
    oracle's ORSet ops."""
    rng = np.random.default_rng(77)
    n_sets, n_elems, pool = 400, 40, 64
    empty = np.empty(0, jg.REC_DTYPE)
    acc_a, acc_r = empty, empty
    s = jg.ORSetStore(ctx, 0, 0)
    d = jg.ORSetStore(ctx, 0, 0)
    try:
        for step in range(8):
            xa = _rand_recs(rng, 60_000, n_sets, n_elems, pool)
            xr = _rand_recs(rng, 20_000, n_sets, n_elems, pool)
            if step % 2:
                s.merge(xa, xr)                      # host records
            else:
                src = _store(ctx, xa, xr)           # device store
                s.merge_store(src)
                src.close()
            d.merge(xa, xr)
            acc_a, acc_r = orc.orset_merge(acc_a, acc_r, xa, xr)
            ga, gr = s.read()
            assert orc.same_orset(ga, gr, acc_a, acc_r), step
        # Clear sets 20..379 through the op path: most of the stream's chunks become empty
        sets = np.arange(20, 380, dtype=np.uint32)
        ops = np.full(len(sets), 3, np.uint8)
        zero = np.zeros(len(sets), np.uint64)
        ea, er, eres = orc.orset_apply_ops(acc_a, acc_r, sets, sets * 0, ops, zero, zero)
        assert np.array_equal(s.apply_ops(sets, sets * 0, ops, zero, zero), eres)
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
        q_s = rng.integers(0, n_sets, 5000).astype(np.uint32)
        q_e = rng.integers(0, n_elems, 5000).astype(np.uint32)
        assert np.array_equal(s.contains(q_s, q_e), orc.orset_contains(ea, er, q_s, q_e))
        # unions over the cleared (sparse-chunk) store, both as A and as B
        out = jg.ORSetStore(ctx, 0, 0)
        jg.ORSetStore.union(d, s, out)
        ua, ur = out.read()
        assert orc.same_orset(ua, ur, *orc.orset_merge(acc_a, acc_r, ea, er))
        jg.ORSetStore.union(s, s, out)
        ua, ur = out.read()
        assert orc.same_orset(ua, ur, ea, er)
        xa = _rand_recs(rng, 30_000, n_sets, n_elems, pool)
        s.merge(xa, empty)
        ga, _ = s.read()
        assert orc.same_stream(ga, orc.orset_merge(ea, er, xa, empty)[0], False)
        out.close()
    finally:
        s.close()
        d.close()


@pytest.mark.parametrize("seed,n_sets,n_elems,pool", [(5, 30, 12, 8), (6, 5, 200, 3), (7, 200, 4, 10)])
def test_lookup_all_matches_oracle(ctx, seed, n_sets, n_elems, pool):
    """ORSet.LookupAll order (ORSet.cs:204-227): add-only elements, then elements whose tag sets differ
    from their tombstones, then null — against the oracle's LookupAll on the merged state."""
    rng = np.random.default_rng(seed)
    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=n_sets, n_elems=n_elems, pool=pool)
    ea, er = orc.orset_merge(La, Lr, Ra, Rr)
    st = _store(ctx, La, Lr)
    try:
        st.merge(Ra, Rr)
        ids = np.arange(n_sets + 2, dtype=np.uint32)  # includes sets with no records
        got = st.lookup_all(ids)
        for s_id, g in zip(ids, got):
            exp = orc.orset_lookup_all(ea, er, int(s_id))
            assert np.array_equal(g, exp), f"set {s_id}"
        assert sum(len(g) for g in got) > 0
    finally:
        st.close()


@pytest.mark.parametrize("n_sets", [1, 37, 3000])
def test_read_sets_matches_full_read(ctx, n_sets):
    """jg_orset_read_sets (the per-set GetLastSynchronizedUpdate) = the slices of the full snapshot,
    for sets in any order, repeated, empty and out-of-range ids — on a chunked union output too."""
    rng = np.random.default_rng(n_sets)
    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=n_sets, n_elems=5, pool=6)
    s = _store(ctx, La, Lr)
    try:
        s.merge(Ra, Rr)
        A, Rm = s.read()
        q = np.concatenate([rng.permutation(n_sets + 2), [0, 0, n_sets + 5, 0xFFFFFFFF]]).astype(np.uint32)
        got = s.read_sets(q)
        for sid, (ga, gr) in zip(q, got):
            ea = A[(A["key"] >> np.uint64(32)) == sid]
            er = Rm[(Rm["key"] >> np.uint64(32)) == sid]
            assert np.array_equal(ga, ea) and np.array_equal(gr, er), sid
    finally:
        s.close()


def test_ord_renumbering_keeps_order(ctx, monkeypatch):
    """Device ords are 32-bit: a union whose ords would pass the limit renumbers its inputs first (order
    kept, ties by record order).  With the limit lowered to force a renumbering on most merges, a chain
    of merges (host records, device stores, op batches) still enumerates exactly like the oracle."""
    monkeypatch.setenv("JANUS_TEST_ORD_LIMIT", "25000")  # > any union's record count here (<= 2 x 9600)
    rng = np.random.default_rng(31)
    n_sets, n_elems, pool = 30, 8, 40
    empty = np.empty(0, jg.REC_DTYPE)
    acc_a, acc_r = empty, empty
    span = 0  # what the add stream's ords would reach without renumbering
    s = jg.ORSetStore(ctx, 0, 0)
    try:
        for step in range(10):
            xa = _rand_recs(rng, 2500, n_sets, n_elems, pool)
            xr = _rand_recs(rng, 900, n_sets, n_elems, pool)
            xa["ord"] = xa["ord"] + np.uint64(step * 500)  # ords far from 0: spans add up quickly
            if step % 3 == 0:
                src = _store(ctx, xa, xr)
                s.merge_store(src)
                src.close()
            else:
                s.merge(xa, xr)
            acc_a, acc_r = orc.orset_merge(acc_a, acc_r, xa, xr)
            span += int(xa["ord"].max()) + 1
            if step % 4 == 3:  # a batch of ops between merges
                n_ops = 200
                sets = rng.integers(0, n_sets, n_ops).astype(np.uint32)
                elems = rng.integers(0, n_elems, n_ops).astype(np.uint32)
                ops = np.where(rng.random(n_ops) < 0.5, 1, 2).astype(np.uint8)
                lo = rng.integers(1, 1 << 63, n_ops, dtype=np.uint64)
                hi = rng.integers(1, 1 << 63, n_ops, dtype=np.uint64)
                acc_a, acc_r, eres = orc.orset_apply_ops(acc_a, acc_r, sets, elems, ops, lo, hi)
                assert np.array_equal(s.apply_ops(sets, elems, ops, lo, hi), eres)
            ga, gr = s.read()
            assert orc.same_orset(ga, gr, acc_a, acc_r), step
            assert int(ga["ord"].max()) < 25000 and int(gr["ord"].max()) < 25000
        assert span > 25000  # so the chain above did renumber
    finally:
        s.close()


def test_enumeration_order_scenario(ctx):
    """The oracle's Json_ORSetEnumerationOrder KAT (oracle/test_kat.cpp) on the device: tags enumerate in
    insertion order, not sorted; the tombstone Dictionary in first-Remove order; Merge appends."""
    K = lambda e: (0 << 32) | e  # noqa: E731
    b, a, NUL = 1, 0, jg.NULL_ELEM
    t3, t1, t2, t9 = (3, 0), (1, 0), (2, 0), (9, 0)
    s = jg.ORSetStore(ctx, 0, 0)
    r = jg.ORSetStore(ctx, 0, 0)
    try:
        # s: Add(b,t3) Add(a,t1) Add(b,t2) Add(null,t9) Add(null,t1); Remove(b); Remove(a)
        res = s.apply_ops([0] * 7, [b, a, b, NUL, NUL, b, a], [1, 1, 1, 1, 1, 2, 2],
                          [t3[0], t1[0], t2[0], t9[0], t1[0], 0, 0], [0] * 7)
        assert list(res) == [1] * 7
        ga, gr = s.read()
        va, vr = orc.enum_view(ga, False), orc.enum_view(gr, True)
        assert [(int(k), int(lo)) for k, lo, _ in va] == [(K(a), 1), (K(b), 3), (K(b), 2), (K(NUL), 9), (K(NUL), 1)]
        assert [(int(k), int(lo)) for k, lo, _ in vr] == [(K(b), 3), (K(b), 2), (K(a), 1)]
        # r: Add(a,t9) Add(b,t2); then merge s's state: a gets t1 appended, b gets t3 appended
        r.apply_ops([0, 0], [a, b], [1, 1], [t9[0], t2[0]], [0, 0])
        r.merge_store(s)
        ga, gr = r.read()
        va, vr = orc.enum_view(ga, False), orc.enum_view(gr, True)
        assert [(int(k), int(lo)) for k, lo, _ in va] == [(K(a), 9), (K(a), 1), (K(b), 2), (K(b), 3), (K(NUL), 9), (K(NUL), 1)]
        assert [(int(k), int(lo)) for k, lo, _ in vr] == [(K(b), 3), (K(b), 2), (K(a), 1)]
    finally:
        s.close()
        r.close()
