"""GPU parity of the PN-Counter path (through the C ABI) against the oracle.

Bit-exact: every comparison is array_equal.  Oracle = dictionary-faithful PNCounter
(oracle/oracle.hpp), pinned by the reference's known-answer tests.
"""
import numpy as np
import pytest

import janus_gpu as jg
import oracle_ref as orc
from gen import random_pnc

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1), (3, 5), (257, 64), (100, 130), (1000, 7), (4097, 2)]


@pytest.mark.parametrize("eb", [4, 8])
@pytest.mark.parametrize("n_keys,R", SHAPES)
def test_merge_identity_rows(ctx, eb, n_keys, R):
    rng = np.random.default_rng(n_keys * 131 + R * 7 + eb)
    AP, AN = random_pnc(rng, n_keys, R, eb, absent=False), random_pnc(rng, n_keys, R, eb, absent=False)
    BP, BN = random_pnc(rng, n_keys, R, eb), random_pnc(rng, n_keys, R, eb)
    s = jg.PNCStore(ctx, n_keys, R, eb)
    try:
        s.write_rows(AP, AN)
        s.merge_rows(BP, BN)
        P, N = s.read_rows()
    finally:
        s.close()
    eP, eN = orc.pnc_merge(AP, AN, BP, BN)
    assert np.array_equal(P, eP) and np.array_equal(N, eN)


@pytest.mark.parametrize("eb", [4, 8])
def test_merge_indexed_repeated_keys(ctx, eb):
    """A committed batch holds many states of the same key (SafeCRDTManager.cs:122-146)."""
    rng = np.random.default_rng(5 + eb)
    n_keys, R, M = 300, 9, 5000
    AP, AN = random_pnc(rng, n_keys, R, eb, absent=False), random_pnc(rng, n_keys, R, eb, absent=False)
    BP, BN = random_pnc(rng, M, R, eb), random_pnc(rng, M, R, eb)
    keys = rng.integers(0, 20, M).astype(np.uint32)  # hot keys
    s = jg.PNCStore(ctx, n_keys, R, eb)
    try:
        s.write_rows(AP, AN)
        s.merge_rows(BP, BN, keys)
        P, N = s.read_rows()
    finally:
        s.close()
    eP, eN = orc.pnc_merge(AP, AN, BP, BN, keys)
    assert np.array_equal(P, eP) and np.array_equal(N, eN)


@pytest.mark.parametrize("eb", [4, 8])
@pytest.mark.parametrize("R", [32, 64, 130])
def test_merge_indexed_unique_and_repeated_rows(ctx, eb, R):
    """The grouped path (R x width a whole number of 16-B vectors, R >= 32): every key's rows are folded
    by its list head (one A row load and store; a key seen once is its own list); heads are reset, so the
    next batch over the same keys merges exactly too.  Round 3 mixes unique, 7-, 64-, 65- and 400-row keys
    in one batch."""
    rng = np.random.default_rng(R * 10 + eb)
    n_keys, M = 20_000, 6_000
    AP, AN = random_pnc(rng, n_keys, R, eb, absent=False), random_pnc(rng, n_keys, R, eb, absent=False)
    s = jg.PNCStore(ctx, n_keys, R, eb)
    eP, eN = AP, AN
    mixed = np.concatenate([np.arange(2000, 4000), np.repeat(np.arange(10), 7), np.repeat([77, 78], 64), np.repeat([5000], 65),
                            np.repeat([6000], 400)])
    try:
        s.write_rows(AP, AN)
        for rnd in range(4):
            if rnd == 3:
                keys = rng.permutation(mixed).astype(np.uint32)
            else:
                keys = rng.integers(0, n_keys if rnd != 1 else 50, M).astype(np.uint32)  # mostly unique / hot keys
            BP, BN = random_pnc(rng, keys.size, R, eb), random_pnc(rng, keys.size, R, eb)
            s.merge_rows(BP, BN, keys)
            eP, eN = orc.pnc_merge(eP, eN, BP, BN, keys)
        P, N = s.read_rows()
    finally:
        s.close()
    assert np.array_equal(P, eP) and np.array_equal(N, eN)


def test_grouped_heads_across_the_generation_wrap(ctx, monkeypatch):
    """Grouped-merge list heads carry the batch generation (gen << 32 | row); after 2^32 - 1 batches the heads
    are cleared and the generation restarts.  A store whose first generation is set just below the wrap
    (JANUS_TEST_HEAD_GEN) merges batches of repeated keys before, at and after it exactly."""
    monkeypatch.setenv("JANUS_TEST_HEAD_GEN", str(2**32 - 3))
    rng = np.random.default_rng(91)
    n_keys, R, eb, M = 5000, 64, 8, 3000
    AP, AN = random_pnc(rng, n_keys, R, eb, absent=False), random_pnc(rng, n_keys, R, eb, absent=False)
    s = jg.PNCStore(ctx, n_keys, R, eb)
    eP, eN = AP, AN
    try:
        s.write_rows(AP, AN)
        for rnd in range(6):  # generations 2^32-2, 2^32-1, then 1, 2, 3, 4 after the clear
            keys = rng.integers(0, 400 if rnd % 2 else n_keys, M).astype(np.uint32)
            BP, BN = random_pnc(rng, M, R, eb), random_pnc(rng, M, R, eb)
            s.merge_rows(BP, BN, keys)
            eP, eN = orc.pnc_merge(eP, eN, BP, BN, keys)
            P, N = s.read_rows()
            assert np.array_equal(P, eP) and np.array_equal(N, eN), rnd
    finally:
        s.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_merge_batch_device_rows(ctx, eb):
    rng = np.random.default_rng(21)
    n_keys, R = 777, 13
    AP, AN = random_pnc(rng, n_keys, R, eb, absent=False), random_pnc(rng, n_keys, R, eb, absent=False)
    BP, BN = random_pnc(rng, n_keys, R, eb), random_pnc(rng, n_keys, R, eb)
    CP, CN = random_pnc(rng, 50, R, eb), random_pnc(rng, 50, R, eb)
    ck = rng.integers(0, n_keys, 50).astype(np.uint32)
    s = jg.PNCStore(ctx, n_keys, R, eb)
    b = jg.Rows(ctx, n_keys, R, eb)
    c = jg.Rows(ctx, 50, R, eb)
    try:
        s.write_rows(AP, AN)
        b.upload(BP, BN)
        c.upload(CP, CN, ck)
        s.merge_batch(b, async_=True)
        s.merge_batch(c, async_=True)
        ctx.fence()
        P, N = s.read_rows()
    finally:
        for h in (s, b, c):
            h.close()
    eP, eN = orc.pnc_merge(AP, AN, BP, BN)
    eP, eN = orc.pnc_merge(eP, eN, CP, CN, ck)
    assert np.array_equal(P, eP) and np.array_equal(N, eN)


def test_partial_identity_and_scatter_write_read(ctx):
    rng = np.random.default_rng(8)
    s = jg.PNCStore(ctx, 100, 6, 8)
    try:
        AP, AN = random_pnc(rng, 100, 6, 8, absent=False), random_pnc(rng, 100, 6, 8, absent=False)
        s.write_rows(AP, AN)
        keys = rng.permutation(100)[:17].astype(np.uint32)
        P2, N2 = random_pnc(rng, 17, 6, 8, absent=False), random_pnc(rng, 17, 6, 8, absent=False)
        s.write_rows(P2, N2, keys)
        AP[keys], AN[keys] = P2, N2
        gP, gN = s.read_rows(keys[::-1])
        assert np.array_equal(gP, AP[keys[::-1]]) and np.array_equal(gN, AN[keys[::-1]])
        BP, BN = random_pnc(rng, 40, 6, 8), random_pnc(rng, 40, 6, 8)
        s.merge_rows(BP, BN)  # rows 0..39 only
        eP, eN = orc.pnc_merge(AP, AN, BP, BN)
        P, N = s.read_rows()
        assert np.array_equal(P, eP) and np.array_equal(N, eN)
    finally:
        s.close()


@pytest.mark.parametrize("eb", [4, 8])
@pytest.mark.parametrize("R", [1, 4, 64, 65, 200])
def test_values_checked_sum(ctx, eb, R):
    """PNCounter.Get: order-sensitive checked Sum -> overflow flag; unchecked subtraction."""
    rng = np.random.default_rng(R * 3 + eb)
    info = np.iinfo(np.int32 if eb == 4 else np.int64)
    n = 600
    P = random_pnc(rng, n, R, eb, absent=False, lo=info.min // (2 * R), hi=info.max // (2 * R))
    N = random_pnc(rng, n, R, eb, absent=False, lo=info.min // (2 * R), hi=info.max // (2 * R))
    # keys 0-49 overflow at the 2nd prefix; keys 50-99 hold the same multiset in an order that
    # never overflows (the checked Sum is order-sensitive); keys 100-199 wrap in ΣP - ΣN.
    P[:200] = 0
    N[:200] = 0
    P[:100, 0] = info.max
    if R >= 3:
        P[:50, 1], P[:50, 2] = 1, -5
        P[50:100, 1], P[50:100, 2] = -5, 1
    elif R == 2:
        P[:50, 1] = 1
    P[100:200, 0] = 1
    N[100:200, 0] = info.min
    s = jg.PNCStore(ctx, n, R, eb)
    try:
        s.write_rows(P, N)
        v, o = s.values()
        keys = rng.integers(0, n, 333).astype(np.uint32)
        v2, o2 = s.values(keys)
    finally:
        s.close()
    ev, eo = orc.pnc_values(P, N)
    assert np.array_equal(o, eo) and np.array_equal(v, ev)
    assert np.array_equal(v2, ev[keys]) and np.array_equal(o2, eo[keys])
    if R >= 2:
        assert eo[:50].all() and not eo[50:200].any()


@pytest.mark.parametrize("eb", [4, 8])
def test_apply_ops_wrapping(ctx, eb):
    rng = np.random.default_rng(40 + eb)
    n_keys, R, n_ops = 50, 4, 20000
    info = np.iinfo(np.int32 if eb == 4 else np.int64)
    P = random_pnc(rng, n_keys, R, eb, absent=False)
    N = random_pnc(rng, n_keys, R, eb, absent=False)
    key = rng.integers(0, 5, n_ops).astype(np.uint32)  # hot keys
    col = rng.integers(0, R, n_ops).astype(np.uint32)
    delta = rng.integers(info.min // 2, info.max // 2, n_ops).astype(np.int64)
    is_n = rng.integers(0, 2, n_ops).astype(np.uint8)
    s = jg.PNCStore(ctx, n_keys, R, eb)
    try:
        s.write_rows(P, N)
        s.apply_ops(key, col, delta, is_n)
        gP, gN = s.read_rows()
    finally:
        s.close()
    eP, eN = orc.pnc_apply_ops(P, N, key, col, delta, is_n)
    assert np.array_equal(gP, eP) and np.array_equal(gN, eN)


def test_golden_fixture(ctx):
    from pathlib import Path
    z = np.load(Path(__file__).parent / "golden" / "pnc_merge_i32.npz")
    s = jg.PNCStore(ctx, 256, 8, 4)
    try:
        s.write_rows(z["AP"], z["AN"])
        s.merge_rows(z["BP"], z["BN"], z["keys"])
        P, N = s.read_rows()
        v, o = s.values()
    finally:
        s.close()
    assert np.array_equal(P, z["outP"]) and np.array_equal(N, z["outN"])
    assert np.array_equal(v, z["values"]) and np.array_equal(o, z["ovf"])


@pytest.mark.parametrize("eb", [4, 8])
def test_synth_matches_host_generator(ctx, eb):
    seed, n_keys, R = 0x4A414E5553, 321, 11
    s = jg.PNCStore(ctx, n_keys, R, eb)
    r = jg.Rows(ctx, 40, R, eb)
    try:
        s.synth(seed)
        r.synth(seed, key0=100)
        P, N = s.read_rows()
        s2 = jg.PNCStore(ctx, 40, R, eb)
        s2.merge_batch(r)  # zero store max'd with rows == rows with ABSENT -> untouched 0
        bP, bN = s2.read_rows()
        s2.close()
    finally:
        s.close()
        r.close()
    assert np.array_equal(P, orc.synth_pnc(seed, 0, 0, n_keys, R, eb))
    assert np.array_equal(N, orc.synth_pnc(seed, 1, 0, n_keys, R, eb))
    hp = orc.synth_pnc(seed, 2, 100, 40, R, eb)
    assert np.array_equal(bP, np.where(hp == np.iinfo(hp.dtype).min, 0, np.maximum(hp, 0)))


def test_full_size_c2_properties(ctx):
    """BASELINE config C2 (10M keys x 64 replicas, int64): merge on device-resident synthetic data,
    then check all ~3000 sampled rows exactly against the host oracle on the same synthetic rows, plus
    idempotence (merging the same batch again changes nothing)."""
    seed, n_keys, R = 0x4A414E5553, 10_000_000, 64
    s = jg.PNCStore(ctx, n_keys, R, 8)
    b = jg.Rows(ctx, n_keys, R, 8)
    try:
        s.synth(seed)
        b.synth(seed)
        s.merge_batch(b)
        rng = np.random.default_rng(1)
        keys = np.unique(np.concatenate([rng.integers(0, n_keys, 3000), [0, n_keys - 1]])).astype(np.uint32)
        P1, N1 = s.read_rows(keys)
        s.merge_batch(b)
        P2, N2 = s.read_rows(keys)
    finally:
        s.close()
        b.close()
    for i, k in enumerate(keys):  # every sampled row against the oracle (was the first 300)
        AP, AN = orc.synth_pnc(seed, 0, int(k), 1, R, 8), orc.synth_pnc(seed, 1, int(k), 1, R, 8)
        BP, BN = orc.synth_pnc(seed, 2, int(k), 1, R, 8), orc.synth_pnc(seed, 3, int(k), 1, R, 8)
        eP, eN = orc.pnc_merge(AP, AN, BP, BN)
        assert np.array_equal(P1[i], eP[0]) and np.array_equal(N1[i], eN[0]), k
    assert np.array_equal(P1, P2) and np.array_equal(N1, N2)


def test_full_size_c4_shard_properties(ctx):
    """BASELINE config C4 (200M keys x 128 replicas over 8 GPUs): one GPU's shard, 25M keys x 128 replicas
    int64 — A and B resident, 102.4 GB — merged on the device; 3.2G cells per array, so cell offsets pass
    2^32 (64-bit indexing).  Sampled rows (first, last, random) exactly against the oracle, Get on them
    against the oracle's checked sums, then idempotence."""
    seed, n_keys, R = 0x4A414E5553 + 7, 25_000_000, 128
    s = jg.PNCStore(ctx, n_keys, R, 8)
    b = jg.Rows(ctx, n_keys, R, 8)
    try:
        s.synth(seed)
        b.synth(seed)
        s.merge_batch(b)
        rng = np.random.default_rng(4)
        keys = np.unique(np.concatenate([rng.integers(0, n_keys, 2000), [0, 1, n_keys // 2, n_keys - 2, n_keys - 1]])).astype(np.uint32)
        P1, N1 = s.read_rows(keys)
        v1, o1 = s.values(keys)
        s.merge_batch(b)
        P2, N2 = s.read_rows(keys)
    finally:
        s.close()
        b.close()
    check = np.concatenate([np.arange(200), np.arange(keys.size - 5, keys.size)])
    for i in check:
        k = int(keys[i])
        AP, AN = orc.synth_pnc(seed, 0, k, 1, R, 8), orc.synth_pnc(seed, 1, k, 1, R, 8)
        BP, BN = orc.synth_pnc(seed, 2, k, 1, R, 8), orc.synth_pnc(seed, 3, k, 1, R, 8)
        eP, eN = orc.pnc_merge(AP, AN, BP, BN)
        assert np.array_equal(P1[i], eP[0]) and np.array_equal(N1[i], eN[0]), k
        ev, eo = orc.pnc_values(eP, eN)
        assert v1[i] == ev[0] and o1[i] == eo[0], k
    assert np.array_equal(P1, P2) and np.array_equal(N1, N2)


def test_errors_are_codes(ctx):
    with pytest.raises(jg.JanusError) as e:
        jg.PNCStore(ctx, 10, 4, 3)
    assert e.value.code == jg.JG_EINVAL
    s = jg.PNCStore(ctx, 10, 4, 8)
    try:
        with pytest.raises(jg.JanusError) as e:
            s.merge_rows(np.zeros((1, 4), np.int64), np.zeros((1, 4), np.int64), [10])
        assert e.value.code == jg.JG_EINVAL
        r = jg.Rows(ctx, 2, 5, 8)
        with pytest.raises(jg.JanusError) as e:
            s.merge_batch(r)
        assert e.value.code == jg.JG_ETYPE
        r.close()
        with pytest.raises(jg.JanusError):
            s.apply_ops([0], [4], [1], [0])
    finally:
        s.close()
