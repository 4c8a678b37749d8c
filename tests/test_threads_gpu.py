"""Concurrent callers on one context (include/janus_gpu.h threading rule): the reference merges
prospective copies on many receiver threads under lock(crdt) (MergeSharp/MergeSharp/ReplicationManager.cs:333)
while readers query (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:64-78).  The context's scratch buffers and stream
are shared by all of its handles, so every call holds the context's lock; these tests hammer one
context from several threads (ctypes releases the GIL during each call) and check every answer
against the oracle computed up front."""
import threading

import numpy as np
import pytest

import oracle_ref as orc
from gen import random_orset_pair, random_pnc

pytestmark = pytest.mark.gpu


def test_concurrent_readers_and_merges_on_one_context(ctx):
    import janus_gpu as jg
    rng = np.random.default_rng(77)
    K, R = 4096, 8
    AP = random_pnc(rng, K, R, 8, absent=False, lo=0, hi=1 << 40)
    AN = random_pnc(rng, K, R, 8, absent=False, lo=0, hi=1 << 40)
    store = jg.PNCStore(ctx, K, R, 8)
    store.write_rows(AP, AN)
    ev, eo = orc.pnc_values(AP, AN)

    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=64, n_elems=40, pool=12)
    os_ = jg.ORSetStore(ctx, len(La), len(Lr))
    os_.load(La, Lr)
    sets = np.repeat(np.arange(64, dtype=np.uint32), 41)
    elems = np.tile(np.array(list(range(40)) + [jg.NULL_ELEM], np.uint32), 64)
    want_c = orc.orset_contains(La, Lr, sets, elems)

    # a second PN-Counter store on the same context takes merges while the readers run
    BP = random_pnc(rng, 2048, R, 8, lo=0, hi=1 << 40)
    BN = random_pnc(rng, 2048, R, 8, lo=0, hi=1 << 40)
    keys = rng.integers(0, K, 2048).astype(np.uint32)
    other = jg.PNCStore(ctx, K, R, 8)
    other.write_rows(AP, AN)
    eP, eN = orc.pnc_merge(AP, AN, BP, BN, keys)

    errors = []

    def reader_pnc():
        try:
            for _ in range(40):
                v, o = store.values()
                if not (np.array_equal(v, ev) and np.array_equal(o, eo)):
                    errors.append("pnc values differ")
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    def reader_orset():
        try:
            for _ in range(40):
                if not np.array_equal(os_.contains(sets, elems), want_c):
                    errors.append("orset contains differs")
                    return
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    def merger():
        try:
            for i in range(8):  # idempotent: merging the same batch again leaves the same state
                other.merge_rows(BP, BN, keys)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=f) for f in (reader_pnc, reader_pnc, reader_orset, reader_orset, merger)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), "a caller did not finish"
    assert not errors, errors
    P, N = other.read_rows()
    assert np.array_equal(P, eP) and np.array_equal(N, eN)
    for h in (store, os_, other):
        h.close()
