"""GPU parity of the committed-wave apply loop behind the C ABI (jg_apply_committed / jg_apply_block,
csrc/node.hip) against the oracle.

The checker restates SafeCRDTManager.HandleAfterConsensusUpdates (BFT-CRDT/CRDTManagers/
SafeCRDTManager.cs:109-160) over the oracle's per-type stable-apply loops (tests/oracle_ref.py:
pnc_apply_json = Decode + PNCounter.Merge, orset_apply_json = Decode + ORSet.Merge): skip
ManagerMsg_Create and Guid.Empty (:133-134) and unknown uids (:136), stop at the first state a Decode /
Merge rejects (the apply Task faults there), and TryRemove each applied message's identity from the
tracker, notifying its origin in commit order (:141-142).  Comparisons are exact: every PN-Counter row
(values and replica columns), the OR-Set record streams with their enumeration order, the completed
origins in order, the cut, and the entries left in the tracker.
"""
import numpy as np
import pytest

import janus_gpu as jg
import jsongen as J
import oracle_ref as orc

pytestmark = pytest.mark.gpu

R, EB = 6, 4


class Model:
    """The oracle node: PN-Counter rows, OR-Set model, uid table, tracker."""

    def __init__(self, n_pnc, rng):
        self.P = np.zeros((n_pnc, R), np.int32)
        self.N = np.zeros((n_pnc, R), np.int32)
        self.cols = np.zeros((n_pnc, R), jg.GUID_DTYPE)
        self.ncols = np.zeros(n_pnc, np.uint32)
        own = J.random_guids(rng, n_pnc)  # the stable instance's own replica (column 0, PNCounters.cs:73-81)
        for k, g in enumerate(own):
            self.cols[k, 0] = g
            self.ncols[k] = 1
        self.own = own
        self.names, self.state = {}, {}
        self.keys = {}  # uid -> (type, idx)
        self.tracker = {}  # seq -> origin (insertion order = dict order)

    def apply(self, wave, block=False):
        """wave: list of (uid, type, seq, payload).  Returns (completed origins, cut or None)."""
        live = []  # (commit index, type, idx, payload)
        cut = None
        for i, (uid, t, seq, p) in enumerate(wave):
            if t == 0 or uid == (0, 0):
                continue
            if uid not in self.keys:
                if block:
                    cut = i
                    break
                continue
            kt, idx = self.keys[uid]
            ok = orc.json_accepts_pnc(p, EB) if kt == 0 else (
                (d := orc.json_decode_orset(p)) is not None and all(is_null or tags for _, is_null, _, tags in d))
            if not ok:
                cut = i
                break
            live.append((i, kt, idx, p, seq))
        pm = [(idx, p) for _, kt, idx, p, _ in live if kt == 0]
        if pm:
            self.P, self.N, self.cols, self.ncols, bad, rc = orc.pnc_apply_json(self.P, self.N, self.cols, self.ncols,
                                                                                [x[0] for x in pm], [x[1] for x in pm], EB)
            assert bad is None, "the model's acceptance check disagrees with the oracle's loop"
        om = [(idx, p) for _, kt, idx, p, _ in live if kt == 1]
        ea, er, bad, _ = orc.orset_apply_json([x[0] for x in om], [x[1] for x in om], self.names, self.state)
        assert bad is None
        self.orset = (ea, er)
        done = [self.tracker.pop(seq) for _, _, _, _, seq in live if seq in self.tracker]
        return done, cut


def _setup(ctx, rng, n_pnc, n_set):
    pnc = jg.PNCStore(ctx, n_pnc, R, EB)
    st = jg.ORSetStore(ctx)
    node = jg.Node(pnc, st)
    tr = jg.Tracker(ctx)
    m = Model(n_pnc, rng)
    pnc.intern(np.arange(n_pnc), [g[0] for g in m.own], [g[1] for g in m.own])
    uids = J.random_guids(rng, n_pnc + n_set)
    types = [0] * n_pnc + [1] * n_set
    idx = list(range(n_pnc)) + list(range(n_set))
    node.register([u[0] for u in uids], [u[1] for u in uids], types, idx)
    for u, t, i in zip(uids, types, idx):
        m.keys[u] = (t, i)
    return pnc, st, node, tr, m, uids


def _wave(rng, m, uids, n_pnc, n_set, n, pcl, ocl, seq0, bad_at=None, extras=True):
    """n messages: PN-Counter and OR-Set states of registered keys, plus (extras) creation messages,
    key-space (Guid.Empty) messages and states of unknown uids.  Half the states are tracked; some
    identities repeat inside the wave (only the first occurrence completes)."""
    wave, seqs = [], []
    for i in range(n):
        r = rng.random()
        if extras and r < 0.03:
            wave.append(((int(rng.integers(1, 2**62)), 5), 1, 0, b'{"pVector":{},"nVector":{}}'))  # unknown uid
            continue
        if extras and r < 0.05:
            wave.append((uids[int(rng.integers(0, len(uids)))], 0, 0, b"junk: ManagerMsg_Create"))  # creation message
            continue
        if extras and r < 0.06:
            wave.append(((0, 0), 1, 0, b"key space"))  # Guid.Empty (the replicated key-space set)
            continue
        k = int(rng.integers(0, n_pnc + n_set))
        if k < n_pnc:
            p = pcl.message(k)
        else:
            sid = k - n_pnc
            a, rr, na, nr = ocl.state(sid)
            p = J.encode_orset(a, rr, na, nr)
        seq = 0
        if rng.random() < 0.5:
            if seqs and rng.random() < 0.05:
                seq = seqs[int(rng.integers(0, len(seqs)))]  # the same message object committed twice
            else:
                seq = seq0 + i + 1
                seqs.append(seq)
                origin = int(rng.integers(1, 1000))
                m.tracker[seq] = origin
        wave.append((uids[k], 1, seq, p))
    if bad_at is not None:
        u, t, s, _ = wave[bad_at]
        wave[bad_at] = (uids[0], 1, s, b'{"pVector":{}}')  # a PNCounterMsg Decode rejects (missing nVector)
    return wave


def _run(ctx, seed, n_pnc, n_set, waves, n, chunk=None, monkeypatch=None, bad=False, block=False, shard=None, pinned=False, stream=0):
    rng = np.random.default_rng(seed)
    if chunk and monkeypatch:
        monkeypatch.setenv("JANUS_WAVE_CHUNK", str(chunk))
        monkeypatch.setenv("JANUS_HOST_PAR_MIN", "1")
    pnc, st, node, tr, m, uids = _setup(ctx, rng, n_pnc, n_set)
    if shard:
        node.set_shard(*shard)
    pcl = J.Cluster(rng, n_pnc, R - 1, EB, stable=None)
    ocl = J.ORSetCluster(rng, n_set)
    added = set()
    try:
        for w in range(waves):
            bad_at = int(rng.integers(0, n)) if bad else None
            wave = _wave(rng, m, uids, n_pnc, n_set, n, pcl, ocl, seq0=w * 10 * n, bad_at=bad_at, extras=not block)
            new = [(s, o) for s, o in m.tracker.items() if s not in added]
            if new:
                tr.add([s for s, _ in new], [o for _, o in new])
                added.update(s for s, _ in new)
            exp_done, exp_cut = m.apply(wave, block=block)
            lo = [x[0][0] for x in wave]
            hi = [x[0][1] for x in wave]
            types = [x[1] for x in wave]
            seqs = [x[2] for x in wave]
            msgs = [x[3] for x in wave]
            if block:
                cut, rc = node.apply_block(lo, hi, types, msgs)
                done = []
            elif stream:  # the wave handed over in `stream` parts of random sizes (jg_apply_stream_*)
                cuts = sorted(set(rng.integers(0, len(wave) + 1, stream - 1).tolist()) | {0, len(wave)})
                parts = [(lo[a:b], hi[a:b], types[a:b], seqs[a:b], msgs[a:b]) for a, b in zip(cuts, cuts[1:])]
                done, cut, rc = node.apply_stream(tr, parts, pinned=ctx if pinned else None)
            else:
                done, cut, rc = node.apply_committed(tr, lo, hi, types, seqs, msgs, pinned=ctx if pinned else None)
            assert cut == exp_cut, (cut, exp_cut)
            assert (rc == jg.JG_OK) == (exp_cut is None)
            assert list(done) == exp_done
            P, N = pnc.read_rows()
            assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
            g, nc = pnc.columns(np.arange(n_pnc))
            assert np.array_equal(nc, m.ncols)
            assert all(np.array_equal(g[k, :nc[k]], m.cols[k, :nc[k]]) for k in range(n_pnc))
            ga, gr = st.read()
            assert orc.same_orset(ga, gr, *m.orset)
            if not block:
                assert tr.size() == len(m.tracker)
                left = list(m.tracker)
                if left:
                    assert tr.contains(left).all()
            s = node.stats()
            assert s["msgs_applied"] == sum(1 for i, (u, t, _, _) in enumerate(wave)
                                            if t != 0 and u in m.keys and (exp_cut is None or i < exp_cut))
            st.names_sync()  # nothing pending: the store's element table is the wave path's own
    finally:
        for h in (node, tr, pnc, st):
            h.close()


@pytest.mark.parametrize("seed,n_pnc,n_set,waves,n", [(1, 20, 8, 3, 300), (2, 200, 60, 3, 4000), (3, 3000, 500, 2, 30000)])
def test_mixed_waves_match_oracle(ctx, seed, n_pnc, n_set, waves, n):
    _run(ctx, seed, n_pnc, n_set, waves, n)


def test_mixed_waves_many_chunks(ctx, monkeypatch):
    """Waves cut into 97-message chunks gathered by every worker: chunk-relative offsets rebased, classify
    and both parses per chunk, completions across chunks."""
    _run(ctx, 5, 150, 40, 3, 2500, chunk=97, monkeypatch=monkeypatch)


@pytest.mark.parametrize("chunk,bad", [(None, False), (83, False), (61, True)])
def test_direct_upload_from_pinned_payloads(ctx, monkeypatch, chunk, bad):
    """Payloads the caller holds in page-locked memory (jg_host_alloc) are uploaded in place, chunk by chunk
    (no gather into the library's staging): the same stores, completions and cut as the gathered path."""
    if chunk:
        _run(ctx, 11, 120, 40, 3, 2000, chunk=chunk, monkeypatch=monkeypatch, bad=bad, pinned=True)
    else:
        _run(ctx, 13, 200, 60, 3, 4000, bad=bad, pinned=True)


@pytest.mark.parametrize("chunk", [None, 61])
def test_rejected_state_cuts_the_wave(ctx, monkeypatch, chunk):
    """A state Decode rejects stops the loop there: the prefix is applied (both kinds) and its completions
    reported, nothing after it, and the tracker keeps the entries of the messages not applied."""
    _run(ctx, 7, 80, 30, 4, 1500, chunk=chunk, monkeypatch=monkeypatch, bad=True)


def test_block_receipt_unknown_uid(ctx):
    """jg_apply_block (ReplicationManager.ReceivedUpdateSyncMsg): a CRDT state of an unknown uid stops the
    block there with JG_EINVAL (KeyNotFoundException), after the states before it."""
    rng = np.random.default_rng(11)
    pnc, st, node, tr, m, uids = _setup(ctx, rng, 30, 10)
    pcl = J.Cluster(rng, 30, R - 1, EB, stable=None)
    try:
        wave = [(uids[k], 1, 0, pcl.message(k)) for k in rng.integers(0, 30, 200).tolist()]
        wave[120] = ((123, 456), 1, 0, b'{"pVector":{},"nVector":{}}')
        exp_done, exp_cut = m.apply(wave, block=True)
        cut, rc = node.apply_block([x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave], [x[3] for x in wave])
        assert cut == exp_cut == 120 and rc == jg.JG_EINVAL
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
    finally:
        for h in (node, tr, pnc, st):
            h.close()


def test_shard_shortcut_matches_the_table(ctx):
    """A node declared shard r of w gathers only its shard's states (jg_shard_of): the same result as the
    uid table's skip.  A registered uid of another shard turns the shortcut off, and set_shard rescans."""
    rng = np.random.default_rng(13)
    world = 3
    pnc, st, node, tr, m, uids = _setup(ctx, rng, 40, 12)
    try:
        mine = [u for u in uids if jg.shard_of(u[0], u[1], world) == 1]
        assert 0 < len(mine) < len(uids)
        node.set_shard(1, world)  # foreign uids are registered: the shortcut stays off
        pcl = J.Cluster(rng, 40, R - 1, EB, stable=None)
        ocl = J.ORSetCluster(rng, 12)
        wave = _wave(rng, m, uids, 40, 12, 800, pcl, ocl, seq0=0)
        exp_done, exp_cut = m.apply(wave)
        done, cut, rc = node.apply_committed(None, [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave], None,
                                             [x[3] for x in wave])
        assert cut is None and rc == jg.JG_OK
        s = node.stats()
        assert s["msgs_uploaded"] == len(wave)  # the table decided
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
    finally:
        for h in (node, tr, pnc, st):
            h.close()
    # a node that holds only its shard's keys: the gather drops the other shards' states
    rng = np.random.default_rng(14)
    pnc = jg.PNCStore(ctx, 40, R, EB)
    node = jg.Node(pnc, None)
    try:
        keys = J.random_guids(rng, 120)
        own = [k for k in keys if jg.shard_of(k[0], k[1], world) == 2][:40]
        node.register([k[0] for k in own], [k[1] for k in own], [0] * len(own), list(range(len(own))))
        node.set_shard(2, world)
        msgs, lo, hi = [], [], []
        for i in range(600):
            k = keys[int(rng.integers(0, len(keys)))]
            lo.append(k[0])
            hi.append(k[1])
            msgs.append(J.encode_pnc([(5, 7)], [i], [0]))
        done, cut, rc = node.apply_committed(None, lo, hi, [1] * len(msgs), None, msgs)
        assert cut is None
        s = node.stats()
        kept = sum(1 for a, b in zip(lo, hi) if jg.shard_of(a, b, world) == 2)
        assert s["msgs_uploaded"] == kept < len(msgs)
        mine = {k: i for i, k in enumerate(own)}
        exp = np.zeros(len(own), np.int64)
        for a, b, i in zip(lo, hi, range(600)):
            if (a, b) in mine:
                exp[mine[(a, b)]] = max(exp[mine[(a, b)]], i)
        assert s["msgs_applied"] == sum(1 for a, b in zip(lo, hi) if (a, b) in mine)
        v, o = pnc.values(np.arange(len(own)))
        assert np.array_equal(v, exp)
    finally:
        node.close()
        pnc.close()


def test_tracker_add_contains_and_growth(ctx):
    """TryAdd / ContainsKey / Count of the device tracker, an identity added twice kept once, and the
    table rebuilt (tombstones dropped) as waves complete and new entries arrive."""
    tr = jg.Tracker(ctx)
    pnc = jg.PNCStore(ctx, 4, R, EB)
    node = jg.Node(pnc, None)
    try:
        tr.add([5, 6, 7], [50, 60, 70])
        tr.add([6], [99])  # TryAdd of a present identity: false, the first origin stays
        assert tr.size() == 3
        assert list(tr.contains([5, 6, 7, 8])) == [1, 1, 1, 0]
        u = (0xABC, 0xDEF)
        node.register([u[0]], [u[1]], [0], [0])
        live = {5: 50, 6: 60, 7: 70}
        seq = 100
        for w in range(6):
            new = list(range(seq, seq + 20000))
            seq += 20000
            tr.add(new, [s % 997 + 1 for s in new])
            live.update({s: s % 997 + 1 for s in new})
            take = [s for i, s in enumerate(list(live)) if i % 3 != 1]
            msgs = [J.encode_pnc([(1, 2)], [1], [0])] * len(take)
            done, cut, rc = node.apply_committed(tr, [u[0]] * len(take), [u[1]] * len(take), [1] * len(take), take, msgs)
            assert list(done) == [live.pop(s) for s in take]
            assert tr.size() == len(live)
        rest = list(live)
        assert tr.contains(rest).all() and not tr.contains(take).any()
    finally:
        node.close()
        pnc.close()
        tr.close()


def test_register_rejects_bad_keys(ctx):
    pnc = jg.PNCStore(ctx, 4, R, EB)
    node = jg.Node(pnc, None)
    try:
        node.register([1], [2], [0], [0])
        for lo, hi, t, i in ([0], [0], [0], [1]), ([1], [2], [0], [1]), ([3], [4], [0], [4]), ([3], [4], [1], [0]), ([3, 3], [4, 4], [0, 0], [1, 2]):
            with pytest.raises(jg.JanusError) as e:
                node.register(lo, hi, t, i)
            assert e.value.code == jg.JG_EINVAL
        node.register([3], [4], [0], [1])  # nothing of the rejected calls was registered
    finally:
        node.close()
        pnc.close()


@pytest.mark.parametrize("drop", ["dip", "collapse"])
def test_decreasing_offsets_reject_the_wave(ctx, monkeypatch, drop):
    """Contiguous payload offsets that decrease inside a later chunk (checked by each chunk's first pass)
    reject the whole wave with JG_EINVAL before anything of it is applied; the tracker claims the chunks
    already classified took are released, so the same wave with correct offsets then applies exactly as
    the oracle's loop does (completions included)."""
    monkeypatch.setenv("JANUS_WAVE_CHUNK", "50")
    monkeypatch.setenv("JANUS_HOST_PAR_MIN", "1")
    rng = np.random.default_rng(17)
    n_pnc, n_set, n = 60, 20, 400
    pnc, st, node, tr, m, uids = _setup(ctx, rng, n_pnc, n_set)
    try:
        pcl = J.Cluster(rng, n_pnc, R - 1, EB, stable=None)
        ocl = J.ORSetCluster(rng, n_set)
        wave = _wave(rng, m, uids, n_pnc, n_set, n, pcl, ocl, seq0=0, extras=False)
        tr.add(list(m.tracker), list(m.tracker.values()))
        lo, hi = [x[0][0] for x in wave], [x[0][1] for x in wave]
        types, seqs = [x[1] for x in wave], [x[2] for x in wave]
        data, off = jg.pack_wave([x[3] for x in wave])
        bad = np.array(off, np.uint64).copy()
        if drop == "dip":
            bad[301] = bad[300] - 1  # message 300 (a later 50-message chunk) ends before it starts
        else:  # every offset from message 301 on falls back by off[300]: off[n] is smaller than earlier chunks' ends,
            bad[301:] -= bad[300]  # which must be refused before those chunks are uploaded into buffers sized from it
        with pytest.raises(jg.JanusError) as e:
            node.apply_committed(tr, lo, hi, types, seqs, data=data, off=bad)
        assert e.value.code == jg.JG_EINVAL and "offsets decrease" in str(e.value)
        if drop == "dip":
            assert "at message 300" in str(e.value)
        P0, N0 = pnc.read_rows()
        assert np.array_equal(P0, m.P) and np.array_equal(N0, m.N)  # nothing applied
        exp_done, exp_cut = m.apply(wave)
        done, cut, rc = node.apply_committed(tr, lo, hi, types, seqs, data=data, off=off)
        assert rc == jg.JG_OK and cut is None and exp_cut is None
        assert list(done) == exp_done
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
        ga, gr = st.read()
        assert orc.same_orset(ga, gr, *m.orset)
        assert tr.size() == len(m.tracker)
    finally:
        for h in (node, tr, pnc, st):
            h.close()


def test_tracker_adds_across_empty_waves(ctx):
    """an empty wave flushes the pending tracker adds and returns; the next adds go into the other
    page-locked buffer, the wave after that flushes them and reuses the first one.  Every add must reach the
    device table intact (no buffer rewritten or freed while its upload is queued), in add order."""
    tr = jg.Tracker(ctx)
    pnc = jg.PNCStore(ctx, 4, R, EB)
    node = jg.Node(pnc, None)
    try:
        u = (0x1234, 0x5678)
        node.register([u[0]], [u[1]], [0], [0])
        origin = {}
        seq = 1
        for rnd in range(4):
            for _ in range(3):  # adds, then an empty wave (flushes them), twice over; the buffers alternate
                new = list(range(seq, seq + 5000))
                seq += 5000
                tr.add(new, [s % 991 + 1 for s in new])
                origin.update({s: s % 991 + 1 for s in new})
                done, cut, rc = node.apply_committed(tr, [], [], [], [], [])
                assert cut is None and rc == jg.JG_OK and len(done) == 0
            take = sorted(origin)[::2]
            msgs = [J.encode_pnc([(1, 2)], [1], [0])] * len(take)
            done, cut, rc = node.apply_committed(tr, [u[0]] * len(take), [u[1]] * len(take), [1] * len(take), take, msgs)
            assert cut is None and list(done) == [origin.pop(s) for s in take]
            assert tr.size() == len(origin)
    finally:
        node.close()
        pnc.close()
        tr.close()


def test_tracker_first_add_wins_within_a_batch(ctx):
    """ConcurrentDictionary.TryAdd (SafeCRDT.cs:55): an identity added twice before one flush keeps the
    origin of its first add, whichever device lane inserts it."""
    tr = jg.Tracker(ctx)
    pnc = jg.PNCStore(ctx, 4, R, EB)
    node = jg.Node(pnc, None)
    try:
        u = (0x99, 0x77)
        node.register([u[0]], [u[1]], [0], [0])
        ids = list(range(1000, 1000 + 4096))
        # each identity added 8 times in one batch (first origin = id % 13 + 1), interleaved
        for r in range(8):
            tr.add(ids, [i % 13 + 1 + 100 * r for i in ids])
        tr.add([ids[0]], [777])  # a later batch: TryAdd of a present identity keeps the first origin too
        msgs = [J.encode_pnc([(1, 2)], [1], [0])] * len(ids)
        done, cut, rc = node.apply_committed(tr, [u[0]] * len(ids), [u[1]] * len(ids), [1] * len(ids), ids, msgs)
        assert list(done) == [i % 13 + 1 for i in ids]
        assert tr.size() == 0
    finally:
        node.close()
        pnc.close()
        tr.close()


def test_orset_id_space_rejects_before_anything_commits(ctx):
    """A wave whose new element names could run a set past 2^32 - 2 ids is rejected (JG_ESTATE) by the check,
    before the PN-Counter commit: no PN-Counter row and no OR-Set record of the wave is applied, and the
    tracker claims are released (the OR-Set commit used to fail after the PN-Counter one)."""
    rng = np.random.default_rng(21)
    pnc, st, node, tr, m, uids = _setup(ctx, rng, 10, 2)
    try:
        pcl = J.Cluster(rng, 10, R - 1, EB, stable=None)
        st.names_sync(sets=[0], next_ids=[0xFFFFFFFD], cleared=[0])
        P0, N0 = pnc.read_rows()
        a0, r0 = st.read()
        tr.add([41], [9])
        wave = [(uids[0], 1, 41, pcl.message(0)), (uids[10], 1, 0, J.encode_orset([("n1", [(1, 2)]), ("n2", [(3, 4)])], []))]
        with pytest.raises(jg.JanusError) as e:
            node.apply_committed(tr, [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave], [x[2] for x in wave],
                                 [x[3] for x in wave])
        assert e.value.code == jg.JG_ESTATE
        P, N = pnc.read_rows()
        assert np.array_equal(P, P0) and np.array_equal(N, N0)
        a, r = st.read()
        assert orc.same_orset(a, r, a0, r0)
        # one new name still fits (id 2^32 - 3): the same PN-Counter message then completes its identity
        wave[1] = (uids[10], 1, 0, J.encode_orset([("n1", [(1, 2)])], []))
        done, cut, rc = node.apply_committed(tr, [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave],
                                             [x[2] for x in wave], [x[3] for x in wave])
        assert rc == jg.JG_OK and cut is None and list(done) == [9]
        assert st.wave_names() == [(0, 0xFFFFFFFD, b"n1")]
    finally:
        for h in (node, tr, pnc, st):
            h.close()


def test_orset_commit_failure_still_reports_completions():
    """the OR-Set commit's error flag is read with the wave's final read, after k_complete has taken
    the safe-update completions off the tracker.  A failing commit (forced by JANUS_TEST_ORSET_COMMIT_FAIL, an
    injector only the test build lib/libjanusgpu_test.so has: ADVICE r05) returns its error AFTER the completions:
    the caller gets every completed origin, in commit order, and the tracker holds exactly the entries not
    completed.  Runs in a child process that loads the test build (JANUS_GPU_LIB)."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    lib = root / "janus-crdt_amd" / "lib" / "libjanusgpu_test.so"
    assert lib.exists(), "the test build is made by __graft_entry__.build()"
    env = dict(os.environ, JANUS_GPU_LIB=str(lib), JANUS_TEST_ORSET_COMMIT_FAIL="1")
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import janus_gpu as jg, test_node_gpu as t\n"
            "ctx = jg.Context(0)\nt._commit_failure_scenario(ctx)\nctx.close()\nprint('SCENARIO OK')\n"
            % (str(root / "janus-crdt_amd"), str(root / "tests")))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=str(root / "tests"))
    assert out.returncode == 0 and "SCENARIO OK" in out.stdout, out.stdout[-2000:] + out.stderr[-3000:]


def _commit_failure_scenario(ctx):
    assert "libjanusgpu_test" in str(jg.LIB_PATH)
    rng = np.random.default_rng(29)
    pnc, st, node, tr, m, uids = _setup(ctx, rng, 60, 20)
    pcl = J.Cluster(rng, 60, R - 1, EB, stable=None)
    ocl = J.ORSetCluster(rng, 20)
    try:
        wave = _wave(rng, m, uids, 60, 20, 1500, pcl, ocl, seq0=0)
        tr.add(list(m.tracker), list(m.tracker.values()))
        exp_done, exp_cut = m.apply(wave)
        assert exp_cut is None and len(exp_done) > 100
        with pytest.raises(jg.JanusError) as ei:
            node.apply_committed(tr, [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave], [x[2] for x in wave],
                                 [x[3] for x in wave])
        assert ei.value.code == jg.JG_ESTATE
        assert list(ei.value.completed) == exp_done
        assert tr.size() == len(m.tracker)
        P, N = pnc.read_rows()  # the PN-Counter commit went through
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
    finally:
        for h in (node, tr, pnc, st):
            h.close()


@pytest.mark.parametrize("pinned,chunk,bad", [(False, None, False), (True, None, False), (True, 53, True), (False, 71, False)])
def test_streamed_wave_matches_one_call(ctx, monkeypatch, pinned, chunk, bad):
    """jg_apply_stream_begin / _append / _end (a wave handed over in parts): the same stores,
    completions, cut and tracker as the oracle's loop over the whole wave — parts of random sizes (empty ones too),
    from page-locked memory (uploaded in place, the device reading them after each append returns) or gathered,
    with small chunks inside parts, and a rejected state in some part."""
    if chunk:
        _run(ctx, 21, 90, 30, 3, 1500, chunk=chunk, monkeypatch=monkeypatch, bad=bad, pinned=pinned, stream=5)
    else:
        _run(ctx, 23, 150, 50, 3, 3000, bad=bad, pinned=pinned, stream=7)


def test_streamed_wave_rules(ctx):
    """A part past the begin's bounds rejects the wave (nothing applied, stream closed); append / end without an
    open stream and a second begin are refused; jg_apply_committed is refused while a stream is open."""
    import ctypes as C
    rng = np.random.default_rng(3)
    pnc, st, node, tr, m, uids = _setup(ctx, rng, 20, 5)
    pcl = J.Cluster(rng, 20, R - 1, EB, stable=None)
    lib = jg.load()
    try:
        wave = [(uids[k], 1, 0, pcl.message(k)) for k in rng.integers(0, 20, 50).tolist()]
        lo, hi = [x[0][0] for x in wave], [x[0][1] for x in wave]
        types, seqs, msgs = [x[1] for x in wave], [x[2] for x in wave], [x[3] for x in wave]
        with pytest.raises(jg.JanusError):  # 50 messages into a stream declared for 10
            node.apply_stream(tr, [(lo, hi, types, seqs, msgs)], n_max=10)
        P, N = pnc.read_rows()
        assert not P.any() and not N.any()  # nothing applied
        assert lib.jg_apply_stream_append(node._h, None) == jg.JG_EINVAL
        at, nd = jg._u64(), jg._u64()
        assert lib.jg_apply_stream_end(node._h, None, C.byref(nd), C.byref(at)) == jg.JG_EINVAL
        assert lib.jg_apply_stream_begin(node._h, None, 100, 1 << 20) == jg.JG_OK
        assert lib.jg_apply_stream_begin(node._h, None, 100, 1 << 20) == jg.JG_EINVAL
        with pytest.raises(jg.JanusError):
            node.apply_committed(tr, lo, hi, types, seqs, msgs)
        assert lib.jg_apply_stream_end(node._h, None, C.byref(nd), C.byref(at)) == jg.JG_OK  # an empty stream
        done, cut, rc = node.apply_stream(tr, [(lo[:20], hi[:20], types[:20], seqs[:20], msgs[:20]), (lo[20:], hi[20:], types[20:], seqs[20:], msgs[20:])])
        exp_done, exp_cut = m.apply(wave)
        assert rc == jg.JG_OK and cut is None and list(done) == exp_done
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
    finally:
        for h in (node, tr, pnc, st):
            h.close()


def _known_states(rng, n_pnc):
    """Per key three replica Guids and a state message listing all of them (the wave after it is fully known)."""
    reps = [J.random_guids(rng, 3) for _ in range(n_pnc)]
    return reps, lambda k, v: J.encode_pnc(reps[k], [v, v + 1, v + 2], [v // 2, 0, v // 3])


@pytest.mark.parametrize("how", ["block_unknown_uid", "orset_rejects_first"])
def test_cut_at_message_zero_applies_nothing(ctx, how):
    """a node wave cut at its first message applies nothing.  The chunks' fused pass A has
    already raised the counters of every PN-Counter state whose replicas the store knows; the prefix of length 0
    must take them back too (pnc_node_prefix used to return before its undo).  The cut comes from block mode's
    unknown uid at index 0 (KeyNotFoundException, ReplicationManager.cs:329) or from the OR-Set check rejecting
    message 0 (the apply Task faults there, SafeCRDTManager.cs:136-139)."""
    rng = np.random.default_rng(31)
    n_pnc = 40
    pnc, st, node, tr, m, uids = _setup(ctx, rng, n_pnc, 6)
    reps, state = _known_states(rng, n_pnc)
    try:
        warm = [(uids[k], 1, 0, state(k, 10 + k)) for k in range(n_pnc)]
        m.apply(warm)
        done, cut, rc = node.apply_committed(None, [x[0][0] for x in warm], [x[0][1] for x in warm], [1] * n_pnc, None, [x[3] for x in warm])
        assert rc == jg.JG_OK and cut is None
        wave = [(uids[k % n_pnc], 1, 0, state(k % n_pnc, 1000 + 7 * k)) for k in range(400)]
        if how == "block_unknown_uid":
            wave[0] = ((0x5151, 0x7373), 1, 0, b'{"pVector":{},"nVector":{}}')
        else:
            wave[0] = (uids[n_pnc], 1, 0, b'{"addSet":{}}')  # an ORSetMsg Decode rejects (missing members)
        exp_done, exp_cut = m.apply(wave, block=how == "block_unknown_uid")
        assert exp_cut == 0
        lo, hi, types = [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave]
        if how == "block_unknown_uid":
            cut, rc = node.apply_block(lo, hi, types, [x[3] for x in wave])
        else:
            done, cut, rc = node.apply_committed(tr, lo, hi, types, [0] * len(wave), [x[3] for x in wave])
        assert cut == 0 and rc != jg.JG_OK
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)  # the fused raises of messages 1..399 undone
        assert node.stats()["msgs_applied"] == 0
    finally:
        for h in (node, tr, pnc, st):
            h.close()


def test_streamed_wave_holds_its_stores(ctx):
    """between jg_apply_stream_begin and _end (unlocked calls) the stores' wave scratch, fused pass
    A's undo records and the OR-Set wave tables belong to the open wave.  Every call that writes the stores, a
    jg_pnc_wave_* / jg_orset_wave_* wave, another node's wave over a shared store and the tracker's destroy are
    refused (JG_EINVAL) and change nothing; reads are allowed.  The wave then ends exactly as the oracle's loop
    says and the stores are free again.  A node destroyed with a stream open aborts it: nothing of it stays."""
    import ctypes as C
    rng = np.random.default_rng(37)
    n_pnc = 30
    pnc, st, node, tr, m, uids = _setup(ctx, rng, n_pnc, 4)
    reps, state = _known_states(rng, n_pnc)
    lib = jg.load()
    other = None
    try:
        warm = [(uids[k], 1, 0, state(k, 5 + k)) for k in range(n_pnc)]
        m.apply(warm)
        node.apply_committed(None, [x[0][0] for x in warm], [x[0][1] for x in warm], [1] * n_pnc, None, [x[3] for x in warm])
        wave = [(uids[k % n_pnc], 1, 0, state(k % n_pnc, 500 + 3 * k)) for k in range(300)]
        lo, hi, types, msgs = [x[0][0] for x in wave], [x[0][1] for x in wave], [x[1] for x in wave], [x[3] for x in wave]
        assert lib.jg_apply_stream_begin(node._h, tr._h, len(wave), sum(map(len, msgs))) == jg.JG_OK
        c, keep = node._commit(lo[:150], hi[:150], types[:150], None, msgs[:150])
        assert lib.jg_apply_stream_append(node._h, C.byref(c)) == jg.JG_OK  # pass A ran (fused) on these 150
        one = np.zeros((1, R), np.int32)
        refused = [
            lambda: pnc.merge_rows(one + 2**30, one + 2**30, [0]),
            lambda: pnc.write_rows(one, one, [0]),
            lambda: pnc.apply_ops([0], [0], [5], [0]),
            lambda: pnc.wave_begin(10, 1000),
            lambda: pnc.merge_json([0], [state(0, 9999)]),
            lambda: st.merge(jg.records(n=0), jg.records(n=0)),
            lambda: st.merge_json([0], [J.encode_orset([("e", [(1, 2)])], [])]),
        ]
        for f in refused:
            with pytest.raises(jg.JanusError) as e:
                f()
            assert e.value.code == jg.JG_EINVAL and "node wave" in str(e.value)
        assert lib.jg_tracker_destroy(tr._h) == jg.JG_EINVAL
        other = jg.Node(pnc, None)
        other.register([uids[0][0]], [uids[0][1]], [0], [0])
        with pytest.raises(jg.JanusError) as e:
            other.apply_committed(None, [uids[0][0]], [uids[0][1]], [1], None, [state(0, 12345)])
        assert e.value.code == jg.JG_EINVAL
        pnc.values()  # reads are allowed
        c2, keep2 = node._commit(lo[150:], hi[150:], types[150:], None, msgs[150:])
        assert lib.jg_apply_stream_append(node._h, C.byref(c2)) == jg.JG_OK
        at, nd = jg._u64(), jg._u64()
        done = np.zeros(len(wave), np.uint64)
        assert lib.jg_apply_stream_end(node._h, jg._ptr(done), C.byref(nd), C.byref(at)) == jg.JG_OK
        m.apply(wave)
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
        pnc.merge_rows(one, one, [0])  # free again (a no-op merge)
        # a stream left open when its node is destroyed: aborted, the fused raises taken back, the stores let go
        assert lib.jg_apply_stream_begin(node._h, None, 100, 1 << 20) == jg.JG_OK
        c3, keep3 = node._commit(lo[:100], hi[:100], types[:100], None, [state(k % n_pnc, 10**6 + k) for k in range(100)])
        assert lib.jg_apply_stream_append(node._h, C.byref(c3)) == jg.JG_OK
        node.close()
        P, N = pnc.read_rows()
        assert np.array_equal(P, m.P) and np.array_equal(N, m.N)
        pnc.merge_rows(one, one, [0])
        other.apply_committed(None, [uids[0][0]], [uids[0][1]], [1], None, [J.encode_pnc(reps[0], [1, 1, 1], [0, 0, 0])])
    finally:
        for h in (other, node, tr, pnc, st):
            if h is not None:
                h.close()
