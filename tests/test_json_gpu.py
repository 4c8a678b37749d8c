"""GPU parity of the wire-format apply path (janus-crdt_amd/csrc/json.hip, SURVEY.md §8f F1 + §8a A2/A13)
against the oracle's Decode + Merge loop (oracle/json.hpp, oracle/capi.cpp orc_pnc_apply_json), through
the C ABI: the decode contract, replica interning in commit order, all-or-nothing errors, row capacity,
and the device-resident wave.  Bit-exact on values, replica Guids and column order."""
import hashlib

import numpy as np
import pytest

import janus_gpu as jg
import oracle_ref as orc
from jsongen import CONTRACT, G1, G2, Cluster, encode_pnc, guid_d, random_guids

pytestmark = pytest.mark.gpu


def _guid_arr(gs):
    a = np.empty(len(gs), orc.GUID_DTYPE)
    a["lo"] = [g[0] for g in gs]
    a["hi"] = [g[1] for g in gs]
    return a


class Pair:
    """A GPU store and the oracle's dense image of the same state."""

    def __init__(self, ctx, n_keys, R, eb, stable):
        self.s = jg.PNCStore(ctx, n_keys, R, eb)
        ga = _guid_arr(stable)
        cols0 = self.s.intern(np.arange(n_keys, dtype=np.uint32), ga["lo"], ga["hi"])
        assert (cols0 == 0).all()
        dt = np.int32 if eb == 4 else np.int64
        self.P = np.zeros((n_keys, R), dt)
        self.N = np.zeros((n_keys, R), dt)
        self.cols = np.zeros((n_keys, R), orc.GUID_DTYPE)
        self.cols[:, 0] = ga
        self.ncols = np.ones(n_keys, np.uint32)
        self.eb, self.n_keys = eb, n_keys

    def oracle(self, keys, msgs):
        self.P, self.N, self.cols, self.ncols, bad, rc = orc.pnc_apply_json(self.P, self.N, self.cols, self.ncols, keys, msgs, self.eb)
        return bad, rc

    def check(self):
        P, N = self.s.read_rows()
        g, n = self.s.columns(np.arange(self.n_keys, dtype=np.uint32))
        assert np.array_equal(n, self.ncols), "column counts differ"
        for k in range(self.n_keys):
            c = int(n[k])
            assert np.array_equal(g[k, :c], self.cols[k, :c]), f"replica order differs at key {k}"
        assert np.array_equal(P, self.P) and np.array_equal(N, self.N), "values differ"

    def close(self):
        self.s.close()


GROUPS = ["1", "8", "16", "32", "64"]  # JANUS_JSON_GROUP: lanes per message (1 = the serial parser)


@pytest.mark.parametrize("group", GROUPS)
@pytest.mark.parametrize("eb", [4, 8])
def test_decode_contract_on_device(ctx, eb, group, monkeypatch):
    monkeypatch.setenv("JANUS_JSON_GROUP", group)
    for i, (payload, ok4, ok8) in enumerate(CONTRACT):
        ok = ok4 if eb == 4 else ok8
        pr = Pair(ctx, 2, 4, eb, [(7, 7), (8, 8)])
        bad, rc = pr.oracle(np.array([1], np.uint32), [payload])
        assert (bad is None) == ok, f"oracle disagrees with the contract on case {i}"
        if ok:
            pr.s.merge_json([1], [payload])
        else:
            with pytest.raises(jg.JanusError) as e:
                pr.s.merge_json([1], [payload])
            assert e.value.code == jg.JG_EINVAL and e.value.bad_msg == 0, f"case {i}: {e.value}"
        try:
            pr.check()
        except AssertionError as e:
            raise AssertionError(f"case {i} {payload[:160]!r}: {e}") from None
        pr.close()


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("ws", [0.0, 0.3])
@pytest.mark.parametrize("group", ["1", "8", "16"])
@pytest.mark.parametrize("eb,R,pool", [(4, 8, 6), (8, 8, 6), (4, 64, 40), (8, 200, 150)])
def test_random_waves_match_oracle(ctx, eb, R, pool, group, ws, fuse, monkeypatch):
    """ws: the fraction of states written with a space after every ':' (valid, not the compact form), so
    one row's walk mixes group-parsed and serially parsed messages: pass C hands a walk to the serial
    resume kernel, which also resolves the records of the compact messages after it.  fuse: pass A applies
    the messages whose replicas are all known itself (JANUS_JSON_FUSE, default on) or leaves them to pass B."""
    monkeypatch.setenv("JANUS_JSON_GROUP", group)
    monkeypatch.setenv("JANUS_JSON_FUSE", fuse)
    rng = np.random.default_rng(R * 10 + eb + int(ws * 100))
    n_keys = 40
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, R, eb, stable)
    cl = Cluster(rng, n_keys, pool, eb, stable)
    for wave in range(5):
        n = int(rng.integers(1, 1500))
        keys = rng.integers(0, n_keys, n).astype(np.uint32)
        msgs = [cl.message(int(k), grow=0.05 if R > 8 else 0.3) for k in keys]
        msgs = [m.replace(b'":', b'": ') if rng.random() < ws else m for m in msgs]
        bad, rc = pr.oracle(keys, msgs)
        assert bad is None and rc == 0
        pr.s.merge_json(keys, msgs)
        pr.check()
    pr.close()


def _stj_variant(rng, m: bytes, eb) -> bytes:
    """The same decoded state written the ways System.Text.Json also accepts (oracle/json.hpp, round 6): an unknown
    member before it, an earlier pVector occurrence the real one replaces, a key repeated in its vector with the
    LARGEST value first (max-merging every occurrence would differ from the last-value rule), a key repeated after
    itself, an escaped key."""
    import re
    s = m.decode()
    k = int(rng.integers(0, 5))
    hi = 2**31 - 1 if eb == 4 else 2**63 - 1
    if k == 0:
        return ('{"zz":{"a":[1,-2.5e3,{"b":null}],"c":"\\u00e9"},' + s[1:]).encode()
    if k == 1:
        return ('{"pVector":{"' + guid_d(*G1) + '":' + str(hi) + '},' + s[1:]).encode()
    ents = list(re.finditer(r'"([0-9a-fA-F-]{36})":(-?[0-9]+)', s))
    if not ents:
        return m
    e = ents[int(rng.integers(0, len(ents)))]
    g, v = e.group(1), e.group(2)
    if k == 2:  # an earlier occurrence holding the largest value
        return (s[:e.start()] + f'"{g}":{hi},' + s[e.start():]).encode()
    if k == 3:  # the same key again right after, with a smaller value: it wins
        return (s[:e.end()] + f',"{g}":{max(0, int(v) // 2)}' + s[e.end():]).encode()
    return (s[:e.start()] + '"\\u00' + format(ord(g[0]), "02x") + g[1:] + '":' + v + s[e.end():]).encode()


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("group", ["1", "8"])
@pytest.mark.parametrize("eb", [4, 8])
def test_stj_forms_match_oracle(ctx, eb, group, fuse, monkeypatch):
    """states System.Text.Json decodes beyond the compact form — unknown members, a repeated
    vector, a key repeated inside one vector (last value, first place), escaped keys — merge on the device exactly
    as the oracle's Decode + Merge loop merges them, mixed into waves of compact states: the fast path hands them to
    the serial parser (a repeat among known replicas) or voids the earlier entries in pass C (a repeat among new
    ones).  Parity unpinned by reference fixtures (none hold such a state)."""
    monkeypatch.setenv("JANUS_JSON_GROUP", group)
    monkeypatch.setenv("JANUS_JSON_FUSE", fuse)
    rng = np.random.default_rng(eb * 7 + int(group) + int(fuse))
    n_keys = 30
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, 8, eb, stable)
    cl = Cluster(rng, n_keys, 6, eb, stable)
    try:
        for wave in range(5):
            n = int(rng.integers(50, 1200))
            keys = rng.integers(0, n_keys, n).astype(np.uint32)
            msgs = [cl.message(int(k)) for k in keys]
            msgs = [_stj_variant(rng, m, eb) if rng.random() < 0.3 else m for m in msgs]
            bad, rc = pr.oracle(keys, msgs)
            assert bad is None and rc == 0
            pr.s.merge_json(keys, msgs)
            pr.check()
    finally:
        pr.close()


@pytest.mark.parametrize("group", ["8", "16"])
@pytest.mark.parametrize("eb", [4, 8])
def test_columns_past_the_repeat_mask(ctx, eb, group, monkeypatch):
    """Compact states naming columns >= 64 (kMaskCols): the group parse hands them to the serial parser,
    which applies them; a Guid repeated in one vector past column 64 takes its LAST value (System.Text.Json's
    Dictionary indexer, oracle/json.hpp) — the first occurrence carries a value larger than any cell, which a
    max over every occurrence would keep."""
    monkeypatch.setenv("JANUS_JSON_GROUP", group)
    rng = np.random.default_rng(640 + eb)
    stable = random_guids(rng, 2)
    reps = random_guids(rng, 90)
    pr = Pair(ctx, 2, 128, eb, stable)
    # wave 1: 90 new replicas on key 1, 10 per compact state (appended in commit order)
    keys = np.ones(9, np.uint32)
    msgs = [encode_pnc(reps[10 * i:10 * i + 10], [int(v) for v in rng.integers(0, 1000, 10)], [None] * 10) for i in range(9)]
    assert pr.oracle(keys, msgs) == (None, 0)
    pr.s.merge_json(keys, msgs)
    pr.check()
    # wave 2: states mixing columns below and past 64, in both vectors
    msgs = []
    for _ in range(200):
        pick = sorted(int(x) for x in rng.choice(90, 12, replace=False))
        g = [reps[i] for i in pick]
        pv = [int(v) if rng.random() < 0.7 else None for v in rng.integers(0, 5000, 12)]
        nv = [int(v) if rng.random() < 0.5 else None for v in rng.integers(0, 5000, 12)]
        msgs.append(encode_pnc(g, pv, nv))
    keys = np.ones(len(msgs), np.uint32)
    assert pr.oracle(keys, msgs) == (None, 0)
    pr.s.merge_json(keys, msgs)
    pr.check()
    # wave 3: a repeated Guid at a column past 64 (and one below it): the last value, at the first place
    dup = encode_pnc([reps[80], reps[3], reps[80], reps[3]], [9000, 9001, 4999, 17], [None] * 4)
    keys = np.ones(3, np.uint32)
    wave = [msgs[0], dup, msgs[1]]
    assert pr.oracle(keys, wave) == (None, 0)
    pr.s.merge_json(keys, wave)
    pr.check()
    pr.close()


def _mutants(rng, cl, keys, n):
    """Near-compact payloads: one byte replaced, deleted or inserted, vectors swapped, a space added."""
    alpha = b'"{},:-0123456789abcdefABCDEF xnpV\\'
    out = []
    for _ in range(n):
        k = int(keys[int(rng.integers(0, len(keys)))])
        m = bytearray(cl.message(k))
        op = int(rng.integers(0, 5))
        i = int(rng.integers(0, len(m)))
        if op == 0:
            m[i] = alpha[int(rng.integers(0, len(alpha)))]
        elif op == 1:
            del m[i]
        elif op == 2:
            m.insert(i, alpha[int(rng.integers(0, len(alpha)))])
        elif op == 3:
            s_ = bytes(m)
            j = s_.index(b',"nVector"')
            m = bytearray(b'{' + s_[j + 1:-1] + b',' + s_[1:j] + b'}')
        else:
            m.insert(i, ord(" "))
        out.append((k, bytes(m)))
    return out


@pytest.mark.parametrize("group", GROUPS[1:])
@pytest.mark.parametrize("eb", [4, 8])
def test_group_parse_near_compact(ctx, eb, group, monkeypatch):
    """The group parse (json_wave.hpp) proves a payload compact or hands it to the serial parser:
    single-byte mutations of reference-shaped states (every token position), vector swaps and stray
    whitespace are accepted or rejected exactly as the oracle's Decode does, and a store fed through the
    group parse ends bit-identical to one fed through the serial parser (JANUS_JSON_GROUP=1).  Mutated
    Guids may sit in one vector only, a state no reference node produces (the shared column order of
    DESIGN.md §2 then differs from the oracle's P order), so the state check is serial-vs-group."""
    rng = np.random.default_rng(int(group) * 7 + eb)
    n_keys, R = 6, 64
    stable = random_guids(rng, n_keys)
    ga = _guid_arr(stable)
    stores = {}
    for G in (group, "1"):
        stores[G] = jg.PNCStore(ctx, n_keys, R, eb)
        stores[G].intern(np.arange(n_keys, dtype=np.uint32), ga["lo"], ga["hi"])
    cl = Cluster(rng, n_keys, 6, eb, stable)
    keys = np.arange(n_keys, dtype=np.uint32)
    dt = np.int32 if eb == 4 else np.int64
    z = np.zeros((n_keys, R), dt)
    cols0 = np.zeros((n_keys, R), orc.GUID_DTYPE)
    n_bad = 0
    for k, msg in _mutants(rng, cl, keys, 160):
        wave = (np.array([k, k], np.uint32), [cl.message(k), msg])
        *_, bad, rc = orc.pnc_apply_json(z, z, cols0, np.zeros(n_keys, np.uint32), np.array([k], np.uint32), [msg], eb)
        n_bad += bad is not None
        for G, st in stores.items():
            monkeypatch.setenv("JANUS_JSON_GROUP", G)
            if bad is None:
                st.merge_json(*wave)
            else:
                with pytest.raises(jg.JanusError) as e:
                    st.merge_json(*wave)
                assert e.value.code == jg.JG_EINVAL and e.value.bad_msg == 1, (G, msg)
    a, b = stores[group], stores["1"]
    for x, y in zip(a.read_rows(), b.read_rows()):
        assert np.array_equal(x, y)
    ga_, na = a.columns(keys)
    gb_, nb = b.columns(keys)
    assert np.array_equal(na, nb)
    for k in range(n_keys):
        assert np.array_equal(ga_[k, : na[k]], gb_[k, : nb[k]]), f"replica order differs at key {k}"
    assert 20 < n_bad < 160  # both outcomes exercised
    a.close()
    b.close()


def test_wild_values_and_vector_orders(ctx):
    """Negative and extreme values, pVector/nVector in different orders, replicas only in one vector."""
    rng = np.random.default_rng(11)
    n_keys, R = 8, 16
    stable = random_guids(rng, n_keys)
    pool = [random_guids(rng, 10) for _ in range(n_keys)]
    pr = Pair(ctx, n_keys, R, 4, stable)
    keys, msgs = [], []
    for _ in range(400):
        k = int(rng.integers(0, n_keys))
        gs = [pool[k][i] for i in rng.permutation(10)[: int(rng.integers(0, 6))]]
        vals = rng.integers(-2**31, 2**31, len(gs))
        pv = [int(v) if rng.random() < 0.8 else None for v in vals]
        nv = [int(v) ^ 0x55 if rng.random() < 0.5 else None for v in vals]
        p = ",".join(f'"{jg_guid(g)}":{v}' for g, v in zip(gs, pv) if v is not None)
        order = list(zip(gs, nv))[::-1]
        q = ",".join(f'"{jg_guid(g)}":{v}' for g, v in order if v is not None)
        msgs.append(('{"nVector":{' + q + '},"pVector":{' + p + "}}").encode())
        keys.append(k)
    keys = np.array(keys, np.uint32)
    bad, rc = pr.oracle(keys, msgs)
    assert bad is None and rc == 0
    pr.s.merge_json(keys, msgs)
    # values per replica Guid must agree; the column order can differ only where a message lists its
    # vectors' replicas in different orders (never produced by the reference)
    P, N = pr.s.read_rows()
    g, n = pr.s.columns(np.arange(n_keys, dtype=np.uint32))
    for k in range(n_keys):
        got = {(int(x["lo"]), int(x["hi"])): (P[k, c], N[k, c]) for c, x in enumerate(g[k, : n[k]])}
        exp = {(int(x["lo"]), int(x["hi"])): (pr.P[k, c], pr.N[k, c]) for c, x in enumerate(pr.cols[k, : pr.ncols[k]])}
        # the oracle's export lists P's keys; replicas seen only in nVector exist in the GPU table with P = 0
        for key, (p, q) in got.items():
            if key in exp:
                assert (p, q) == exp[key], f"key {k}"
            else:
                assert p == 0
    pr.close()


def jg_guid(g):
    from jsongen import guid_d
    return guid_d(*g)


def test_bad_message_is_all_or_nothing_then_prefix(ctx):
    rng = np.random.default_rng(5)
    n_keys = 30
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, 8, 4, stable)
    cl = Cluster(rng, n_keys, 6, 4, stable)
    keys = rng.integers(0, n_keys, 1000).astype(np.uint32)
    msgs = [cl.message(int(k)) for k in keys]
    msgs[700] = msgs[700].replace(b'"nVector"', b'"mVector"')
    msgs[901] = b"{"
    with pytest.raises(jg.JanusError) as e:
        pr.s.merge_json(keys, msgs)
    assert e.value.code == jg.JG_EINVAL and e.value.bad_msg == 700
    pr.check()  # nothing applied (columns included)
    bad, rc = pr.oracle(keys, msgs)  # the reference's loop: messages before the throwing one applied
    assert bad == 700
    pr.s.merge_json(keys[:700], msgs[:700])  # the host re-submits the prefix
    pr.check()
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_fused_apply_undone_on_failure(ctx, eb):
    """The fused pass A applies every message whose replicas are all known before the wave is judged; a wave
    that then fails (a bad message late in it, a streamed wave aborted after its chunks) must leave the store as
    it was: the undo records take every raised cell back (k_undo_applied).  Waves of growing states over known
    replicas, so nearly every entry raises its cell, several messages per key."""
    rng = np.random.default_rng(70 + eb)
    n_keys = 200
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, 8, eb, stable)
    cl = Cluster(rng, n_keys, 5, eb, stable)
    keys = rng.integers(0, n_keys, 3000).astype(np.uint32)
    msgs = [cl.message(int(k), grow=0.3) for k in keys]
    assert pr.oracle(keys, msgs) == (None, 0)
    pr.s.merge_json(keys, msgs)  # every replica known from here on
    pr.check()
    keys = rng.integers(0, n_keys, 3000).astype(np.uint32)
    msgs = [cl.message(int(k), grow=0.0) for k in keys]  # larger values, the same replicas
    bad_msgs = list(msgs)
    bad_msgs[2990] = b'{"pVector":{},"nVector":{}'
    with pytest.raises(jg.JanusError) as e:
        pr.s.merge_json(keys, bad_msgs)
    assert e.value.code == jg.JG_EINVAL and e.value.bad_msg == 2990
    pr.check()  # every raise undone
    # the same as a device-resident wave, and as a streamed wave that is aborted after its appends
    w = jg.Wave(ctx, 3000, 4 << 20)
    w.upload(keys, bad_msgs)
    with pytest.raises(jg.JanusError):
        pr.s.merge_wave(w)
    pr.check()
    w.close()
    pr.s.wave_begin(3000, 4 << 20)
    for c in range(0, 3000, 1000):
        pr.s.wave_append(keys[c:c + 1000], msgs[c:c + 1000])
    pr.s.wave_abort()
    pr.check()
    assert pr.oracle(keys, msgs) == (None, 0)
    pr.s.merge_json(keys, msgs)
    pr.check()
    pr.close()


def test_row_capacity_rolls_back(ctx):
    rng = np.random.default_rng(6)
    stable = random_guids(rng, 3)
    pr = Pair(ctx, 3, 3, 4, stable)
    gs = random_guids(rng, 4)
    msgs = [encode_pnc(gs[:1], [1], [0]), encode_pnc(gs[:2], [2, 2], [0, 0]), encode_pnc([gs[0]], [3], [0]),
            encode_pnc(gs[:3], [1, 1, 1], [0, 0, 0])]
    keys = np.array([2, 1, 1, 2], np.uint32)  # key 2 would need 1 + 3 = 4 columns
    with pytest.raises(jg.JanusError) as e:
        pr.s.merge_json(keys, msgs)
    assert e.value.code == jg.JG_ESTATE and e.value.bad_msg == 3
    pr.check()  # key 1's new columns rolled back too
    bad, rc = pr.oracle(keys[:3], msgs[:3])
    pr.s.merge_json(keys[:3], msgs[:3])
    pr.check()
    pr.close()


@pytest.mark.parametrize("group", ["1", "8"])
def test_rolled_back_slots_never_match(ctx, group, monkeypatch):
    """Pass A finds a row's columns as its leading non-zero slots (it reads no column count), so a roll-back
    must zero the slots it uncounts: a failed wave appended gs[0], gs[1] to key 1 and was rolled back; the
    next wave names gs[1] alone, which must become key 1's column 1 (the oracle's order), not match the
    stale slot 2 the failed walk wrote.  Then steady waves over the new columns (the fused path)."""
    monkeypatch.setenv("JANUS_JSON_GROUP", group)
    rng = np.random.default_rng(61)
    stable = random_guids(rng, 3)
    pr = Pair(ctx, 3, 3, 4, stable)
    gs = random_guids(rng, 4)
    msgs = [encode_pnc(gs[:2], [2, 2], [0, 0]), encode_pnc(gs[:3], [1, 1, 1], [0, 0, 0])]
    keys = np.array([1, 2], np.uint32)  # key 2 would need 1 + 3 = 4 columns: the wave fails in pass C
    with pytest.raises(jg.JanusError):
        pr.s.merge_json(keys, msgs)
    pr.check()
    for wave in ([encode_pnc([gs[1]], [5], [1])], [encode_pnc([gs[1], gs[2]], [6, 7], [1, 2])],
                 [encode_pnc([stable[1], gs[1], gs[2]], [1, 9, 9], [0, 3, 3])]):
        keys = np.array([1], np.uint32)
        assert pr.oracle(keys, wave) == (None, 0)
        pr.s.merge_json(keys, wave)
        pr.check()
    pr.close()


def test_all_zero_guid_replica(ctx):
    """A replica whose Guid is all-zero (Guid.Empty) is a column like any other; pass A cannot tell it from an
    unused slot and leaves its messages to the deferred path, whose result must equal the oracle's."""
    rng = np.random.default_rng(62)
    stable = random_guids(rng, 4)
    pr = Pair(ctx, 4, 4, 8, stable)
    zero = (0, 0)
    g1 = random_guids(rng, 1)[0]
    for k, wave in enumerate([[encode_pnc([zero, g1], [3, 4], [0, 1])], [encode_pnc([g1, zero], [5, 2], [1, 7])],
                              [encode_pnc([stable[2], zero, g1], [1, 8, 8], [0, 0, 9])], [encode_pnc([zero], [9], [9])]]):
        keys = np.array([2], np.uint32)
        assert pr.oracle(keys, wave) == (None, 0)
        pr.s.merge_json(keys, wave)
        pr.check()
    pr.close()


def test_intern_order_repeats_and_capacity(ctx):
    s = jg.PNCStore(ctx, 4, 3, 8)
    keys = np.array([1, 0, 1, 1, 0, 1], np.uint32)
    lo = np.array([10, 20, 11, 10, 21, 12], np.uint64)
    cols = s.intern(keys, lo, lo * 3)
    assert cols.tolist() == [0, 0, 1, 0, 1, 2]
    g, n = s.columns(np.array([0, 1, 2], np.uint32))
    assert n.tolist() == [2, 3, 0]
    assert g[1, :3]["lo"].tolist() == [10, 11, 12] and g[0, :2]["lo"].tolist() == [20, 21]
    with pytest.raises(jg.JanusError) as e:
        s.intern(np.array([2, 1], np.uint32), np.array([5, 99], np.uint64), np.array([5, 99], np.uint64))
    assert e.value.code == jg.JG_ESTATE
    g2, n2 = s.columns(np.array([0, 1, 2], np.uint32))
    assert n2.tolist() == [2, 3, 0]  # all or nothing: key 2's registration was rolled back too
    s.close()


def test_device_resident_wave_equals_host_call(ctx):
    rng = np.random.default_rng(8)
    n_keys = 64
    stable = random_guids(rng, n_keys)
    a = Pair(ctx, n_keys, 8, 8, stable)
    b = Pair(ctx, n_keys, 8, 8, stable)
    cl = Cluster(rng, n_keys, 6, 8, stable)
    w = jg.Wave(ctx, 5000, 5_000_000)
    for _ in range(3):
        keys = rng.integers(0, n_keys, 3000).astype(np.uint32)
        msgs = [cl.message(int(k)) for k in keys]
        a.oracle(keys, msgs)
        a.s.merge_json(keys, msgs)
        w.upload(keys, msgs)
        b.s.merge_wave(w)
        b.s.merge_wave(w)  # idempotent: the same wave twice changes nothing
        b.P, b.N, b.cols, b.ncols = a.P, a.N, a.cols, a.ncols
        a.check()
        b.check()
    w.close()
    a.close()
    b.close()


def test_c5_shaped_wave(ctx):
    """Banking-shaped wave (4 nodes, replicas = stable + one per node): 100k messages over 20k accounts,
    checked against the oracle on every account."""
    rng = np.random.default_rng(9)
    n_keys, nodes = 20_000, 4
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, nodes + 1, 4, stable)
    reps = [random_guids(rng, nodes) for _ in range(n_keys)]
    P = np.zeros((n_keys, nodes), np.int64)
    keys = rng.integers(0, n_keys, 100_000).astype(np.uint32)
    msgs = []
    for k in keys:
        n = int(rng.integers(0, nodes))
        P[k, n] += int(rng.integers(1, 1000))
        msgs.append(encode_pnc(reps[k], P[k].tolist(), [0] * nodes))
    bad, rc = pr.oracle(keys, msgs)
    assert bad is None and rc == 0
    pr.s.merge_json(keys, msgs)
    pr.check()
    v, o = pr.s.values()
    # every message carries its node's full row, and rows only grow: Get = the latest row sums
    assert (o == 0).all() and np.array_equal(v, np.where(np.isin(np.arange(n_keys), keys), P.sum(axis=1), 0))
    pr.close()


def test_streamed_wave_chunks_equal_one_call(ctx):
    """jg_pnc_wave_begin/append/commit over uneven chunks (capacity hint exceeded, so the wave buffers
    and the deferred list grow mid-wave) = one jg_pnc_merge_json of the concatenation."""
    rng = np.random.default_rng(12)
    n_keys = 300
    stable = random_guids(rng, n_keys)
    a = Pair(ctx, n_keys, 8, 4, stable)
    b = Pair(ctx, n_keys, 8, 4, stable)
    cl = Cluster(rng, n_keys, 6, 4, stable)
    for wave in range(3):
        keys = rng.integers(0, n_keys, 5000).astype(np.uint32)
        msgs = [cl.message(int(k)) for k in keys]
        a.oracle(keys, msgs)
        a.s.merge_json(keys, msgs)
        b.s.wave_begin(100, 10_000)  # deliberately short hints
        cuts = sorted(set([0, 5000] + rng.integers(0, 5000, 6).tolist()))
        for c0, c1 in zip(cuts, cuts[1:]):
            b.s.wave_append(keys[c0:c1], msgs[c0:c1])
        b.s.wave_append(np.zeros(0, np.uint32), [])
        b.s.wave_commit()
        b.P, b.N, b.cols, b.ncols = a.P, a.N, a.cols, a.ncols
        a.check()
        b.check()
    a.close()
    b.close()


def test_streamed_wave_error_and_abort(ctx):
    rng = np.random.default_rng(13)
    n_keys = 50
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, 8, 8, stable)
    cl = Cluster(rng, n_keys, 6, 8, stable)
    keys = rng.integers(0, n_keys, 900).astype(np.uint32)
    msgs = [cl.message(int(k)) for k in keys]
    msgs[650] = b'{"pVector":{},"nVector":{}'
    pr.s.wave_begin(900, 1 << 20)
    for c in range(0, 900, 300):
        pr.s.wave_append(keys[c:c + 300], msgs[c:c + 300])
    with pytest.raises(jg.JanusError) as e:
        pr.s.wave_commit()
    assert e.value.code == jg.JG_EINVAL and e.value.bad_msg == 650  # index over the whole wave
    pr.check()  # nothing applied
    pr.s.wave_begin(900, 1 << 20)
    pr.s.wave_append(keys[:300], msgs[:300])
    pr.s.wave_abort()
    pr.check()  # abort applies nothing
    with pytest.raises(jg.JanusError):
        pr.s.wave_commit()  # no open wave
    pr.oracle(keys[:650], msgs[:650])
    pr.s.merge_json(keys[:650], msgs[:650])
    pr.check()
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_encode_matches_oracle_encoder(ctx, eb):
    """GetLastSynchronizedUpdate().Encode() on the device (jg_pnc_encode_json) = the oracle's
    System.Text.Json restatement over the same dictionaries, byte for byte; and re-applying the encoded
    states is idempotent."""
    rng = np.random.default_rng(20 + eb)
    n_keys, R = 60, 16
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, R, eb, stable)
    cl = Cluster(rng, n_keys, 12, eb, stable)
    keys = rng.integers(0, n_keys, 3000).astype(np.uint32)
    msgs = [cl.message(int(k)) for k in keys]
    # extreme values through the wire too
    lim = 2**31 if eb == 4 else 2**63
    msgs.append(encode_pnc([G1, G2], [lim - 1, -lim], [-1, 0]))
    keys = np.append(keys, np.uint32(3))
    pr.oracle(keys, msgs)
    pr.s.merge_json(keys, msgs)
    q = rng.permutation(n_keys).astype(np.uint32)
    got = pr.s.encode_json(q)
    for k, b in zip(q, got):
        c = int(pr.ncols[k])
        exp = orc.json_encode_pnc(pr.cols[k, :c]["lo"], pr.cols[k, :c]["hi"], pr.P[k, :c], pr.N[k, :c], eb)
        assert b == exp, f"key {k}"
    pr.s.merge_json(q, got)  # a state merged into itself changes nothing
    pr.check()
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_encode_before_matches_oracle_encoder(ctx, eb):
    """jg_pnc_encode_json_before: each row as it stood before its last dp / dn of own-column (column 0) amounts
    — the snapshot SafeCRDT.Update shipped after an earlier op of a batch applied at once — equals the oracle's
    encoder over the rewound row, byte for byte, with the cell type's wrapping (amounts that cross the int32 /
    int64 edge included); the same row may be asked several times at different points."""
    rng = np.random.default_rng(40 + eb)
    n_keys, R = 50, 8
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, R, eb, stable)
    cl = Cluster(rng, n_keys, 6, eb, stable)
    keys = rng.integers(0, n_keys, 1500).astype(np.uint32)
    msgs = [cl.message(int(k)) for k in keys]
    pr.oracle(keys, msgs)
    pr.s.merge_json(keys, msgs)
    bits = 32 if eb == 4 else 64
    q = rng.integers(0, n_keys, 400).astype(np.uint32)
    dp = rng.integers(-2**40, 2**40, 400).astype(np.int64)
    dn = rng.integers(0, 2**20, 400).astype(np.int64)
    dp[:20] = 2**31 + 5  # past the int32 edge
    dn[20:40] = -(2**62)
    dp[40:60] = 0
    dn[40:60] = 0

    def wrap(x):
        x = int(x) % (1 << bits)
        return x - (1 << bits) if x >= 1 << (bits - 1) else x

    got = pr.s.encode_json_before(q, dp, dn)
    for i, k in enumerate(q):
        c = int(pr.ncols[k])
        P, N = pr.P[k, :c].astype(object).copy(), pr.N[k, :c].astype(object).copy()
        P[0], N[0] = wrap(int(P[0]) - int(dp[i])), wrap(int(N[0]) - int(dn[i]))
        exp = orc.json_encode_pnc(pr.cols[k, :c]["lo"], pr.cols[k, :c]["hi"], np.array(P, dtype=pr.P.dtype), np.array(N, dtype=pr.N.dtype), eb)
        assert got[i] == exp, f"query {i} key {k}"
    states, h = pr.s.encode_json_before(q, dp, dn, sha=True)  # and each state's SHA-256, hashed on the device
    assert states == got
    assert all(h[i].tobytes() == hashlib.sha256(got[i]).digest() for i in range(len(got)))
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
@pytest.mark.parametrize("n_keys,n_ops,merged", [(50, 1500, True), (200000, 100000, False), (3, 1, False)])
def test_apply_ops_encode_matches_oracle(ctx, eb, n_keys, n_ops, merged):
    """jg_pnc_apply_ops_encode (round 6): a batch of own-column Increment / Decrement ops (PNCounters.cs:96-112) and
    the snapshot each op shipped (SafeCRDT.cs:39-62: the key's row right after the op) in ONE call — every snapshot
    equals the oracle's encoder over the row walked op by op (replica columns merged in first, amounts across the
    int32 / int64 edge), each hash is SHA-256 of its bytes, and the store then holds every op's amount.  An output
    buffer too small is refused with JG_ESTATE and NOTHING applied."""
    rng = np.random.default_rng(3 * eb + n_ops)
    R = 8
    stable = random_guids(rng, n_keys)
    pr = Pair(ctx, n_keys, R, eb, stable)
    if merged:  # rows with several replica columns
        cl = Cluster(rng, n_keys, 6, eb, stable)
        mk = rng.integers(0, n_keys, 1500).astype(np.uint32)
        msgs = [cl.message(int(k)) for k in mk]
        pr.oracle(mk, msgs)
        pr.s.merge_json(mk, msgs)
    hot = rng.integers(0, n_keys, max(1, n_keys // 10))
    key = np.where(rng.random(n_ops) < 0.5, rng.choice(hot, n_ops), rng.integers(0, n_keys, n_ops)).astype(np.uint32)
    delta = rng.integers(1, 1000, n_ops).astype(np.int64)
    delta[rng.random(n_ops) < 0.02] = 2**31 - 3  # past the int32 edge once summed
    if eb == 8:
        delta[rng.random(n_ops) < 0.01] = 2**62
    is_n = (rng.random(n_ops) < 0.3).astype(np.uint8)
    P0, N0 = pr.s.read_rows()
    with pytest.raises(jg.JanusError):
        pr.s.apply_ops_encode(key, delta, is_n, cap=16)
    P1, N1 = pr.s.read_rows()
    assert np.array_equal(P0, P1) and np.array_equal(N0, N1), "a refused call applied ops"
    got, h = pr.s.apply_ops_encode(key, delta, is_n)
    assert len(got) == n_ops
    bits = 32 if eb == 4 else 64

    def wrap(x):
        x = int(x) % (1 << bits)
        return x - (1 << bits) if x >= 1 << (bits - 1) else x
    P, N = pr.P.astype(object), pr.N.astype(object)
    for i in range(n_ops):
        k = int(key[i])
        M = N if is_n[i] else P
        M[k, 0] = wrap(M[k, 0] + int(delta[i]))
        c = int(pr.ncols[k])
        exp = orc.json_encode_pnc(pr.cols[k, :c]["lo"], pr.cols[k, :c]["hi"], np.array(P[k, :c], dtype=pr.P.dtype),
                                  np.array(N[k, :c], dtype=pr.N.dtype), eb)
        assert got[i] == exp, f"op {i} key {k}"
    sample = range(n_ops) if n_ops <= 5000 else rng.integers(0, n_ops, 5000)
    assert all(h[i].tobytes() == hashlib.sha256(got[i]).digest() for i in sample)
    pr.P, pr.N = np.array(P, dtype=pr.P.dtype), np.array(N, dtype=pr.N.dtype)
    pr.check()
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
def test_apply_ops_encode_edges(ctx, eb):
    """jg_pnc_apply_ops_encode edges: an empty batch writes off[0] = 0 and touches nothing; an op on a key outside
    the store or a column past the store's replicas is refused with JG_EINVAL before anything is applied; one key
    hit by 70,000 ops (one segment across many scan tiles) with negative amounts and the int64 / int32 extremes
    walks op by op like the oracle, wrapping as the reference's checked-off arithmetic does."""
    rng = np.random.default_rng(90 + eb)
    n_keys, R = 5, 4
    pr = Pair(ctx, n_keys, R, eb, random_guids(rng, n_keys))
    got, h = pr.s.apply_ops_encode(np.zeros(0, np.uint32), np.zeros(0, np.int64), np.zeros(0, np.uint8))
    assert got == [] and h.shape[0] == 0
    P0, N0 = pr.s.read_rows()
    for key, col in ((np.array([0, n_keys], np.uint32), 0), (np.array([1, 2], np.uint32), R)):
        with pytest.raises(jg.JanusError) as e:
            pr.s.apply_ops_encode(key, np.ones(2, np.int64), np.zeros(2, np.uint8), col=col)
        assert e.value.code == jg.JG_EINVAL
    P1, N1 = pr.s.read_rows()
    assert np.array_equal(P0, P1) and np.array_equal(N0, N1), "a refused call applied ops"
    n_ops = 70000
    key = np.where(rng.random(n_ops) < 0.9, 3, rng.integers(0, n_keys, n_ops)).astype(np.uint32)
    delta = rng.integers(-1000, 1000, n_ops).astype(np.int64)
    delta[rng.random(n_ops) < 0.01] = -(2**31)
    delta[rng.random(n_ops) < 0.01] = 2**31 - 1
    if eb == 8:
        delta[rng.random(n_ops) < 0.005] = -(2**63)
        delta[rng.random(n_ops) < 0.005] = 2**63 - 1
    is_n = (rng.random(n_ops) < 0.4).astype(np.uint8)
    got, h = pr.s.apply_ops_encode(key, delta, is_n)
    bits = 32 if eb == 4 else 64

    def wrap(x):
        x = int(x) % (1 << bits)
        return x - (1 << bits) if x >= 1 << (bits - 1) else x
    P, N = pr.P.astype(object), pr.N.astype(object)
    for i in range(n_ops):
        k = int(key[i])
        M = N if is_n[i] else P
        M[k, 0] = wrap(M[k, 0] + int(delta[i]))
        if i % 7 == 0 or i >= n_ops - 50:
            c = int(pr.ncols[k])
            exp = orc.json_encode_pnc(pr.cols[k, :c]["lo"], pr.cols[k, :c]["hi"], np.array(P[k, :c], dtype=pr.P.dtype),
                                      np.array(N[k, :c], dtype=pr.N.dtype), eb)
            assert got[i] == exp, f"op {i} key {k}"
            assert h[i].tobytes() == hashlib.sha256(got[i]).digest()
    pr.P, pr.N = np.array(P, dtype=pr.P.dtype), np.array(N, dtype=pr.N.dtype)
    pr.check()
    pr.close()


@pytest.mark.parametrize("eb", [4, 8])
@pytest.mark.parametrize("n_keys,n_ops", [(40, 3000), (200000, 100000), (3, 1)])
def test_apply_ops_rewind_matches_walk(ctx, eb, n_keys, n_ops):
    """jg_pnc_apply_ops_rewind (round 6): a batch of own-column Increment / Decrement ops (PNCounters.cs:96-112)
    applied at once, and for every op whose snapshot ships (SafeCRDT.cs:39-62) the amounts the batch's LATER ops on
    the same key added to P and N — computed on the device by a sort and a segmented sum — equal the host's
    backward walk (round 5's SubmitClientUpdates), wrapping included; the store then holds every op's amount."""
    rng = np.random.default_rng(7 * eb + n_ops)
    pr = Pair(ctx, n_keys, 4, eb, random_guids(rng, n_keys))
    hot = rng.integers(0, n_keys, max(1, n_keys // 10))
    key = np.where(rng.random(n_ops) < 0.5, rng.choice(hot, n_ops), rng.integers(0, n_keys, n_ops)).astype(np.uint32)
    delta = rng.integers(1, 1000, n_ops).astype(np.int64)
    delta[rng.random(n_ops) < 0.01] = 2**31 - 3  # past the int32 edge once summed
    is_n = (rng.random(n_ops) < 0.3).astype(np.uint8)
    need = (rng.random(n_ops) < 0.6).astype(np.uint8)
    bits = 32 if eb == 4 else 64
    mask = (1 << bits) - 1
    amt = [(int(d) & 0xFFFFFFFF) if eb == 4 else int(d) for d in delta]
    exp_p, exp_n, after = [], [], {}
    for i in range(n_ops - 1, -1, -1):  # the walk: newest first, per key
        a = after.setdefault(int(key[i]), [0, 0])
        if need[i]:
            exp_p.append(a[0])
            exp_n.append(a[1])
        a[int(is_n[i])] += amt[i] if eb == 8 else (amt[i] if amt[i] < 2**31 else amt[i] - 2**32)
    exp_p, exp_n = exp_p[::-1], exp_n[::-1]
    dp, dn = pr.s.apply_ops_rewind(key, delta, is_n, need)

    def w64(x):
        x &= (1 << 64) - 1
        return x - (1 << 64) if x >= 1 << 63 else x
    assert [w64(int(x)) for x in dp] == [w64(x) for x in exp_p]
    assert [w64(int(x)) for x in dn] == [w64(x) for x in exp_n]
    P, N = pr.s.read_rows()
    tot = np.zeros((2, n_keys), object)
    for i in range(n_ops):
        tot[int(is_n[i]), int(key[i])] += int(delta[i])
    for which, M in ((0, P), (1, N)):
        got = [int(x) & mask for x in M[:, 0]]
        assert got == [int(t) & mask for t in tot[which]]
    pr.close()
