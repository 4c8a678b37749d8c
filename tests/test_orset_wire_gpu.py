"""GPU parity of the OR-Set wire path (jg_orset_wave_* / jg_orset_merge_json, csrc/orset_wire.hip).

ORSetMsg<string> payloads are decoded, their element strings interned and the states merged on the
device; the oracle is the restated ORSetMsg.Decode (oracle/json.hpp, ORSet.cs:56-63) driven through
tests/oracle_ref.orset_apply_json: Decode + Merge in commit order, element ids issued per set at first
insertion.  Comparisons are exact: the store's record streams, the ids each wave issued (set, id,
string), and the first rejected message with its code.
"""
import hashlib
import os

import numpy as np
import pytest

import janus_gpu as jg
import jsongen as J
import oracle_ref as orc

pytestmark = pytest.mark.gpu

G1, G2, G3 = (0x1122334455667788, 0x99AABBCCDDEEFF00), (0x0102030405060708, 0x0A0B0C0D0E0F1011), (7, 9)
_A, _B = J.guid_d(*G1), J.guid_d(*G2)


def _model_names(model, before):
    """New (set, id, bytes) entries of the oracle's interning since `before` (a copy), sorted."""
    out = []
    for s, tab in model.items():
        if isinstance(s, tuple):
            continue
        old = before.get(s, {})
        out.extend((s, i, n) for n, i in tab.items() if n not in old)
    return sorted(out)


def _copy(model):
    return {k: (dict(v) if isinstance(v, dict) else v) for k, v in model.items()}


def _stj_state(rng, a, r, na, nr):
    """The same decoded state as (a, r, na, nr) written with System.Text.Json's other accepted forms: an element named
    a second time EARLIER in its map with other tags (its first place moves there, its last tag set stays), or an
    earlier addSet occurrence that the real one replaces, plus (either way) an unknown member."""
    a, r = list(a), list(r)
    if a and rng.random() < 0.6:
        j = int(rng.integers(0, len(a)))
        k = int(rng.integers(0, j + 1))
        a.insert(k, (a[j][0], J.random_guids(rng, 2)))
    elif r and rng.random() < 0.5:
        j = int(rng.integers(0, len(r)))
        r.insert(int(rng.integers(0, j + 1)), (r[j][0], J.random_guids(rng, 1)))
    body = J.encode_orset(a, r, na, nr)
    if rng.random() < 0.5:
        body = b'{"addSet":{"junk":["' + J.guid_d(*G1).encode() + b'"]},' + body[1:]
    return b'{"zz":[1,{"q":"x"},null],' + body[1:]


def _run_waves(ctx, seed, n_sets, waves, per_wave, modes=("default",), chunks=3, stj=0.0):
    rng = np.random.default_rng(seed)
    cl = J.ORSetCluster(rng, n_sets)
    s = jg.ORSetStore(ctx)
    model, state = {}, {}
    try:
        for w in range(waves):
            sets, msgs = [], []
            for i in range(per_wave):
                sid = int(rng.integers(0, n_sets))
                a, r, na, nr = cl.state(sid)
                mode = modes[i % len(modes)]
                if stj and rng.random() < stj:
                    msgs.append(_stj_state(rng, a, r, na, nr))
                else:
                    msgs.append(J.encode_orset(a, r, na, nr, mode=mode, ws=" \t\r\n" if i % 7 == 3 else "",
                                               order=list(reversed(J._ORSET_MEMBERS)) if i % 5 == 2 else None, upper=i % 11 == 4))
                sets.append(sid)
            before = _copy(model)
            ea, er, bad, _ = orc.orset_apply_json(sets, msgs, model, state)  # the whole state so far
            assert bad is None
            cut = sorted(set(int(x) for x in rng.integers(0, len(msgs), chunks - 1)))
            bounds = [0] + cut + [len(msgs)]
            rc, first_bad = s.wave([(sets[b:e], msgs[b:e]) for b, e in zip(bounds, bounds[1:])])
            assert rc == jg.JG_OK and first_bad is None
            assert s.wave_names() == _model_names(model, before)
            ga, gr = s.read()
            assert orc.same_orset(ga, gr, ea, er)  # records and HashSet / Dictionary enumeration order
    finally:
        s.close()


# JANUS_ORSET_TAIL: the per-chunk string / record tables (strict: no fall-back), committed by set buckets
# (JANUS_ORSET_COMMIT=buckets, strict: from the counts the tables' claimants took when the whole wave commits),
# by set buckets counted from the lists (=count), or by the radix path; or the sort path
TAIL = ["tables", "tables-count", "tables-radix", "sort"]


def _tail(monkeypatch, tail):
    monkeypatch.setenv("JANUS_ORSET_TAIL", "tables" if tail.startswith("tables") else tail)
    monkeypatch.setenv("JANUS_ORSET_COMMIT", {"tables-radix": "radix", "tables-count": "count"}.get(tail, "buckets"))
PARSE = ["auto", "serial"]  # JANUS_ORSET_PARSE: one wave per message (k_ow_group) + serial fall-back, or serial only


@pytest.mark.parametrize("tail", TAIL)
@pytest.mark.parametrize("parse", PARSE)
@pytest.mark.parametrize("seed,n_sets,waves,per_wave", [(1, 3, 3, 40), (2, 64, 3, 600), (3, 500, 2, 3000)])
def test_waves_match_oracle(ctx, seed, n_sets, waves, per_wave, parse, tail, monkeypatch):
    monkeypatch.setenv("JANUS_ORSET_PARSE", parse)
    _tail(monkeypatch, tail)
    _run_waves(ctx, seed, n_sets, waves, per_wave, modes=("default", "raw", "all"))


@pytest.mark.parametrize("tail", TAIL)
@pytest.mark.parametrize("parse", ["group", "default"])
def test_compact_waves_match_oracle(ctx, parse, tail, monkeypatch):
    """Reference-shaped compact states only (ASCII names, no whitespace, members in the encoder's order):
    every message takes the group parse (JANUS_ORSET_PARSE=group rejects any message it leaves), and
    with JANUS_ORSET_TAIL=tables every wave commits from the per-chunk tables."""
    _tail(monkeypatch, tail)
    if parse == "group":
        monkeypatch.setenv("JANUS_ORSET_PARSE", "group")
    rng = np.random.default_rng(11)
    s = jg.ORSetStore(ctx)
    model, state = {}, {}
    try:
        for w in range(3):
            sets, msgs = [], []
            for i in range(2000):
                sid = int(rng.integers(0, 50))
                nel = int(rng.integers(0, 40))
                add = [(f"e{sid}_{j}", J.random_guids(rng, int(rng.integers(1, 3)))) for j in range(nel)]
                rem = [(e, ts[:1]) for e, ts in add if rng.random() < 0.3]
                na = J.random_guids(rng, int(rng.integers(0, 3)))
                nr = na[:int(rng.integers(0, len(na) + 1))]
                msgs.append(J.encode_orset(add, rem, na, nr, upper=i % 9 == 4))
                sets.append(sid)
            before = _copy(model)
            ea, er, bad, _ = orc.orset_apply_json(sets, msgs, model, state)
            assert bad is None
            rc, first_bad = s.wave([(sets[:700], msgs[:700]), (sets[700:], msgs[700:])])
            assert rc == jg.JG_OK and first_bad is None
            assert s.wave_names() == _model_names(model, before)
            ga, gr = s.read()
            assert orc.same_orset(ga, gr, ea, er)
    finally:
        s.close()


def _mutants(rng, base, n):
    """Single-byte edits of a payload: replace, delete or insert one byte at a random position."""
    alphabet = b'"{}[]:, \\a0-Gf\x00\xc3\t'
    out = []
    for _ in range(n):
        p = int(rng.integers(0, len(base)))
        ch = bytes([alphabet[int(rng.integers(0, len(alphabet)))]])
        kind = int(rng.integers(0, 3))
        out.append(base[:p] + ch + base[p + 1:] if kind == 0 else base[:p] + base[p + 1:] if kind == 1 else base[:p] + ch + base[p:])
    return out


def test_group_parse_mutants_equal_serial(ctx, monkeypatch):
    """Single-byte mutants of compact reference-shaped states, each merged on its own (one-shot calls, all or
    nothing) into a store per parse mode: the group parse (which proves a payload compact or hands it to the
    serial parse) ends with the same error codes, first bad messages, element ids and records as the serial
    parse alone.  Mutants that stay valid (a changed hex digit, name byte...) are merged by both."""
    rng = np.random.default_rng(12)
    bases = [J.encode_orset([("abcde", [G1]), ("x", [G2, G3])], [("x", [G2])], [G3], []),
             J.encode_orset([], [], [], []),
             J.encode_orset([("k", [G1])], [], [G2], [G2]),
             J.encode_orset([(f"n{j}", [G1, G2]) for j in range(6)], [("n1", [G1])], [], [G3])]
    muts = [m for b in bases for m in _mutants(rng, b, 160)] + bases
    results = {}
    for mode, tail in (("auto", "tables"), ("serial", "sort")):
        monkeypatch.setenv("JANUS_ORSET_PARSE", mode)
        monkeypatch.setenv("JANUS_ORSET_TAIL", tail)
        s = jg.ORSetStore(ctx)
        try:
            codes = []
            for i, m in enumerate(muts):
                try:
                    s.merge_json([i], [m])
                    codes.append((0, None))
                except jg.JanusError as e:
                    codes.append((e.code, e.bad_msg))
            results[mode] = (codes, s.read())
        finally:
            s.close()
    (cg, rg), (cs, rs) = results["auto"], results["serial"]
    assert cg == cs
    assert orc.same_orset(rg[0], rg[1], rs[0], rs[1])  # records and enumeration order (ord values are the engine's own)
    assert sum(c == (0, None) for c in cg) > len(bases)  # some mutants stayed valid
    # the unmutated bases are compact: the group parse alone takes them
    monkeypatch.setenv("JANUS_ORSET_PARSE", "group")
    s = jg.ORSetStore(ctx)
    try:
        s.merge_json(list(range(len(bases))), bases)
    finally:
        s.close()


@pytest.mark.parametrize("parse", PARSE)
def test_group_parse_size_limits(ctx, parse, monkeypatch):
    """States around the group parse's limits (4096 bytes with the 16-byte alignment offset, 192 string
    tokens): the ones past them take the serial parse, with the same result as the oracle."""
    monkeypatch.setenv("JANUS_ORSET_PARSE", parse)
    rng = np.random.default_rng(13)
    msgs, sets = [], []
    for nel in (60, 75, 80, 84, 85, 86, 90, 95, 120):  # "eNN":[guid] = 47-48 bytes per element
        add = [(f"e{j:02d}", J.random_guids(rng, 1)) for j in range(nel)]
        msgs.append(J.encode_orset(add, [], [], []))
        sets.append(len(sets))
    for nt in (90, 95, 100, 110):  # null tags: 39 bytes each, one token each
        msgs.append(J.encode_orset([], [], J.random_guids(rng, nt), []))
        sets.append(len(sets))
    assert min(len(m) for m in msgs) < 4080 < max(len(m) for m in msgs)
    ea, er, bad, _ = orc.orset_apply_json(sets, msgs)
    assert bad is None
    s = jg.ORSetStore(ctx)
    try:
        rc, first_bad = s.wave([(sets, msgs)])
        assert rc == jg.JG_OK and first_bad is None
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
    finally:
        s.close()


def test_hash_collisions_take_the_exact_path(ctx, monkeypatch):
    """With the string hash narrowed to 3 bits every run of equal hashes mixes strings: labels, duplicate
    detection and the element table must still compare strings byte for byte."""
    monkeypatch.setenv("JANUS_TEST_NAME_HASH_BITS", "3")
    _run_waves(ctx, 4, 6, 3, 120, modes=("default", "raw"))


@pytest.mark.parametrize("tail", ["auto", "sort"])
def test_entry_runs_mixing_full_keys(ctx, tail, monkeypatch):
    """With the entry sort narrowed to 4 key bits every run holds strings whose full keys differ: the run is
    labelled string by string and each string is looked up under its own full key."""
    monkeypatch.setenv("JANUS_TEST_ENTRY_SORT_BITS", "4")
    monkeypatch.setenv("JANUS_ORSET_TAIL", tail)
    _run_waves(ctx, 5, 6, 3, 120, modes=("default", "raw"))


def test_names_sync_and_clear(ctx):
    s = jg.ORSetStore(ctx)
    try:
        # host-issued names (ORSet.Add ops) registered first: the wave resolves to them
        s.names_sync(sets=[0, 1], next_ids=[2, 1], cleared=[0, 0], names=[(0, 0, b"x"), (0, 1, "é".encode()), (1, 0, b"x")])
        m = [J.encode_orset([("é", [G1]), ("new", [G2])], [("x", [G3])]), J.encode_orset([("x", [G1])], [], [G2])]
        s.merge_json([0, 1], m)
        assert s.wave_names() == [(0, 2, b"new")]
        ga, gr = s.read()
        exp_a = sorted([(0 << 32 | 1, *G1), (0 << 32 | 2, *G2), (1 << 32 | 0, *G1), (1 << 32 | jg.NULL_ELEM, *G2)])
        assert [tuple(int(v) for v in r) for r in orc.canon(ga)] == exp_a
        assert [tuple(int(v) for v in r) for r in orc.canon(gr)] == [(0 << 32 | 0, *G3)]
        # Clear of set 0: its strings are dropped, ids keep growing; set 1 keeps "x"
        s.names_sync(sets=[0], next_ids=[3], cleared=[1])
        s.merge_json([0, 1, 0], [J.encode_orset([("x", [G2])], []), J.encode_orset([("x", [G3])], []),
                                 J.encode_orset([("new", [G3]), ("x", [G1])], [])])
        assert s.wave_names() == [(0, 3, b"x"), (0, 4, b"new")]
        ga, _ = s.read()
        keys = {int(r["key"]) for r in ga}
        assert {0 << 32 | 3, 0 << 32 | 4, 1 << 32 | 0} <= keys
    finally:
        s.close()


_GOOD = J.encode_orset([("a", [G1])], [("a", [G1])], [G2], [])
# (payload, expected code or None): the ORSetMsg wire contract of oracle/json.hpp, plus the engine's
# empty-tag-set limit (JG_ESTATE, add or tombstone side) and the reader's error order
_CASES = [
    (J.encode_orset([("a", [G1, G1, G2])], []), None),                     # repeated tag in one array: one record
    (J.encode_orset([], [], [], []), None),
    (J.encode_orset([("a", [G1])], [("a", [])]), jg.JG_ESTATE),            # empty tombstone set: no record holds its key
    (J.encode_orset([("a", [G1])], [], [], [], mode="all"), None),         # escaped names and Guids
    (b'{"add\\u0053et":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', None),
    (J.encode_orset([("a", [G1])], [], upper=True, ws="\r\n\t "), None),
    (J.encode_orset([("a", [])], []), jg.JG_ESTATE),
    (J.encode_orset([("a", [G1]), ("b", [])], []), jg.JG_ESTATE),
    # System.Text.Json past the compact form (oracle/json.hpp, round 6): an element named twice in one map keeps its
    # first place and its LAST tag set; unknown members are skipped; a repeated member's last occurrence counts
    (J.encode_orset([("a", [G1]), ("a", [G2])], []), None),
    (J.encode_orset([("a", [G1])], [("b", [G1]), ("b", [])]), jg.JG_ESTATE),  # the last tombstone set is empty
    (J.encode_orset([("a", [G1])], [], mode="all")[:-1] + b',"a":[]}', None),  # an unknown member "a"
    (J.encode_orset([("a", []), ("a", [G1])], []), None),                   # the empty set is replaced
    (J.encode_orset([("a", [G1]), ("a", [])], []), jg.JG_ESTATE),          # the last set is empty
    (J.encode_orset([("x", [G1]), ("a", [G2]), ("y", [G3]), ("a", [G1, G3])], [("a", [G3]), ("x", [G1]), ("a", [G1])]), None),
    (b'{"addSet":{"a":null,"a":["' + _A.encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', None),
    (b'{"addSet":{"a":["' + _A.encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[],"addSet":null}', jg.JG_EINVAL),
    (b'{"q":{"w":[1,2.5,{"e":"\\u00e9"}],"t":true},"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', None),
    (b'{"q":[1,},"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":null,"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":null},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[],"x":[]}', None),
    (b'{"addSet":{"z":["' + _B.encode() + b'"]},"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', None),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]} x', jg.JG_EINVAL),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]', jg.JG_EINVAL),
    (b'{"addSet":{"\xff":["' + _A.encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"\\ud800":["' + _A.encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A[:-1].encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A.replace("-", "x", 1).encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A.encode() + b'",]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a\x01":["' + _A.encode() + b'"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":["' + _B.encode() + b'"],"nullRemoveGuid":null}', jg.JG_EINVAL),
    (b'', jg.JG_EINVAL),
    # the fixed-position Guid decoder's fall-backs: a bad last digit, one digit too many, the payload
    # ending right after / inside a tag
    (b'{"addSet":{"a":["' + _A[:-1].encode() + b'g"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A.encode() + b'0"]},"removeSet":{},"nullAddGuid":[],"nullRemoveGuid":[]}', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A.encode() + b'"', jg.JG_EINVAL),
    (b'{"addSet":{"a":["' + _A[:20].encode(), jg.JG_EINVAL),
    (b'{"addSet":{},"removeSet":{},"nullAddGuid":["' + _B.upper().encode() + b'"],"nullRemoveGuid":[]}', None),
]


@pytest.mark.parametrize("tail", TAIL)
@pytest.mark.parametrize("parse", PARSE)
def test_stj_forms_in_waves_match_oracle(ctx, parse, tail, monkeypatch):
    """states System.Text.Json decodes beyond the compact form — an element named twice in one map
    (first place, last tag set), a replaced addSet, unknown members — mixed into waves of compact states: the group
    parse hands them to the serial parse, whose entries and tags come in ORSet.Merge's walk order; records, arrival
    ordinals (enumeration order) and issued names equal the oracle's.  Parity unpinned by reference fixtures."""
    _tail(monkeypatch, tail)
    monkeypatch.setenv("JANUS_ORSET_PARSE", parse)
    _run_waves(ctx, 91, 40, 3, 500, stj=0.3)


@pytest.mark.parametrize("tail", TAIL)
@pytest.mark.parametrize("parse", PARSE)
@pytest.mark.parametrize("idx", range(len(_CASES)))
def test_contract_case_in_a_wave(ctx, idx, parse, tail, monkeypatch):
    """Case payload at position 3 of a 6-message wave: the first bad message and its code, then the
    prefix before it merges exactly as the oracle's loop leaves the store."""
    monkeypatch.setenv("JANUS_ORSET_PARSE", parse)
    monkeypatch.setenv("JANUS_ORSET_TAIL", tail)
    payload, code = _CASES[idx]
    dec = orc.json_decode_orset(payload)
    if code is None:
        assert dec is not None
    elif code == jg.JG_EINVAL:
        assert dec is None  # the oracle's Decode rejects it too
    msgs = [_GOOD, J.encode_orset([("b", [G2])], []), _GOOD, payload, J.encode_orset([("c", [G3])], []), _GOOD]
    sets = [0, 1, 2, 0, 1, 2]
    s = jg.ORSetStore(ctx)
    try:
        rc, bad = s.wave([(sets[:2], msgs[:2]), (sets[2:], msgs[2:])])
        assert rc == (code or jg.JG_OK)
        assert bad == (None if code is None else 3)
        lim = 6 if code is None else 3
        ea, er, _, _ = orc.orset_apply_json(sets[:lim], msgs[:lim])
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
        # one-shot form: all or nothing
        t = jg.ORSetStore(ctx)
        try:
            if code is None:
                t.merge_json(sets, msgs)
                assert all(np.array_equal(x, y) for x, y in zip(t.read(), s.read()))
            else:
                with pytest.raises(jg.JanusError) as ei:
                    t.merge_json(sets, msgs)
                assert ei.value.code == code and ei.value.bad_msg == 3
                assert [len(x) for x in t.read()] == [0, 0]
        finally:
            t.close()
    finally:
        s.close()


def test_empty_and_all_bad_waves(ctx):
    s = jg.ORSetStore(ctx)
    try:
        s.merge_json([], [])
        assert [len(x) for x in s.read()] == [0, 0]
        rc, bad = s.wave([([5], [b"{"])])
        assert rc == jg.JG_EINVAL and bad == 0
        assert [len(x) for x in s.read()] == [0, 0] and s.wave_names() == []
    finally:
        s.close()


@pytest.mark.parametrize("n_tags", [3, 64, 65, 300])
def test_element_with_many_new_tags(ctx, n_tags):
    """The commit sorts a wave's new records by key and orders each key's tags in place; an element with more
    than 64 new tags in one wave takes the full three-word sort.  Both must give the oracle's records."""
    rng = np.random.default_rng(14 + n_tags)
    big = J.random_guids(rng, n_tags)
    msgs = [J.encode_orset([("big", big), ("x", J.random_guids(rng, 2))], [("x", big[:1])]),
            J.encode_orset([("big", big[: n_tags // 2] + J.random_guids(rng, 5))], [("big", big[:7])], J.random_guids(rng, 70), []),
            J.encode_orset([("y", J.random_guids(rng, 1))], [])]
    sets = [3, 3, 4]
    ea, er, bad, _ = orc.orset_apply_json(sets, msgs)
    assert bad is None
    s = jg.ORSetStore(ctx)
    try:
        s.merge_json(sets, msgs)
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
    finally:
        s.close()


def test_hot_name_in_long_impure_runs(ctx, monkeypatch):
    """A name repeated thousands of times in a run that also holds other strings (the entry sort narrowed to 4
    key bits, so every run mixes strings): labelling scans an impure run only up to 64 entries, then the wave's
    entries are sorted again on their whole keys — linear work, the oracle's result.  (The sort path's
    labelling: JANUS_ORSET_TAIL=sort.)"""
    import time
    monkeypatch.setenv("JANUS_ORSET_TAIL", "sort")
    monkeypatch.setenv("JANUS_TEST_ENTRY_SORT_BITS", "4")
    rng = np.random.default_rng(15)
    hot = J.random_guids(rng, 1)
    msgs, sets = [], []
    for i in range(6000):
        others = [(f"o{int(rng.integers(0, 40))}", J.random_guids(rng, 1))]
        msgs.append(J.encode_orset([("hot", hot)] + others, []))
        sets.append(0)
    s = jg.ORSetStore(ctx)
    try:
        t0 = time.perf_counter()
        s.merge_json(sets, msgs)
        dt = time.perf_counter() - t0
        ga, gr = s.read()
        ea, er, bad, _ = orc.orset_apply_json(sets, msgs)
        assert bad is None and orc.same_orset(ga, gr, ea, er)
        assert dt < 5.0, dt
    finally:
        s.close()


def test_names_log_holds_every_wave_and_sync(ctx):
    """jg_orset_names_since: the store's names log is every wave's issued names (jg_orset_wave_names) and every
    synced name, in the order the table took them; a pull from any point returns its tail."""
    rng = np.random.default_rng(31)
    cl = J.ORSetCluster(rng, 20)
    s = jg.ORSetStore(ctx)
    try:
        log = []
        for w in range(4):
            sets = [int(x) for x in rng.integers(0, 20, 300)]
            msgs = [J.encode_orset(*cl.state(k)) for k in sets]
            rc, bad = s.wave([(sets[:150], msgs[:150]), (sets[150:], msgs[150:])])
            assert rc == jg.JG_OK and bad is None
            log += s.wave_names()
            if w == 1:  # names a caller issued itself (ORSet.Add): appended to the log as synced
                nxt = max(i for st_, i, _ in log if st_ == 3) + 1
                s.names_sync(sets=[3], next_ids=[nxt + 2], cleared=[0], names=[(3, nxt, b"own-a"), (3, nxt + 1, b"own-b")])
                log += [(3, nxt, b"own-a"), (3, nxt + 1, b"own-b")]
        end, got = s.names_since(0)
        assert end == len(log) and got == log
        for k in (1, len(log) // 3, len(log) - 1, len(log)):
            end, tail = s.names_since(k)
            assert end == len(log) and tail == log[k:]
        with pytest.raises(jg.JanusError):
            s.names_since(len(log) + 1)
    finally:
        s.close()


def test_element_id_space_limit(ctx):
    """Ids are issued up to 2^32 - 3 (JG_NULL_ELEM - 1 is reserved): a wave that could pass it is rejected with
    JG_ESTATE and nothing applied; one that fits commits."""
    s = jg.ORSetStore(ctx)
    try:
        s.names_sync(sets=[0], next_ids=[0xFFFFFFFC], cleared=[0])
        with pytest.raises(jg.JanusError) as e:
            s.merge_json([0], [J.encode_orset([("a", [G1]), ("b", [G2]), ("c", [G3])], [])])
        assert e.value.code == jg.JG_ESTATE
        assert all(len(x) == 0 for x in s.read())
        s.merge_json([0], [J.encode_orset([("a", [G1]), ("b", [G2])], [])])
        assert s.wave_names() == [(0, 0xFFFFFFFC, b"a"), (0, 0xFFFFFFFD, b"b")]
    finally:
        s.close()


@pytest.mark.parametrize("tail", ["tables", "sort"])
def test_element_id_room_is_per_set(ctx, monkeypatch, tail):
    """the id-space check is per set.  Set 0 synced 2 ids below the limit does not block a wave of 300
    new names in set 1 (the old global bound refused it), nor one of 2 names in set 0; 3 names in set 0 are refused
    with JG_ESTATE and nothing applied — on both wave paths (tables, sort)."""
    monkeypatch.setenv("JANUS_ORSET_TAIL", tail)
    rng = np.random.default_rng(5)
    s = jg.ORSetStore(ctx)
    try:
        s.names_sync(sets=[0, 1], next_ids=[0xFFFFFFFC, 0], cleared=[0, 0])
        many = [(f"n{j}", J.random_guids(rng, 1)) for j in range(300)]
        s.merge_json([1] * 3, [J.encode_orset(many[k:k + 100], []) for k in range(0, 300, 100)])
        got = s.wave_names()
        assert len(got) == 300 and [i for _, i, _ in got] == list(range(300)) and all(st == 1 for st, _, _ in got)
        with pytest.raises(jg.JanusError) as e:
            s.merge_json([0, 1], [J.encode_orset([("a", [G1]), ("b", [G2]), ("c", [G3])], []), J.encode_orset([("z", [G1])], [])])
        assert e.value.code == jg.JG_ESTATE
        assert sum(len(x) for x in s.read()) == 300  # nothing of the refused wave applied
        s.merge_json([0], [J.encode_orset([("a", [G1]), ("b", [G2])], [])])
        assert s.wave_names() == [(0, 0xFFFFFFFC, b"a"), (0, 0xFFFFFFFD, b"b")]
    finally:
        s.close()


@pytest.mark.parametrize("commit", ["buckets", "radix", "auto"])
def test_big_set_buckets_fall_back(ctx, commit, monkeypatch):
    """A set with more new names / records in one wave than the bucket commit's LDS sorts hold (2048) takes the
    radix path (auto), is refused under JANUS_ORSET_COMMIT=buckets, and either way the ids and records equal
    the oracle's."""
    monkeypatch.setenv("JANUS_ORSET_TAIL", "tables")
    monkeypatch.setenv("JANUS_ORSET_COMMIT", commit)
    rng = np.random.default_rng(41)
    # 60 states of 45 new names each, all of set 0 (spread over the tables' sub-lists), then a small set
    big = [(f"b{j}", J.random_guids(rng, 1)) for j in range(2700)]
    msgs = [J.encode_orset(big[k:k + 45], []) for k in range(0, 2700, 45)] + [J.encode_orset([("x", J.random_guids(rng, 2))], [])]
    sets = [0] * 60 + [1]
    model = {}
    ea, er, bad, _ = orc.orset_apply_json(sets, msgs, model)
    assert bad is None
    s = jg.ORSetStore(ctx)
    try:
        if commit == "buckets":
            with pytest.raises(jg.JanusError) as e:
                s.wave([(sets[:30], msgs[:30]), (sets[30:], msgs[30:])])
            assert e.value.code == jg.JG_ESTATE and "bucket" in str(e.value)
            return
        rc, first_bad = s.wave([(sets[:30], msgs[:30]), (sets[30:], msgs[30:])])
        assert rc == jg.JG_OK and first_bad is None
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
        assert s.wave_names() == _model_names(model, {})
    finally:
        s.close()


@pytest.mark.parametrize("spec", ["1", "0"])
def test_tables_sized_from_the_last_wave(ctx, monkeypatch, spec):
    """The default tail sizes a wave's string / record tables from the previous wave's distinct counts: a small
    wave, then one with ~180k distinct strings (far past the small wave's room: the tables overflow and the wave
    commits by the sort path), then another big one (sized from the bound again): every wave equals the
    oracle.  spec=1 (the default): the check queues the claims' bucket scatter before its read, so on the
    overflowed wave that scatter runs over stale places and must leave without writing (round 5's fault was a
    store of this speculative launch past its arrays); spec=0 (JANUS_ORSET_SPEC=0): nothing is queued
    before the read and a whole-wave commit counts from the lists."""
    for v in ("JANUS_ORSET_TAIL", "JANUS_ORSET_COMMIT", "JANUS_ORSET_PARSE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("JANUS_ORSET_SPEC", spec)
    rng = np.random.default_rng(77)
    s = jg.ORSetStore(ctx)
    model, state = {}, {}
    try:
        for w, (n_msgs, n_names) in enumerate([(3, 2), (3000, 60), (3000, 60)]):
            sets, msgs = [], []
            for i in range(n_msgs):
                sid = int(rng.integers(0, 400))
                add = [(f"w{w}m{i}n{j}", J.random_guids(rng, 1)) for j in range(n_names)]
                msgs.append(J.encode_orset(add, add[:1]))
                sets.append(sid)
            before = _copy(model)
            ea, er, bad, _ = orc.orset_apply_json(sets, msgs, model, state)
            assert bad is None
            half = len(msgs) // 2
            rc, first_bad = s.wave([(sets[:half], msgs[:half]), (sets[half:], msgs[half:])])
            assert rc == jg.JG_OK and first_bad is None
            assert s.wave_names() == _model_names(model, before)
            ga, gr = s.read()
            assert orc.same_orset(ga, gr, ea, er)
    finally:
        s.close()


@pytest.mark.parametrize("chunking", ["one", "odd"])
def test_tag_references_dealt_over_lanes(ctx, monkeypatch, chunking):
    """k_ow_rkeys / k_ow_rins deal four messages' tag references over a wave's 64 lanes in rounds
    (orset_tables.hpp WaveMsgs): tag counts whose running totals fall just below, on and past multiples of 64,
    empty states (no references) between them, and chunks of odd sizes (a wave's four messages start at any
    chunk offset).  Records, arrival ordinals and issued names equal the oracle's; the tables path alone
    (JANUS_ORSET_TAIL=tables: an overflow would be an error, not a fall-back)."""
    monkeypatch.setenv("JANUS_ORSET_TAIL", "tables")
    rng = np.random.default_rng(2024)
    counts = [63, 1, 0, 65, 64, 2, 0, 0, 130, 1, 1, 1, 61, 3, 0, 64, 127, 0, 1, 66, 5]
    sets, msgs, k = [], [], 0
    for i, c in enumerate(counts):
        add = [(f"e{k + j}", J.random_guids(rng, 1)) for j in range(c)]
        k += c
        rem = add[: c // 3]  # tombstones of a third of them: references on both sides
        msgs.append(J.encode_orset(add, rem))
        sets.append(i % 3)
    model = {}
    ea, er, bad, _ = orc.orset_apply_json(sets, msgs, model)
    assert bad is None
    if chunking == "one":
        chunks = [(sets, msgs)]
    else:
        cuts = [0, 3, 8, 9, 14, len(msgs)]
        chunks = [(sets[a:b], msgs[a:b]) for a, b in zip(cuts, cuts[1:])]
    s = jg.ORSetStore(ctx)
    try:
        rc, first_bad = s.wave(chunks)
        assert rc == jg.JG_OK and first_bad is None
        ga, gr = s.read()
        assert orc.same_orset(ga, gr, ea, er)
        assert s.wave_names() == _model_names(model, {})
    finally:
        s.close()


def test_names_since_pull_between_marks_with_out_of_order_pool_bytes(ctx):
    """Regression for round 4's abort inside jg_orset_names_since (gpurun_out/t2.log, rc 134): a wave's
    new names take their pool bytes by device atomics, in workgroup arrival order, not in name (id) order, so a
    pull whose `from` falls inside a wave (between two commit marks) must take the pool range from the mark at or
    before `from`, not from name `from`'s own offset.  Three waves of 800 states naming 3 new elements each, with
    lengths 6..61 bytes (out-of-order claims move bytes by whole names); every pull from every position inside the
    second wave (and a stride over the rest) returns exactly the log's tail, and its size query returns exactly the
    tail's byte count (a short count is what let the fill write past the caller's buffer)."""
    import ctypes as C
    rng = np.random.default_rng(97)
    s = jg.ORSetStore(ctx)
    try:
        log, marks = [], [0]
        for w in range(3):
            sets = [int(x) for x in rng.integers(0, 64, 800)]
            msgs = []
            for m, k in enumerate(sets):
                adds = []
                for j in range(3):
                    ln = int(rng.integers(6, 62))  # a unique 6-byte head (no repeated key inside a message), then padding
                    name = (f"{w}{m:04d}{j}" + "".join(chr(97 + int(c)) for c in rng.integers(0, 26, 64)))[:ln]
                    adds.append((name, J.random_guids(rng, 1)))
                msgs.append(J.encode_orset(adds, []))
            rc, bad = s.wave([(sets[:400], msgs[:400]), (sets[400:], msgs[400:])])
            assert rc == jg.JG_OK and bad is None
            log += s.wave_names()
            marks.append(len(log))
        assert marks[1] > 1000  # names differ by prefix, so almost every element is new
        lib = jg.load()
        positions = list(range(marks[1] - 2, marks[2] + 3)) + list(range(0, len(log) + 1, 97))
        for k in positions:
            to, nb = C.c_uint64(), C.c_uint64()
            assert lib.jg_orset_names_since(s._h, k, C.byref(to), C.byref(nb), None, None, None, None) == jg.JG_OK
            assert to.value == len(log)
            assert nb.value == sum(len(b) for _, _, b in log[k:]), k
            end, tail = s.names_since(k)
            assert end == len(log) and tail == log[k:], k
    finally:
        s.close()


def test_encode_snapshot_limits_equal_step_by_step_states(ctx):
    """jg_orset_apply_ops_ords + jg_orset_encode_json(add_lim, rem_lim): the snapshot of op i's set encoded from the
    store after the WHOLE batch, at op i's ord limits, equals the same set encoded (no limits) from a second store that
    applied only ops[0..i] — SafeCRDT.Update's GetLastSynchronizedUpdate() after every op (SafeCRDT.cs:39-62), from
    one apply call.  Adds, Removes (tombstones) and the null element; Clears only before a set's last snapshot (the
    host mirror cuts its batches at a Clear that follows a needed snapshot).  The encoder's bytes themselves are
    checked against the oracle's System.Text.Json restatement by the host parity run (test_apply_loop_gpu)."""
    rng = np.random.default_rng(12)
    names = [b"a", b"b<&>", "café".encode(), "\U0001F600x".encode(), b"q\"\\", b"\t\x01", b"zz"]
    n_sets, n_ops = 5, 120
    a, b = jg.ORSetStore(ctx), jg.ORSetStore(ctx)
    try:
        for st in (a, b):
            st.names_sync(sets=list(range(n_sets)), next_ids=[len(names)] * n_sets, cleared=[0] * n_sets,
                          names=[(s, i, nm) for s in range(n_sets) for i, nm in enumerate(names)])
        sets = rng.integers(0, n_sets, n_ops).astype(np.uint32)
        elems = rng.integers(0, len(names) + 1, n_ops).astype(np.uint32)
        elems[elems == len(names)] = jg.NULL_ELEM
        ops = np.where(rng.random(n_ops) < 0.7, 1, 2).astype(np.uint8)
        ops[60] = 3  # a Clear: the snapshots checked below stop before it for its set... or are after it
        lo = rng.integers(1, 2**63, n_ops, dtype=np.uint64)
        hi = rng.integers(1, 2**63, n_ops, dtype=np.uint64)
        res, al, rl = a.apply_ops_ords(sets, elems, ops, lo, hi)
        check = [i for i in range(n_ops) if not (i < 60 and sets[i] == sets[60])]
        snaps, h = a.encode_json(sets[check], al[check], rl[check], sha=True)
        assert all(h[k].tobytes() == hashlib.sha256(snaps[k]).digest() for k in range(len(snaps)))  # hashed on the device
        got = dict(zip(check, snaps))
        for i in range(n_ops):
            r = b.apply_ops(sets[i:i + 1], elems[i:i + 1], ops[i:i + 1], lo[i:i + 1], hi[i:i + 1])
            assert r[0] == res[i]
            if i in got:
                exp = b.encode_json([sets[i]])[0]
                assert got[i] == exp, (i, got[i], exp)
        # no limits: the final states of both stores agree
        assert a.encode_json(list(range(n_sets))) == b.encode_json(list(range(n_sets)))
    finally:
        a.close()
        b.close()
