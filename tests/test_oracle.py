"""CPU-only: pin the oracle.

1. The reference's own known-answer tests (transcribed in oracle/test_kat.cpp) pass on the oracle.
2. The dense / record bridges agree with independent plain-Python restatements on seeded inputs.
3. The committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py) still hold.
"""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as orc
from gen import random_orset_pair, random_pnc

ROOT = Path(__file__).resolve().parent.parent
KAT = ROOT / "oracle" / "build" / "test_kat"
GOLDEN = ROOT / "tests" / "golden"


def _kat_names():
    src = (ROOT / "oracle" / "test_kat.cpp").read_text()
    return [l.split("(")[1].split(")")[0] for l in src.splitlines() if l.startswith("TEST(")]


@pytest.fixture(scope="module")
def kat_results():
    out = subprocess.run([str(KAT)], capture_output=True, text=True, timeout=120).stdout
    res = {}
    for line in out.splitlines():
        if line.startswith(("PASS ", "FAIL ")):
            name = line[5:].split(":")[0]
            res[name] = line
    return res


@pytest.mark.parametrize("name", _kat_names())
def test_reference_known_answer(kat_results, name):
    assert name in kat_results, f"{name} did not run"
    assert kat_results[name].startswith("PASS"), kat_results[name]


# ---------------------------------------------------------------- PN-Counter bridges
@pytest.mark.parametrize("eb", [4, 8])
def test_pnc_merge_bridge_matches_rule(eb):
    """Merge visits only the received entries: A = B absent ? A : max(A, B) (absent local = 0)."""
    rng = np.random.default_rng(1 + eb)
    A_P, A_N = random_pnc(rng, 50, 7, eb, absent=False), random_pnc(rng, 50, 7, eb, absent=False)
    B_P, B_N = random_pnc(rng, 50, 7, eb), random_pnc(rng, 50, 7, eb)
    P, N = orc.pnc_merge(A_P, A_N, B_P, B_N)
    absent = np.iinfo(A_P.dtype).min
    assert np.array_equal(P, np.where(B_P == absent, A_P, np.maximum(A_P, B_P)))
    assert np.array_equal(N, np.where(B_N == absent, A_N, np.maximum(A_N, B_N)))


def test_pnc_merge_bridge_repeated_keys():
    rng = np.random.default_rng(7)
    A_P = random_pnc(rng, 10, 5, 8, absent=False)
    A_N = random_pnc(rng, 10, 5, 8, absent=False)
    B_P, B_N = random_pnc(rng, 40, 5, 8), random_pnc(rng, 40, 5, 8)
    keys = rng.integers(0, 10, 40).astype(np.uint32)
    P, N = orc.pnc_merge(A_P, A_N, B_P, B_N, keys)
    eP, eN = A_P.copy(), A_N.copy()
    absent = np.iinfo(np.int64).min
    for m, k in enumerate(keys):
        eP[k] = np.where(B_P[m] == absent, eP[k], np.maximum(eP[k], B_P[m]))
        eN[k] = np.where(B_N[m] == absent, eN[k], np.maximum(eN[k], B_N[m]))
    assert np.array_equal(P, eP) and np.array_equal(N, eN)


def _py_get(prow, nrow, bits):
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1

    def csum(row):
        s = 0
        for v in row:
            s += int(v)
            if s < lo or s > hi:
                return None
        return s

    sp, sn = csum(prow), csum(nrow)
    if sp is None or sn is None:
        return 0, 1
    v = (sp - sn) & ((1 << bits) - 1)
    return (v - (1 << bits) if v > hi else v), 0


@pytest.mark.parametrize("eb", [4, 8])
def test_pnc_values_bridge_checked_sum(eb):
    rng = np.random.default_rng(3)
    info = np.iinfo(np.int32 if eb == 4 else np.int64)
    P = random_pnc(rng, 200, 9, eb, absent=False, lo=info.min // 4, hi=info.max // 3)
    N = random_pnc(rng, 200, 9, eb, absent=False, lo=info.min // 4, hi=info.max // 3)
    P[:10] = 0
    P[:10, 0] = info.max
    P[:5, 3] = 1  # overflow for keys 0..4 at the 4th prefix
    out, ovf = orc.pnc_values(P, N)
    for k in range(200):
        assert (int(out[k]), int(ovf[k])) == _py_get(P[k], N[k], eb * 8), k


def test_pnc_apply_ops_bridge_wraps():
    P = np.zeros((3, 2), np.int32)
    N = np.zeros((3, 2), np.int32)
    P[1, 1] = np.iinfo(np.int32).max
    P2, N2 = orc.pnc_apply_ops(P, N, [1, 1, 2], [1, 1, 0], [1, 5, -3], [0, 0, 1])
    assert P2[1, 1] == np.iinfo(np.int32).min + 5
    assert N2[2, 0] == -3


# ---------------------------------------------------------------- OR-Set bridges
def _py_sets(add, rem):
    d = {}
    for r in add:
        d.setdefault(int(r["key"]), [set(), set()])[0].add((int(r["tag_lo"]), int(r["tag_hi"])))
    for r in rem:
        d.setdefault(int(r["key"]), [set(), set()])[1].add((int(r["tag_lo"]), int(r["tag_hi"])))
    return d


def test_orset_merge_bridge_is_union():
    rng = np.random.default_rng(11)
    La, Lr, Ra, Rr = random_orset_pair(rng)
    oa, orr = orc.orset_merge(La, Lr, Ra, Rr)
    assert np.array_equal(orc.canon(oa), np.unique(np.concatenate([orc.canon(La), orc.canon(Ra)]), axis=0))
    assert np.array_equal(orc.canon(orr), np.unique(np.concatenate([orc.canon(Lr), orc.canon(Rr)]), axis=0))


def test_orset_contains_bridge_rule():
    rng = np.random.default_rng(12)
    La, Lr, _, _ = random_orset_pair(rng)
    d = _py_sets(La, Lr)
    sets = np.repeat(np.arange(8, dtype=np.uint32), 8)
    elems = np.tile(np.array(list(range(7)) + [orc.NULL_ELEM], np.uint32), 8)
    got = orc.orset_contains(La, Lr, sets, elems)
    for s, e, g in zip(sets, elems, got):
        a, r = d.get((int(s) << 32) | int(e), [set(), set()])
        if int(e) == orc.NULL_ELEM:
            exp = a != r
        else:
            exp = ((int(s) << 32) | int(e)) in d and len(a) > 0 and (len(r) == 0 or a != r)
        assert bool(g) == exp, (s, e)


def test_orset_lookup_all_order():
    # Add-only keys first (insertion order), then keys in both with differing sets, null last.
    def rec(s, e, t):
        return ((s << 32) | e, t, 0, 0)

    add = np.array([rec(0, 1, 5), rec(0, 2, 6), rec(0, 3, 7), rec(0, 3, 8), rec(0, orc.NULL_ELEM, 9)], orc.REC_DTYPE)
    rem = np.array([rec(0, 1, 5), rec(0, 3, 7)], orc.REC_DTYPE)
    assert list(orc.orset_lookup_all(add, rem, 0)) == [2, 3, orc.NULL_ELEM]


# ---------------------------------------------------------------- synthetic generators
def _mix64(x):
    m = (1 << 64) - 1
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & m
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & m
    x ^= x >> 31
    return x


def test_synth_pnc_formula():
    """DESIGN.md §Synthetic inputs, restated in plain Python."""
    seed, R = 0x4A414E5553, 5
    got = orc.synth_pnc(seed, 2, 3, 4, R, 8)
    for k in range(4):
        for c in range(R):
            idx = (((3 + k) * R + c) << 2) | 2
            h = _mix64((seed + (idx + 1) * 0x9E3779B97F4A7C15) & ((1 << 64) - 1))
            exp = np.iinfo(np.int64).min if h % 100 < 30 else (h >> 33) % 2147483647
            assert got[k, c] == exp


def test_synth_orset_formula():
    seed = 99
    got = orc.synth_orset(seed, 7, 5, 10, 4, 3)
    for i in range(5):
        r = 7 + i
        g, u = r // 4, 3 + r % 4
        h1 = _mix64(seed ^ _mix64(g * 256 + u + 1))
        h2 = _mix64((h1 + 0x9E3779B97F4A7C15) & ((1 << 64) - 1))
        assert int(got[i]["key"]) == ((g // 10) << 32) | (g % 10)
        assert int(got[i]["tag_lo"]) == (u << 56) | (h1 >> 8)
        assert int(got[i]["tag_hi"]) == h2
        assert int(got[i]["ord"]) == r  # arrival ordinal = the record's index in its stream


# ---------------------------------------------------------------- golden fixtures
def test_golden_pnc():
    z = np.load(GOLDEN / "pnc_merge_i32.npz")
    P, N = orc.pnc_merge(z["AP"], z["AN"], z["BP"], z["BN"], z["keys"])
    assert np.array_equal(P, z["outP"]) and np.array_equal(N, z["outN"])
    v, o = orc.pnc_values(P, N)
    assert np.array_equal(v, z["values"]) and np.array_equal(o, z["ovf"])


def test_golden_orset():
    z = np.load(GOLDEN / "orset_merge.npz")
    oa, orr = orc.orset_merge(z["La"], z["Lr"], z["Ra"], z["Rr"])
    assert np.array_equal(oa, z["out_add"]) and np.array_equal(orr, z["out_rem"])
    got = orc.orset_contains(oa, orr, z["q_set"], z["q_elem"])
    assert np.array_equal(got, z["contains"])


def test_orset_apply_ops_bridge_reference_sequence():
    """ORSetTests.cs:10-40 (SingleORSetValueType1) as an op batch on one set: Add 1, Add 2,
    Remove 1 -> true, Remove 3 -> false, Add 3, then Clear, Add 1."""
    empty = np.empty(0, orc.REC_DTYPE)
    ops = [(1, 1), (1, 2), (2, 1), (2, 3), (1, 3)]
    a, r, res = orc.orset_apply_ops(empty, empty, [0] * 5, [e for _, e in ops], [o for o, _ in ops],
                                    np.arange(1, 6), np.zeros(5))
    assert list(res) == [1, 1, 1, 0, 1]
    assert sorted(orc.orset_lookup_all(a, r, 0)) == [2, 3]
    a2, r2, res2 = orc.orset_apply_ops(a, r, [0, 0], [0, 1], [3, 1], [0, 9], [0, 0])
    assert list(res2) == [1, 1] and list(orc.orset_lookup_all(a2, r2, 0)) == [1] and r2.size == 0


# ---------------------------------------------------------------- enumeration order (jg_tagrec.ord)
def test_orset_merge_bridge_enumeration_order():
    """HashSet / Dictionary insertion order through the record bridge (oracle_ref.enum_view): Merge
    appends R's new tags after L's in R's order, and R's new tombstone elements after L's in R's
    Dictionary order (ORSet.cs:255-282; oracle/oracle.hpp GuidSet)."""
    def rec(e, t, o):
        return (e, t, 0, o)

    La = np.array([rec(1, 5, 0), rec(1, 6, 1), rec(2, 7, 2)], orc.REC_DTYPE)   # 1: [5, 6]; 2: [7]
    Lr = np.array([rec(2, 7, 0)], orc.REC_DTYPE)                               # removeSet: 2
    Ra = np.array([rec(1, 4, 1), rec(1, 6, 2), rec(1, 9, 0)], orc.REC_DTYPE)   # 1: [9, 4, 6]
    Rr = np.array([rec(1, 4, 1), rec(1, 9, 0), rec(3, 1, 5)], orc.REC_DTYPE)   # removeSet: 1 [9, 4], then 3
    oa, orr = orc.orset_merge(La, Lr, Ra, Rr)
    assert [(int(k), int(t)) for k, t, _ in orc.enum_view(oa, False)] == [(1, 5), (1, 6), (1, 9), (1, 4), (2, 7)]
    assert [(int(k), int(t)) for k, t, _ in orc.enum_view(orr, True)] == [(2, 7), (1, 9), (1, 4), (3, 1)]
    # the helpers agree with an explicit canonical ordering
    assert orc.same_orset(oa, orr, oa, orr) and not orc.same_stream(oa, Ra, False)


def test_orset_apply_json_enumeration_order():
    """The Python wire oracle keeps first-insertion order across messages (UnionWith appends)."""
    import jsongen as J
    g = [(i, 0) for i in range(1, 6)]
    m1 = J.encode_orset([("x", [g[2], g[0]])], [("x", [g[0]])])
    m2 = J.encode_orset([("y", [g[4]]), ("x", [g[1], g[0]])], [("y", [g[4]]), ("x", [g[2]])])
    ea, er, bad, _ = orc.orset_apply_json([0, 0], [m1, m2])
    assert bad is None
    assert [(int(k), int(t)) for k, t, _ in orc.enum_view(ea, False)] == [(0, 3), (0, 1), (0, 2), (1, 5)]
    assert [(int(k), int(t)) for k, t, _ in orc.enum_view(er, True)] == [(0, 1), (0, 3), (1, 5)]
