"""ctypes binding of the TEST-ONLY CPU oracle (oracle/capi.cpp).  Only tests/, smoke() and bench.py's
cpu_baseline leg use this; the product path never does."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "oracle" / "build" / "liboracle.so"
REC_DTYPE = np.dtype([("key", "<u8"), ("tag_lo", "<u8"), ("tag_hi", "<u8"), ("ord", "<u8")])  # jg_tagrec
NULL_ELEM = 0xFFFFFFFF

_vp, _u64, _u32, _i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
_SIGS = {
    "orc_version": ([], C.c_int),
    "orc_synth_pnc_rows": ([_u64, _u32, _u64, _u64, _u32, _u32, _vp], None),
    "orc_synth_orset": ([_u64, _u64, _u64, _u32, _u32, _u32, _vp], None),
    "orc_pnc_merge_dense": ([_u64, _u32, _u32, _vp, _vp, _u64, _vp, _vp, _vp], C.c_int),
    "orc_pnc_values_dense": ([_u64, _u32, _u32, _vp, _vp, _u64, _vp, _vp, _vp], C.c_int),
    "orc_pnc_apply_ops_dense": ([_u64, _u32, _u32, _vp, _vp, _u64, _vp, _vp, _vp, _vp], C.c_int),
    "orc_orset_merge": ([_vp, _u64, _vp, _u64, _vp, _u64, _vp, _u64, _vp, C.POINTER(_u64), _vp, C.POINTER(_u64)], C.c_int),
    "orc_orset_contains": ([_vp, _u64, _vp, _u64, _u64, _vp, _vp, _vp], C.c_int),
    "orc_orset_apply_ops": ([_vp, _u64, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.POINTER(_u64), _vp, C.POINTER(_u64)], C.c_int),
    "orc_orset_lookup_all": ([_vp, _u64, _vp, _u64, _u32, _vp, _u64], C.c_int64),
    "orc_bench_pnc_merge": ([_u64, _u32, _u64, _i32, _i32], C.c_double),
    "orc_bench_orset_merge": ([_u64, _u32, _u32, _u32, _u32, _u32, _u64, _i32, _i32], C.c_double),
    "orc_json_encode_pnc": ([_u64, _vp, _vp, _vp, _vp, _u32, _vp, _u64], C.c_int64),
    "orc_json_accepts_pnc": ([C.c_char_p, _u64, _u32], C.c_int),
    "orc_json_decode_orset": ([C.c_char_p, _u64, _vp, _u64], C.c_int64),
    "orc_sha256_batch": ([_u64, _vp, _vp, _vp], None),
    "orc_update_digests": ([_u64, _vp, _vp, _vp, _u64, _vp, _vp, _vp], None),
    "orc_bench_update_digests": ([_u64, _vp, _vp, _u64, _vp, _i32], C.c_double),
    "orc_pnc_apply_json": ([_u64, _u32, _u32, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _vp, C.POINTER(_u64)], C.c_int),
}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise FileNotFoundError(f"oracle not built: {LIB} (make -C oracle)")
        _lib = C.CDLL(str(LIB))
        for n, (a, r) in _SIGS.items():
            f = getattr(_lib, n)
            f.argtypes, f.restype = a, r
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(_vp)


def _dt(eb):
    return np.int32 if eb == 4 else np.int64


# ---- synthetic inputs (host copy of janus-crdt_amd/csrc/synth.hip) ----
def synth_pnc(seed: int, which: int, key0: int, n_keys: int, R: int, eb: int) -> np.ndarray:
    out = np.empty((n_keys, R), _dt(eb))
    lib().orc_synth_pnc_rows(seed, which, key0, n_keys, R, eb, _p(out))
    return out


def synth_orset(seed: int, first: int, n: int, elems_per_set: int, per_group: int, u0: int) -> np.ndarray:
    out = np.empty(n, REC_DTYPE)
    lib().orc_synth_orset(seed, first, n, elems_per_set, per_group, u0, _p(out))
    return out


# ---- PN-Counter ----
def pnc_merge(AP, AN, BP, BN, key_idx=None):
    """PNCounter.Merge of each received row into its key (dictionary-faithful); returns new (P, N)."""
    eb = AP.dtype.itemsize
    AP, AN = np.array(AP, copy=True), np.array(AN, copy=True)
    BP, BN = np.ascontiguousarray(BP), np.ascontiguousarray(BN)
    n_keys, R = AP.shape
    k = None if key_idx is None else np.ascontiguousarray(key_idx, np.uint32)
    n_rows = BP.shape[0]
    rc = lib().orc_pnc_merge_dense(n_keys, R, eb, _p(AP), _p(AN), n_rows, _p(k), _p(BP), _p(BN))
    assert rc == 0, rc
    return AP, AN


def pnc_values(P, N, key_idx=None):
    eb = P.dtype.itemsize
    P, N = np.ascontiguousarray(P), np.ascontiguousarray(N)
    n_keys, R = P.shape
    k = None if key_idx is None else np.ascontiguousarray(key_idx, np.uint32)
    n = n_keys if k is None else k.size
    out, ovf = np.empty(n, np.int64), np.empty(n, np.uint8)
    assert lib().orc_pnc_values_dense(n_keys, R, eb, _p(P), _p(N), n, _p(k), _p(out), _p(ovf)) == 0
    return out, ovf


def pnc_apply_ops(P, N, key, col, delta, is_n):
    eb = P.dtype.itemsize
    P, N = np.array(P, copy=True), np.array(N, copy=True)
    n_keys, R = P.shape
    key, col = np.ascontiguousarray(key, np.uint32), np.ascontiguousarray(col, np.uint32)
    delta, is_n = np.ascontiguousarray(delta, np.int64), np.ascontiguousarray(is_n, np.uint8)
    assert lib().orc_pnc_apply_ops_dense(n_keys, R, eb, _p(P), _p(N), key.size, _p(key), _p(col), _p(delta), _p(is_n)) == 0
    return P, N


# ---- OR-Set ----
def _recs(a):
    return np.ascontiguousarray(a, REC_DTYPE)


def canon(r) -> np.ndarray:
    """(key, tag_lo, tag_hi) rows of a record stream, in its stored (canonical, sorted) order."""
    r = _recs(r)
    return np.stack([r["key"], r["tag_lo"], r["tag_hi"]], 1) if r.size else np.zeros((0, 3), np.uint64)


def enum_view(r, rem: bool) -> np.ndarray:
    """The reference's enumeration order of one record stream (jg_tagrec.ord): (key, tag_lo, tag_hi) rows,
    sets ascending; within a set the Dictionary's elements — add stream: ascending elem id; tombstone
    stream: ascending smallest ord (first insertion into removeSet), then elem — each element's tags by
    (ord, tag); the null element's HashSet last."""
    r = _recs(r)
    if r.size == 0:
        return np.zeros((0, 3), np.uint64)
    key, lo, hi, o = r["key"], r["tag_lo"], r["tag_hi"], r["ord"]
    elem, sid = key & np.uint64(0xFFFFFFFF), key >> np.uint64(32)
    isnull = (elem == np.uint64(NULL_ELEM)).astype(np.uint8)
    if rem:
        uk, inv = np.unique(key, return_inverse=True)
        first = np.full(uk.size, np.iinfo(np.uint64).max, np.uint64)
        np.minimum.at(first, inv, o)
        grp = first[inv]
    else:
        grp = elem
    idx = np.lexsort((hi, lo, o, elem, grp, isnull, sid))
    return np.stack([key[idx], lo[idx], hi[idx]], 1)


def same_stream(g, e, rem: bool) -> bool:
    """Same records and the same enumeration order (ords may differ in value, not in order)."""
    return np.array_equal(canon(g), canon(e)) and np.array_equal(enum_view(g, rem), enum_view(e, rem))


def same_orset(ga, gr, ea, er) -> bool:
    return same_stream(ga, ea, False) and same_stream(gr, er, True)


def enum_is_canonical(r, rem: bool) -> bool:
    """O(n) check that a stream's enumeration order is its canonical (sorted) order: ords increase
    within every element and, for tombstones, elements' first ords increase within every set."""
    r = _recs(r)
    if r.size < 2:
        return True
    key, o = r["key"], r["ord"]
    same = key[1:] == key[:-1]
    if not np.all(~same | (o[1:] > o[:-1])):
        return False
    if not rem:
        return True
    head = np.concatenate([[True], ~same])
    hk, ho = key[head], o[head]  # each element's first record = its smallest ord (ords increase within it)
    hs = hk >> np.uint64(32)
    notnull = (hk[1:] & np.uint64(0xFFFFFFFF)) != np.uint64(NULL_ELEM)
    return bool(np.all((hs[1:] != hs[:-1]) | ~notnull | (ho[1:] > ho[:-1])))


def orset_merge(La, Lr, Ra, Rr):
    """ORSet.Merge per set (dictionary-faithful), exported canonically sorted."""
    La, Lr, Ra, Rr = map(_recs, (La, Lr, Ra, Rr))
    oa = np.empty(La.size + Ra.size, REC_DTYPE)
    orr = np.empty(Lr.size + Rr.size, REC_DTYPE)
    na, nr = _u64(), _u64()
    assert lib().orc_orset_merge(_p(La), La.size, _p(Lr), Lr.size, _p(Ra), Ra.size, _p(Rr), Rr.size,
                                 _p(oa), C.byref(na), _p(orr), C.byref(nr)) == 0
    return oa[: na.value], orr[: nr.value]


def orset_contains(A, Rm, sets, elems):
    A, Rm = _recs(A), _recs(Rm)
    s, e = np.ascontiguousarray(sets, np.uint32), np.ascontiguousarray(elems, np.uint32)
    out = np.empty(s.size, np.uint8)
    assert lib().orc_orset_contains(_p(A), A.size, _p(Rm), Rm.size, s.size, _p(s), _p(e), _p(out)) == 0
    return out


def orset_apply_ops(A, Rm, sets, elems, ops, tag_lo, tag_hi):
    """ORSet.Add/Remove/Clear in order; returns (adds, tombstones, results)."""
    A, Rm = _recs(A), _recs(Rm)
    s, e = np.ascontiguousarray(sets, np.uint32), np.ascontiguousarray(elems, np.uint32)
    o = np.ascontiguousarray(ops, np.uint8)
    lo, hi = np.ascontiguousarray(tag_lo, np.uint64), np.ascontiguousarray(tag_hi, np.uint64)
    res = np.empty(s.size, np.uint8)
    oa = np.empty(A.size + s.size, REC_DTYPE)
    orr = np.empty(Rm.size + A.size + s.size, REC_DTYPE)
    na, nr = _u64(), _u64()
    assert lib().orc_orset_apply_ops(_p(A), A.size, _p(Rm), Rm.size, s.size, _p(s), _p(e), _p(o), _p(lo), _p(hi), _p(res),
                                     _p(oa), C.byref(na), _p(orr), C.byref(nr)) == 0
    return oa[: na.value], orr[: nr.value], res


def orset_lookup_all(A, Rm, set_id, cap=1 << 16):
    A, Rm = _recs(A), _recs(Rm)
    out = np.empty(cap, np.uint32)
    n = lib().orc_orset_lookup_all(_p(A), A.size, _p(Rm), Rm.size, set_id, _p(out), cap)
    assert n >= 0
    return out[:n]


# ---- CPU baseline ----
def bench_pnc_merge(n_keys, R, seed, threads=1, reps=5) -> float:
    return lib().orc_bench_pnc_merge(n_keys, R, seed, threads, reps)


def bench_orset_merge(n_sets, E, a, ov, t, tov, seed, threads=1, reps=5) -> float:
    return lib().orc_bench_orset_merge(n_sets, E, a, ov, t, tov, seed, threads, reps)


# ---- state-message wire codec (oracle/json.hpp) ----
GUID_DTYPE = np.dtype([("lo", "<u8"), ("hi", "<u8")])


def json_encode_pnc(lo, hi, pv, nv, eb: int) -> bytes:
    """PNCounterMsg.Encode of a message whose pVector/nVector hold Guids (lo[i], hi[i]) in order."""
    lo, hi = np.ascontiguousarray(lo, np.uint64), np.ascontiguousarray(hi, np.uint64)
    pv, nv = np.ascontiguousarray(pv, np.int64), np.ascontiguousarray(nv, np.int64)
    buf = C.create_string_buffer(64 + 128 * len(lo))
    n = lib().orc_json_encode_pnc(len(lo), _p(lo), _p(hi), _p(pv), _p(nv), eb, buf, len(buf))
    assert n >= 0
    return buf.raw[:n]


def json_accepts_pnc(payload: bytes, eb: int) -> bool:
    return bool(lib().orc_json_accepts_pnc(payload, len(payload), eb))


def pnc_apply_json(P, N, cols, ncols, key_idx, msgs, eb):
    """Oracle stable-apply loop over encoded states; returns (P, N, cols, ncols, bad_msg, rc).
    cols is a GUID_DTYPE [n_keys x R] array."""
    P, N = P.copy(), N.copy()
    cols, ncols = cols.copy(), np.ascontiguousarray(ncols, np.uint32).copy()
    n_keys, R = P.shape
    k = np.ascontiguousarray(key_idx, np.uint32)
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    data = b"".join(msgs) + b"\0"
    bad = _u64(0)
    rc = lib().orc_pnc_apply_json(n_keys, R, eb, _p(P), _p(N), _p(cols), _p(ncols), len(msgs), _p(k), _p(off), data, C.byref(bad))
    return P, N, cols, ncols, (None if bad.value == 2**64 - 1 else bad.value), rc


def json_decode_orset(payload: bytes):
    """ORSetMsg.Decode of one payload in Merge's walk order: list of (side, is_null, name bytes, [(lo, hi)]),
    or None if Decode throws."""
    n = lib().orc_json_decode_orset(payload, len(payload), None, 0)
    if n < 0:
        return None
    buf = np.empty(max(1, n), np.uint8)
    assert lib().orc_json_decode_orset(payload, len(payload), _p(buf), n) == n
    raw, at, out = buf.tobytes()[:n], 0, []
    while at < n:
        side, is_null = raw[at], raw[at + 1]
        ln = int.from_bytes(raw[at + 2:at + 6], "little")
        name = raw[at + 6:at + 6 + ln]
        at += 6 + ln
        nt = int.from_bytes(raw[at:at + 4], "little")
        at += 4
        tags = np.frombuffer(raw[at:at + 16 * nt], np.uint64).reshape(nt, 2) if nt else np.zeros((0, 2), np.uint64)
        at += 16 * nt
        out.append((side, bool(is_null), name, [(int(a), int(b)) for a, b in tags]))
    return out


def orset_apply_json(set_ids, msgs, names=None, state=None):
    """The stable-apply loop over ORSetMsg payloads (SafeCRDT.ApplyUpdateStable -> Decode -> Merge in
    commit order) with element strings interned per set at first insertion (ids never reused).
    names: {set: {name bytes: id}} carried between calls (updated in place), with "next" ids in
    names[("next", set)].  state: {(side, key): {tag: None}} — the Dictionaries and HashSets in their
    insertion order (Merge appends new keys and UnionWith appends new tags, ORSet.cs:255-282) — carried
    between calls (updated in place) when given.  Returns (add records, tombstone records, first bad
    message or None, its code: "EINVAL" for a Decode error, "ESTATE" for an element's empty tag set): the whole
    state, sorted, ord = the record's position in its stream's enumeration."""
    names = {} if names is None else names
    state = {} if state is None else state
    bad, code = None, None
    for m, (sid, p) in enumerate(zip(set_ids, msgs)):
        d = json_decode_orset(p)
        if d is None:
            bad, code = m, "EINVAL"
            break
        if any(not is_null and not tags for side, is_null, _, tags in d):  # an element with an empty tag set
            bad, code = m, "ESTATE"
            break
        tab = names.setdefault(int(sid), {})
        for side, is_null, name, tags in d:
            if is_null:
                eid = NULL_ELEM
            else:
                if name not in tab:
                    tab[name] = names.get(("next", int(sid)), 0)
                    names[("next", int(sid))] = tab[name] + 1
                eid = tab[name]
            hs = state.setdefault((side, int(sid) << 32 | eid), {})
            for t in tags:
                hs.setdefault(t)
    out = ([], [])
    for (side, key), hs in state.items():  # dict order = first insertion, across sets
        for lo, hi in hs:
            out[side].append((key, lo, hi, len(out[side])))
    mk = lambda v: np.sort(np.array(v, dtype=REC_DTYPE), order=["key", "tag_lo", "tag_hi"]) if v else np.zeros(0, REC_DTYPE)
    return mk(out[0]), mk(out[1]), bad, code


# ---- UpdateMessage.ComputeDigest (oracle/digest.hpp) ----
def _pack(msgs):
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([0 if m is None else len(m) for m in msgs], dtype=np.uint64) if msgs else []
    data = np.frombuffer(b"".join(b"" if m is None else m for m in msgs) + b"\0", np.uint8)
    return data, off


def sha256_batch(msgs) -> np.ndarray:
    data, off = _pack(msgs)
    out = np.zeros((len(msgs), 32), np.uint8)
    lib().orc_sha256_batch(len(msgs), _p(off), _p(data), _p(out))
    return out


def update_digests(msgs, first):
    """(digests u8[n_updates, 32], per-message u8[n, 32]) for updates msgs[first[u]:first[u+1]]."""
    data, off = _pack(msgs)
    is_null = np.array([m is None for m in msgs] or [False], np.uint8)
    first = np.ascontiguousarray(first, np.uint64)
    nu = first.size - 1
    dig = np.zeros((max(nu, 0), 32), np.uint8)
    md = np.zeros((len(msgs), 32), np.uint8)
    lib().orc_update_digests(len(msgs), _p(off), _p(data), _p(is_null), nu, _p(first), _p(md), _p(dig))
    return dig, md
