"""Seeded random CRDT states for parity tests (shared by the test modules)."""
import numpy as np

from oracle_ref import NULL_ELEM, REC_DTYPE


def recs(keys, lo, hi, rng=None):
    """Records sorted by (key, tag_lo, tag_hi), duplicate-free; ord = a random arrival order (rng), else
    the canonical order."""
    r = np.zeros(len(keys), REC_DTYPE)
    r["key"], r["tag_lo"], r["tag_hi"] = keys, lo, hi
    r = np.unique(r)
    r["ord"] = rng.permutation(r.size).astype(np.uint64) if rng is not None else np.arange(r.size, dtype=np.uint64)
    return r


def random_orset_pair(rng, n_sets=8, n_elems=6, pool=12, p_l=0.5, p_r=0.5, p_rem=0.4, p_full_rem=0.2,
                      null_elem=True, tag_bits=64):
    """Local and received OR-Set states over the same keyspace.  Each (set, elem) group has a pool of
    Guid tags; each side observed a random subset of it and tombstoned a subset of what it observed
    (sometimes all of it, so elements really disappear).  Returns (La, Lr, Ra, Rr)."""
    elems = list(range(n_elems)) + ([NULL_ELEM] if null_elem else [])
    out = {s: ([], [], [], []) for s in "LR"}
    mask = (1 << tag_bits) - 1 if tag_bits < 64 else (1 << 64) - 1
    for s_id in range(n_sets):
        for e in elems:
            key = (s_id << 32) | e
            lo = rng.integers(0, 1 << 63, pool, dtype=np.uint64) & np.uint64(mask)
            hi = rng.integers(0, 1 << 63, pool, dtype=np.uint64)
            for side, p in (("L", p_l), ("R", p_r)):
                seen = np.nonzero(rng.random(pool) < p)[0]
                if len(seen) == 0:
                    continue
                if rng.random() < p_full_rem:
                    dead = seen
                else:
                    dead = seen[rng.random(len(seen)) < p_rem]
                ka, kr = out[side][0], out[side][1]
                ka.extend((key, lo[i], hi[i]) for i in seen)
                kr.extend((key, lo[i], hi[i]) for i in dead)
    res = []
    for side in "LR":
        for lst in out[side][:2]:
            if lst:
                a = np.array(lst, dtype=object)
                res.append(recs(a[:, 0].astype(np.uint64), a[:, 1].astype(np.uint64), a[:, 2].astype(np.uint64), rng))
            else:
                res.append(np.empty(0, REC_DTYPE))
    return tuple(res)  # La, Lr, Ra, Rr


def random_pnc(rng, n_keys, R, eb, p_absent=0.3, lo=None, hi=None, absent=True):
    dt = np.int32 if eb == 4 else np.int64
    info = np.iinfo(dt)
    lo = info.min + 1 if lo is None else lo
    hi = info.max if hi is None else hi
    a = rng.integers(lo, hi, (n_keys, R), dtype=dt, endpoint=True)
    if absent:
        a[rng.random((n_keys, R)) < p_absent] = info.min
    return a
