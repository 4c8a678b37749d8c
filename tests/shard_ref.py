"""Host restatement of the cross-shard routing rule (csrc/route.hip) — TEST-ONLY, the checker for the
device route kernels and the reference the gloo tests route with.

Owner of global key k (PN-Counter row / OR-Set set id) = k % world; its local key there = k // world.
A route is a STABLE partition by owner: each destination's run keeps batch order.
"""
import numpy as np

from oracle_ref import REC_DTYPE


def owner_of_key(k, world):
    """The rank that owns global key k (csrc/jg_internal.hpp owner_of_key)."""
    return int(k) % world


def local_of_key(k, world):
    """Global key k's local key on its owner (csrc/jg_internal.hpp local_of_key)."""
    return int(k) // world


def route_rows(keys, P, N, world):
    """-> (counts[world], local keys, P, N) grouped by destination rank, batch order within a group."""
    keys = np.asarray(keys, np.uint32)
    owner = keys % world
    order = np.argsort(owner, kind="stable")
    counts = np.bincount(owner, minlength=world).astype(np.uint64)
    return counts, (keys[order] // world).astype(np.uint32), np.asarray(P)[order], np.asarray(N)[order]


def route_records(recs, world):
    """-> (counts[world], records grouped by destination with set ids rewritten to set // world)."""
    recs = np.ascontiguousarray(recs, REC_DTYPE)
    sets = recs["key"] >> np.uint64(32)
    owner = (sets % np.uint64(world)).astype(np.int64)
    order = np.argsort(owner, kind="stable")
    out = recs[order].copy()
    s = sets[order]
    out["key"] = ((s // np.uint64(world)) << np.uint64(32)) | (out["key"] & np.uint64(0xFFFFFFFF))
    return np.bincount(owner, minlength=world).astype(np.uint64), out


def shard_rows(P, world, rank):
    """Rows of a global [keys x R] array owned by `rank`, in local-key order."""
    return np.asarray(P)[rank::world]


def shard_records(recs, world, rank):
    """Records of a global stream owned by `rank`, set ids made local (stays sorted)."""
    counts, out = route_records(recs, world)
    lo = int(counts[:rank].sum())
    return out[lo: lo + int(counts[rank])]
