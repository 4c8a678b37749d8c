"""Seeded PNCounterMsg wire payloads for the JSON-path tests (test infrastructure).

Payloads are written the way System.Text.Json serializes PNCounterMsg (PNCounters.cs:46-49):
{"pVector":{"<guid D>":int,...},"nVector":{...}}; tests/test_json.py checks this writer against the
oracle's restatement (oracle/json.hpp) byte for byte.  `uuid.UUID(bytes_le=...)` prints a Guid's 16
bytes in .NET's "D" layout (the first three groups little-endian).
"""
from __future__ import annotations

import uuid

import numpy as np


def guid_d(lo: int, hi: int) -> str:
    return str(uuid.UUID(bytes_le=int(lo).to_bytes(8, "little") + int(hi).to_bytes(8, "little")))


def encode_pnc(guids, pv, nv) -> bytes:
    """guids: list of (lo, hi); pv / nv: values (None = entry absent from that vector)."""
    p = ",".join(f'"{guid_d(*g)}":{int(v)}' for g, v in zip(guids, pv) if v is not None)
    n = ",".join(f'"{guid_d(*g)}":{int(v)}' for g, v in zip(guids, nv) if v is not None)
    return ('{"pVector":{' + p + '},"nVector":{' + n + "}}").encode()


def random_guids(rng, n):
    return [(int(a), int(b)) for a, b in zip(rng.integers(1, 2**63, n, dtype=np.uint64), rng.integers(0, 2**63, n, dtype=np.uint64))]


class Cluster:
    """Reference-shaped PN-Counter states: key k has a pool of replica Guids (its per-node instances);
    a node's state of k lists the replicas it has seen, in the order it first saw them, with
    non-decreasing values (what GetLastSynchronizedUpdate of a real node would carry)."""

    def __init__(self, rng, n_keys, pool, eb, stable):
        self.rng, self.eb = rng, eb
        self.pool = [random_guids(rng, pool) for _ in range(n_keys)]
        self.stable = stable  # key -> the stable instance's own Guid (column 0)
        self.seen = [[] for _ in range(n_keys)]  # union order in which replicas appear in messages
        self.P = [dict() for _ in range(n_keys)]
        self.N = [dict() for _ in range(n_keys)]
        self.hi = 2**31 - 1 if eb == 4 else 2**62

    def message(self, k, grow=0.3, max_step=None):
        rng = self.rng
        seen = self.seen[k]
        if not seen or (len(seen) < len(self.pool[k]) and rng.random() < grow):
            g = self.pool[k][len(seen)]
            seen.append(g)
            self.P[k][g] = 0
            self.N[k][g] = 0
        step = max_step or (self.hi // 1000)
        for g in seen:
            if rng.random() < 0.5:
                self.P[k][g] = min(self.hi, self.P[k][g] + int(rng.integers(0, step)))
            if rng.random() < 0.2:
                self.N[k][g] = min(self.hi, self.N[k][g] + int(rng.integers(0, step)))
        # a node only knows a prefix of the replicas (it may lag behind)
        m = int(rng.integers(1, len(seen) + 1))
        gs = seen[:m]
        return encode_pnc(gs, [self.P[k][g] for g in gs], [self.N[k][g] for g in gs])


G1 = (0x1122334455667788, 0x99AABBCCDDEEFF00)
G2 = (0x0102030405060708, 0x0A0B0C0D0E0F1011)
_A, _B = guid_d(*G1), guid_d(*G2)

# (payload, accepted at int32, accepted at int64): the wire contract of oracle/json.hpp.
CONTRACT = [
    (encode_pnc([G1, G2], [5, 0], [1, 2]), True, True),
    (b'{"pVector":{},"nVector":{}}', True, True),
    (f' \t{{ "nVector" : {{ "{_A}" : 3 }} ,\r\n "pVector":{{"{_B}":4,"{_A.upper()}":-7}} }}\n'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":-2147483648}},"nVector":{{"{_A}":2147483647}}}}'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":-0}},"nVector":{{}}}}'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":2147483648}},"nVector":{{}}}}'.encode(), False, True),
    (f'{{"pVector":{{"{_A}":-9223372036854775808}},"nVector":{{}}}}'.encode(), False, True),
    (f'{{"pVector":{{"{_A}":9223372036854775808}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":99999999999999999999999}},"nVector":{{}}}}'.encode(), False, False),
    (b'{"pVector":{}}', False, False),
    (b'{"nVector":{}}', False, False),
    (b'{}', False, False),
    (b'', False, False),
    (b'   ', False, False),
    (b'{"pVector":null,"nVector":{}}', False, False),
    (b'{"pVector":{},"nVector":{},"x":1}', False, False),
    (b'{"pVector":{},"nVector":{},"pVector":{}}', False, False),
    (b'{"pvector":{},"nVector":{}}', False, False),
    (b'{"p\\u0056ector":{},"nVector":{}}', False, False),
    (f'{{"pVector":{{"{_A}":1,"{_A}":2}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":1,"{_A.upper()}":2}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":1}},"nVector":{{"{_A}":1,"{_B}":0,"{_A}":3}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":01}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":1.0}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":1e3}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":+1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":-}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":"1"}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A[:-1]}":1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}0":1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A.replace("-", "", 1)}-":1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A[:3]}g{_A[4:]}":1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{{{_A}}}":1}},"nVector":{{}}}}'.encode(), False, False),
    (f'{{"pVector":{{"{_A}":1,}},"nVector":{{}}}}'.encode(), False, False),
    (b'{"pVector":{},"nVector":{},}', False, False),
    (b'{"pVector":{},"nVector":{}} x', False, False),
    (b'{"pVector":{},"nVector":{}}}', False, False),
    (b'{"pVector":{},"nVector":{}', False, False),
    (b'{"pVector":[],"nVector":{}}', False, False),
    (b'\xef\xbb\xbf{"pVector":{},"nVector":{}}', False, False),
]
