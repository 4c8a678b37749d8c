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
    # System.Text.Json past the compact form (oracle/json.hpp, round 6): unknown members skipped, a repeated member's
    # last occurrence, a repeated key's last value at its first place, escaped names and keys, MaxDepth 64
    (b'{"pVector":{},"nVector":{},"x":1}', True, True),
    (b'{"pVector":{},"nVector":{},"pVector":{}}', True, True),
    (b'{"pvector":{},"nVector":{}}', False, False),
    (b'{"p\\u0056ector":{},"nVector":{}}', True, True),
    (f'{{"pVector":{{"{_A}":1,"{_A}":2}},"nVector":{{}}}}'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":1,"{_A.upper()}":2}},"nVector":{{}}}}'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":1,"{_B}":2}},"nVector":{{"{_A}":1,"{_B}":0,"{_A}":3}}}}'.encode(), True, True),
    (f'{{"pVector":{{"\\u0031{_B[1:]}":5}},"nVector":{{}}}}'.encode(), True, True),
    (f'{{"zz":{{"a":[1,-2.5e+3,{{"b":null}},true,false],"c":"\\u00e9x"}},"pVector":{{"{_A}":1}},"nVector":{{}}}}'.encode(), True, True),
    (f'{{"pVector":null,"nVector":{{}},"pVector":{{"{_A}":9}}}}'.encode(), True, True),
    (f'{{"pVector":{{"{_A}":9}},"nVector":{{}},"pVector":null}}'.encode(), False, False),
    (b'{"x":' + b'[' * 63 + b']' * 63 + b',"pVector":{},"nVector":{}}', True, True),
    (b'{"x":' + b'[' * 64 + b']' * 64 + b',"pVector":{},"nVector":{}}', False, False),
    (b'{"x":[1,],"pVector":{},"nVector":{}}', False, False),
    (b'{"x":01,"pVector":{},"nVector":{}}', False, False),
    (b'{"x":"\\q","pVector":{},"nVector":{}}', False, False),
    (b'{"x":nul,"pVector":{},"nVector":{}}', False, False),
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


# ---- ORSetMsg<string> payloads (ORSet.cs:56-69) ------------------------------------------------------
_ORSET_MEMBERS = ("addSet", "removeSet", "nullAddGuid", "nullRemoveGuid")


def json_str(s: str, mode: str = "default") -> str:
    """A JSON string literal for s.  default: JavaScriptEncoder.Default's shape (printable ASCII except
    " & ' + < > ` \\ kept, every other UTF-16 unit as \\uXXXX); raw: UTF-8 kept, only what JSON requires
    escaped; all: every character as \\uXXXX (surrogate pairs above U+FFFF)."""
    out = []
    for ch in s:
        c = ord(ch)
        units = [c] if c < 0x10000 else [0xD800 | (c - 0x10000) >> 10, 0xDC00 | ((c - 0x10000) & 0x3FF)]
        if mode == "all":
            out.extend(f"\\u{u:04X}" for u in units)
        elif mode == "raw":
            if ch == '"':
                out.append('\\"')
            elif ch == "\\":
                out.append("\\\\")
            elif c < 0x20:
                out.append({8: "\\b", 9: "\\t", 10: "\\n", 12: "\\f", 13: "\\r"}.get(c, f"\\u{c:04x}"))
            else:
                out.append(ch)
        else:
            if 0x20 <= c < 0x7F and ch not in "\"&'+<>`\\":
                out.append(ch)
            elif ch == "\\":
                out.append("\\\\")
            else:
                out.extend(f"\\u{u:04X}" for u in units)
    return '"' + "".join(out) + '"'


def encode_orset(add, rem, nadd=(), nrem=(), mode="default", ws="", order=None, upper=False) -> bytes:
    """add / rem: list of (element str, [(lo, hi) tags]); nadd / nrem: null tag lists.  ws is put
    between tokens; order permutes the four members; upper prints Guid hex upper-case."""
    def g(t):
        s = guid_d(*t)
        return json_str(s.upper() if upper else s, "raw" if mode == "all" else mode) if mode != "all" else json_str(s, "all")

    def tags(ts):
        return "[" + ws + ("," + ws).join(g(t) for t in ts) + ws + "]"

    def dmap(m):
        return "{" + ws + ("," + ws).join(json_str(e, mode) + ws + ":" + ws + tags(ts) for e, ts in m) + ws + "}"

    vals = {"addSet": dmap(add), "removeSet": dmap(rem), "nullAddGuid": tags(nadd), "nullRemoveGuid": tags(nrem)}
    names = order or _ORSET_MEMBERS
    body = ("," + ws).join(json_str(k, "raw") + ws + ":" + ws + vals[k] for k in names)
    return (ws + "{" + ws + body + ws + "}" + ws).encode()


class ORSetCluster:
    """Valid ORSetMsg states of many sets: each set has a growing pool of element strings (ASCII words,
    escapes-needing text, non-BMP characters, the empty string) and per-element tag pools; a state lists
    a random subset of the set's elements with non-empty add tag sets, tombstones drawn from them, and
    optional null tag sets."""

    WORDS = ["a", "bb", "x y", "q\"uote", "back\\slash", "tab\tnl\n", "café", "中文", "emoji\U0001F600", "", "<&'+>`",
             "ctl\u0001", "ÿĀ", "z" * 40]

    def __init__(self, rng, n_sets, grow=0.3):
        self.rng, self.grow = rng, grow
        self.elems = [[] for _ in range(n_sets)]
        self.tags = [{} for _ in range(n_sets)]
        self.null_tags = [random_guids(rng, 3) for _ in range(n_sets)]

    def _new_elem(self, s):
        rng = self.rng
        k = len(self.elems[s])
        base = self.WORDS[int(rng.integers(0, len(self.WORDS)))]
        e = base + ("" if k == 0 and base == "" else f"#{k}")
        self.elems[s].append(e)
        self.tags[s][e] = random_guids(rng, int(rng.integers(1, 4)))
        return e

    def state(self, s):
        rng = self.rng
        if not self.elems[s] or rng.random() < self.grow:
            self._new_elem(s)
        es = self.elems[s]
        pick = [e for e in es if rng.random() < 0.7] or [es[-1]]
        rng.shuffle(pick)
        add = [(e, [t for t in self.tags[s][e] if rng.random() < 0.8] or self.tags[s][e][:1]) for e in pick]
        rem = [(e, ts[: int(rng.integers(1, len(ts) + 1))]) for e, ts in add if rng.random() < 0.3]  # Remove copies a non-empty set
        nadd = self.null_tags[s][: int(rng.integers(0, 4))]
        nrem = nadd[: int(rng.integers(0, len(nadd) + 1))]
        return add, rem, nadd, nrem
