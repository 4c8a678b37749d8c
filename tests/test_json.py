"""Wire codec of the state messages on the CPU: the test writer against the
oracle's System.Text.Json restatement (oracle/json.hpp), the accepted decode contract, and the
oracle's decode-and-merge apply loop.  The reference pins the codec only by round trip
(PNCounterTests.cs:46-66, ORSetTests.cs:453-474 — transcribed in oracle/test_kat.cpp); the exact
byte layout is parity unpinned (no .NET here), restated from System.Text.Json 6.0's documented
defaults."""
import numpy as np
import pytest

import oracle_ref as orc
from jsongen import CONTRACT, G1, G2, Cluster, encode_pnc, guid_d, random_guids


def test_guid_d_layout():
    # Guid.ToString("D") of bytes 88 77 66 55 44 33 22 11 00 FF EE DD CC BB AA 99
    assert guid_d(*G1) == "55667788-3344-1122-00ff-eeddccbbaa99"


@pytest.mark.parametrize("eb", [4, 8])
def test_writer_matches_oracle_encoder(eb):
    rng = np.random.default_rng(eb)
    for n in (0, 1, 5, 64):
        gs = random_guids(rng, n)
        lo, hi = [g[0] for g in gs], [g[1] for g in gs]
        lim = 2**31 if eb == 4 else 2**63
        pv = rng.integers(-lim, lim, n, dtype=np.int64)
        nv = rng.integers(-lim, lim, n, dtype=np.int64)
        assert orc.json_encode_pnc(lo, hi, pv, nv, eb) == encode_pnc(gs, pv, nv)


@pytest.mark.parametrize("i", range(len(CONTRACT)))
def test_decode_contract(i):
    payload, ok4, ok8 = CONTRACT[i]
    assert orc.json_accepts_pnc(payload, 4) == ok4, payload
    assert orc.json_accepts_pnc(payload, 8) == ok8, payload


def _empty_store(n_keys, R, eb, stable):
    dt = np.int32 if eb == 4 else np.int64
    P = np.zeros((n_keys, R), dt)
    N = np.zeros((n_keys, R), dt)
    cols = np.zeros((n_keys, R), orc.GUID_DTYPE)
    ncols = np.zeros(n_keys, np.uint32)
    for k, g in enumerate(stable):
        cols[k, 0] = g
        ncols[k] = 1
    return P, N, cols, ncols


def _py_apply(stable, keys, msgs):
    """Plain-Python Decode + Merge (PNCounters.cs:131-144) with insertion-ordered dicts."""
    import json
    import uuid
    P = [{g: 0} for g in stable]
    N = [{g: 0} for g in stable]
    for k, m in zip(keys, msgs):
        d = json.loads(m)
        for vec, st in (("pVector", P[k]), ("nVector", N[k])):
            for s, v in d[vec].items():
                b = uuid.UUID(s).bytes_le
                g = (int.from_bytes(b[:8], "little"), int.from_bytes(b[8:], "little"))
                st[g] = max(st.get(g, 0), v)
    return P, N


@pytest.mark.parametrize("eb", [4, 8])
def test_oracle_apply_json_matches_dict_semantics(eb):
    """The oracle's dense apply loop = per-key ordered dictionaries fed Decode(payload) in order."""
    rng = np.random.default_rng(3 + eb)
    n_keys, R = 6, 8
    stable = random_guids(rng, n_keys)
    cl = Cluster(rng, n_keys, 6, eb, stable)
    keys = rng.integers(0, n_keys, 300).astype(np.uint32)
    msgs = [cl.message(int(k)) for k in keys]
    P, N, cols, ncols = _empty_store(n_keys, R, eb, stable)
    P2, N2, cols2, ncols2, bad, rc = orc.pnc_apply_json(P, N, cols, ncols, keys, msgs, eb)
    assert rc == 0 and bad is None
    eP, eN = _py_apply(stable, keys, msgs)
    for k in range(n_keys):
        assert int(ncols2[k]) == len(eP[k])
        for c, (g, v) in enumerate(eP[k].items()):
            assert (int(cols2[k, c]["lo"]), int(cols2[k, c]["hi"])) == g
            assert P2[k, c] == v and N2[k, c] == eN[k][g]


def test_oracle_apply_json_stops_at_bad_message():
    rng = np.random.default_rng(4)
    stable = random_guids(rng, 2)
    P, N, cols, ncols = _empty_store(2, 4, 4, stable)
    msgs = [encode_pnc([G1], [5], [0]), b'{"pVector":{}}', encode_pnc([G2], [9], [0])]
    P2, N2, cols2, ncols2, bad, rc = orc.pnc_apply_json(P, N, cols, ncols, [0, 0, 1], msgs, 4)
    assert bad == 1 and rc == 0
    assert P2[0, 1] == 5 and ncols2[1] == 1  # message 0 applied, message 2 not
