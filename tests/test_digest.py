"""UpdateMessage.ComputeDigest (BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:32-55).

CPU tests pin the oracle (oracle/digest.hpp) against hashlib and the committed golden fixture
(tests/golden/update_digests.npz, made by hashlib alone); GPU tests compare the HIP kernels
(jg_update_digests / jg_wave_update_digests) byte for byte with both.  Integer/byte work: bit-exact."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

import oracle_ref as orc

GOLD = Path(__file__).resolve().parent / "golden" / "update_digests.npz"


def rent_length(n: int) -> int:  # .NET 6 ArrayPool<byte>.Shared.Rent(n).Length
    return 0 if n == 0 else (n if n > 1 << 20 else max(16, 1 << (n - 1).bit_length()))


def py_digest(msgs) -> bytes:
    buf = bytearray(rent_length(32 * len(msgs)))
    for i, m in enumerate(msgs):
        if m is not None:
            buf[32 * i:32 * i + 32] = hashlib.sha256(m).digest()
    return hashlib.sha256(bytes(buf)).digest()


def golden():
    z = np.load(GOLD)
    data, off, nul = z["data"].tobytes(), z["off"], z["is_null"]
    msgs = [None if nul[i] else data[off[i]:off[i + 1]] for i in range(off.size - 1)]
    return msgs, z["first"], z["digest"], z["msg_digest"]


def random_msgs(rng, n, lo=0, hi=700, null_every=0):
    out = []
    for i in range(n):
        if null_every and i % null_every == null_every - 1:
            out.append(None)
        else:
            out.append(rng.integers(0, 256, int(rng.integers(lo, hi + 1))).astype(np.uint8).tobytes())
    return out


# ---------------------------------------------------------------- CPU: the oracle
def test_oracle_sha256_matches_hashlib():
    rng = np.random.default_rng(1)
    msgs = [bytes(rng.integers(0, 256, n).astype(np.uint8)) for n in list(range(0, 200)) + [1000, 4097, 70001]]
    got = orc.sha256_batch(msgs)
    for m, g in zip(msgs, got):
        assert g.tobytes() == hashlib.sha256(m).digest()


def test_oracle_against_golden():
    msgs, first, digest, msg_digest = golden()
    d, md = orc.update_digests(msgs, first)
    assert np.array_equal(d, digest)
    assert np.array_equal(md, msg_digest)


def test_oracle_rent_boundary():
    # 32768 payloads = exactly 2^20 digest bytes (pooled bucket); 32769 -> above the pool (exact length)
    rng = np.random.default_rng(2)
    msgs = random_msgs(rng, 32769, 0, 8)
    for cnt in (32768, 32769):
        d, _ = orc.update_digests(msgs[:cnt], [0, cnt])
        assert d[0].tobytes() == py_digest(msgs[:cnt])


# ---------------------------------------------------------------- GPU: the HIP kernels
@pytest.mark.gpu
def test_gpu_golden(ctx):
    import janus_gpu as jg
    msgs, first, digest, msg_digest = golden()
    d, md = jg.update_digests(ctx, msgs, first, msg_digests=True)
    assert np.array_equal(d, digest)
    assert np.array_equal(md, msg_digest)


@pytest.mark.gpu
def test_gpu_every_length_and_alignment(ctx):
    # every length 0..300 (all padding cases: 55/56/63/64/119/120 ...) at every start offset mod 16
    import janus_gpu as jg
    rng = np.random.default_rng(3)
    msgs = []
    for n in range(0, 301):
        msgs.append(rng.integers(0, 256, n).astype(np.uint8).tobytes())
        msgs.append(rng.integers(0, 256, int(rng.integers(0, 16))).astype(np.uint8).tobytes())  # shifts the next start
    d, md = jg.update_digests(ctx, msgs, [0, len(msgs)], msg_digests=True)
    for m, g in zip(msgs, md):
        assert g.tobytes() == hashlib.sha256(m).digest(), len(m)
    assert d[0].tobytes() == py_digest(msgs)


@pytest.mark.gpu
def test_gpu_updates_nulls_and_empty(ctx):
    import janus_gpu as jg
    rng = np.random.default_rng(4)
    msgs = random_msgs(rng, 2600, 0, 1500, null_every=7)
    sizes = [0, 1, 1, 2, 3, 4, 5, 31, 32, 33, 64, 1000, 0, 1424]
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    assert first[-1] == len(msgs)
    d, md = jg.update_digests(ctx, msgs, first, msg_digests=True)
    ed, emd = orc.update_digests(msgs, first)
    assert np.array_equal(md, emd)
    assert np.array_equal(d, ed)
    for u in range(len(sizes)):
        assert d[u].tobytes() == py_digest(msgs[first[u]:first[u + 1]])


@pytest.mark.gpu
def test_gpu_sha256_batch_and_second_level_of(ctx):
    """jg_sha256_batch = hashlib per payload; jg_update_digests_of over those hashes = jg_update_digests over the
    payloads (nulls zeroed whatever their rows hold, rent boundaries, empty updates) — the producer path hashes
    each snapshot where it was encoded and takes the second level from the hashes (host/janus_host.cpp DigestsOf)."""
    import janus_gpu as jg
    rng = np.random.default_rng(14)
    msgs = random_msgs(rng, 3000, 0, 1500, null_every=9)
    h = jg.sha256_batch(ctx, [b"" if m is None else m for m in msgs])
    for i in range(0, 3000, 37):
        assert h[i].tobytes() == hashlib.sha256(b"" if msgs[i] is None else msgs[i]).digest()
    sizes = [0, 1, 2, 31, 32, 33, 1000, 0, 1901]
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    assert first[-1] == len(msgs)
    is_null = np.array([m is None for m in msgs], np.uint8)
    got = jg.update_digests_of(ctx, h, first, is_null)
    want = jg.update_digests(ctx, msgs, first)
    assert np.array_equal(got, want)
    for u in range(len(sizes)):
        assert got[u].tobytes() == py_digest(msgs[first[u]:first[u + 1]])
    assert jg.sha256_batch(ctx, []).shape == (0, 32)
    assert jg.update_digests_of(ctx, np.zeros((0, 32), np.uint8), [0]).shape == (0, 32)


@pytest.mark.gpu
def test_gpu_no_updates_and_all_null(ctx):
    import janus_gpu as jg
    d = jg.update_digests(ctx, [], [0])
    assert d.shape == (0, 32)
    d = jg.update_digests(ctx, [None, None, None], [0, 3])
    assert d[0].tobytes() == hashlib.sha256(bytes(128)).digest()
    d = jg.update_digests(ctx, [b""], [0, 1])
    assert d[0].tobytes() == hashlib.sha256(hashlib.sha256(b"").digest()).digest()


@pytest.mark.gpu
def test_gpu_rent_boundary(ctx):
    import janus_gpu as jg
    rng = np.random.default_rng(5)
    msgs = random_msgs(rng, 32769, 0, 40)
    d = jg.update_digests(ctx, msgs, [0, 32768, 32768, 32769])  # second update empty
    assert d[0].tobytes() == py_digest(msgs[:32768])
    assert d[1].tobytes() == hashlib.sha256(b"").digest()
    assert d[2].tobytes() == py_digest(msgs[32768:])
    d = jg.update_digests(ctx, msgs, [0, 32769])
    assert d[0].tobytes() == py_digest(msgs)


@pytest.mark.gpu
def test_gpu_bad_arguments(ctx):
    import janus_gpu as jg
    with pytest.raises(jg.JanusError):
        jg.update_digests(ctx, [b"a", b"b"], [0, 1])      # first[-1] != payload count
    with pytest.raises(jg.JanusError):
        jg.update_digests(ctx, [b"a", b"b"], [0, 2, 1])   # decreasing


@pytest.mark.gpu
def test_gpu_wave_resident_pnc_payloads(ctx):
    # the wave path over PNCounterMsg JSON payloads (what SafeCRDT.Update ships), 1000 per UpdateMessage
    import janus_gpu as jg
    rng = np.random.default_rng(6)
    msgs = []
    for i in range(5000):
        g = ["%032x" % int(rng.integers(0, 2**63)) for _ in range(5)]
        body = ",".join('"%s-%s-%s-%s-%s":%d' % (x[:8], x[8:12], x[12:16], x[16:20], x[20:], rng.integers(0, 2**31)) for x in g)
        msgs.append(('{"pVector":{%s},"nVector":{%s}}' % (body, body[:len(body) // 2].rsplit(",", 1)[0])).encode())
    w = jg.Wave(ctx, len(msgs), sum(map(len, msgs)))
    try:
        w.upload(np.zeros(len(msgs), np.uint32), msgs=msgs)
        first = np.arange(0, 5001, 1000, dtype=np.uint64)
        d, md = w.update_digests(first, msg_digests=True)
    finally:
        w.close()
    for m, g in zip(msgs, md):
        assert g.tobytes() == hashlib.sha256(m).digest()
    for u in range(5):
        assert d[u].tobytes() == py_digest(msgs[1000 * u:1000 * (u + 1)])


@pytest.mark.gpu
def test_gpu_wave_sha256_device_output(ctx):
    # jg_wave_sha256: per-payload SHA256.HashData into device memory (digest bytes)
    import torch
    import janus_gpu as jg
    rng = np.random.default_rng(7)
    msgs = random_msgs(rng, 3000, 0, 900)
    w = jg.Wave(ctx, len(msgs), sum(map(len, msgs)))
    try:
        w.upload(np.zeros(len(msgs), np.uint32), msgs=msgs)
        out = torch.zeros(len(msgs) * 32, dtype=torch.uint8, device=torch.device("cuda", ctx.device))
        w.sha256_device(out.data_ptr())
        got = out.cpu().numpy().reshape(-1, 32)
    finally:
        w.close()
    for m, g in zip(msgs, got):
        assert g.tobytes() == hashlib.sha256(m).digest()


@pytest.mark.gpu
def test_gpu_full_wave_sampled(ctx):
    # full C5 size (1M payloads of 340-375 B, 1000 UpdateMessages of 1000, as bench.py): every update
    # digest is computed on the device; three updates and 2000 payload hashes are recomputed by hashlib
    import torch
    import janus_gpu as jg
    rng = np.random.default_rng(8)
    n, per = 1_000_000, 1000
    lens = rng.integers(340, 376, n).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(32, 127, int(off[-1]), dtype=np.uint8)
    first = np.arange(0, n + 1, per, dtype=np.uint64)
    w = jg.Wave(ctx, n, data.size)
    try:
        w.upload(np.zeros(n, np.uint32), data=data, off=off)
        d = w.update_digests(first)
        out = torch.zeros(n * 32, dtype=torch.uint8, device=torch.device("cuda", ctx.device))
        w.sha256_device(out.data_ptr())
        md = out.cpu().numpy().reshape(-1, 32)
    finally:
        w.close()
    buf = data.tobytes()
    msg = lambda i: buf[int(off[i]):int(off[i + 1])]  # noqa: E731
    for u in (0, 499, 999):
        assert d[u].tobytes() == py_digest([msg(i) for i in range(u * per, (u + 1) * per)])
    for i in rng.integers(0, n, 2000):
        assert md[i].tobytes() == hashlib.sha256(msg(i)).digest()


@pytest.mark.gpu
def test_gpu_waves_pipelined(ctx):
    # jg_waves_update_digests: five waves of different sizes and UpdateMessage splits in one pipelined
    # call (wave k+1's first level beside wave k's chain; slots reused from wave 2 on), one wave listed
    # twice, one with empty UpdateMessages: byte for byte vs hashlib and
    # vs the single-wave call
    import janus_gpu as jg
    rng = np.random.default_rng(9)
    sizes = [3000, 1, 2500, 4000, 700]
    msgs = [random_msgs(rng, n, 0, 600) for n in sizes]
    firsts = [np.array([0, 1000, 1000, 2999, 3000]), np.array([0, 1]), np.array([0, 2500]),
              np.arange(0, 4001, 100), np.array([0, 0, 700, 700])]
    waves = []
    try:
        for m in msgs:
            w = jg.Wave(ctx, len(m), max(1, sum(map(len, m))))
            w.upload(np.zeros(len(m), np.uint32), msgs=m)
            waves.append(w)
        order = [0, 1, 2, 3, 4, 0]
        got = jg.waves_update_digests([waves[k] for k in order], [firsts[k] for k in order])
        single = [waves[k].update_digests(firsts[k]) for k in range(len(waves))]
        assert jg.waves_update_digests([], []) == []
        with pytest.raises(jg.JanusError):
            jg.waves_update_digests([waves[0], waves[1]], [firsts[0], np.array([0, 2])])  # first[-1] != count
    finally:
        for w in waves:
            w.close()
    for j, k in enumerate(order):
        f = firsts[k]
        assert np.array_equal(got[j], single[k])
        for u in range(f.size - 1):
            assert got[j][u].tobytes() == py_digest(msgs[k][int(f[u]):int(f[u + 1])])


@pytest.mark.gpu
def test_gpu_waves_pipelined_large(ctx):
    # Four large distinct waves (200k payloads, 200 UpdateMessages each) in one pipelined call: the kernels
    # run long enough that wave k+2's first level overwrites the slot wave k's chain may still read unless
    # the chain_free / level1_done events order them.  Each wave's digests equal its single-wave call.
    import janus_gpu as jg
    rng = np.random.default_rng(77)
    n, per = 200_000, 1000
    first = np.arange(0, n + 1, per, dtype=np.uint64)
    waves, single = [], []
    try:
        for k in range(4):
            lens = rng.integers(300, 420, n).astype(np.uint64)
            off = np.zeros(n + 1, np.uint64)
            off[1:] = np.cumsum(lens)
            data = rng.integers(32, 127, int(off[-1]), dtype=np.uint8)
            w = jg.Wave(ctx, n, data.size)
            w.upload(np.zeros(n, np.uint32), data=data, off=off)
            waves.append(w)
            single.append(w.update_digests(first))
        order = [0, 1, 2, 3, 1, 0]
        got = jg.waves_update_digests([waves[k] for k in order], [first] * len(order))
    finally:
        for w in waves:
            w.close()
    for j, k in enumerate(order):
        assert np.array_equal(got[j], single[k]), f"pipelined wave {j} (wave {k}) differs from its single-wave digests"
    assert not np.array_equal(single[0], single[1])


def test_waves_update_digests_argument_check():
    # host-side check of the pipelined binding: one first[] per wave (raised before the library is called)
    import janus_gpu as jg
    with pytest.raises(ValueError):
        jg.waves_update_digests([object(), object()], [np.array([0])])
