"""Regenerate tests/golden/update_digests.npz (run from the repo root:
`python tests/golden/make_golden_digest.py`).

Expected values come from Python's hashlib (OpenSSL SHA-256, the same primitive .NET 6's
SHA256.HashData calls on Linux) plus the ArrayPool<byte>.Shared bucket rule (oracle/digest.hpp),
independently of the C++ oracle, so the fixture pins both the oracle and the HIP kernels.  Inputs:
PNCounterMsg-shaped JSON payloads of every length class around the SHA-256 padding boundaries,
C# null payloads, and UpdateMessages of 0, 1, 2, 3, 17 and 1000 payloads
(BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:32-55)."""
import hashlib
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent


def rent_length(n: int) -> int:  # ArrayPool<byte>.Shared.Rent(n).Length, .NET 6
    if n == 0:
        return 0
    if n > 1 << 20:
        return n
    return max(16, 1 << (n - 1).bit_length())


def compute_digest(msgs) -> bytes:  # UpdateMessage.ComputeDigest
    buf = bytearray(rent_length(32 * len(msgs)))
    for i, m in enumerate(msgs):
        if m is not None:
            buf[32 * i:32 * i + 32] = hashlib.sha256(m).digest()
    return hashlib.sha256(bytes(buf)).digest()


def payload(rng, n_bytes: int) -> bytes:
    g = "".join(f"{x:02x}" for x in rng.integers(0, 256, 16))
    s = '{"pVector":{"%s-%s-%s-%s-%s":%d},"nVector":{}}' % (g[:8], g[8:12], g[12:16], g[16:20], g[20:], rng.integers(0, 2**31))
    s = s.encode()
    if len(s) >= n_bytes:
        return s[:n_bytes]
    return s + bytes(rng.integers(32, 127, n_bytes - len(s)).astype(np.uint8))


def main():
    rng = np.random.default_rng(0x6469676573)
    lens = list(range(0, 130)) + [183, 247, 255, 256, 357, 1000, 1392, 4096, 65536 + 7]
    msgs = [payload(rng, n) for n in lens]
    msgs += [None if k % 5 == 2 else payload(rng, int(rng.integers(300, 420))) for k in range(1000 + 17 + 20)]
    sizes = [0, 1, 2, 3, 17, 1000, 0]
    sizes.append(len(msgs) - sum(sizes))
    first = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    digest = np.array([list(compute_digest(msgs[first[u]:first[u + 1]])) for u in range(len(sizes))], np.uint8)
    msg_digest = np.array([list(bytes(32) if m is None else hashlib.sha256(m).digest()) for m in msgs], np.uint8)
    is_null = np.array([m is None for m in msgs], np.uint8)
    off = np.concatenate([[0], np.cumsum([0 if m is None else len(m) for m in msgs])]).astype(np.uint64)
    data = np.frombuffer(b"".join(b"" if m is None else m for m in msgs), np.uint8)
    np.savez_compressed(HERE / "update_digests.npz", data=data, off=off, is_null=is_null, first=first, digest=digest,
                        msg_digest=msg_digest)
    print(f"{len(msgs)} payloads, {len(sizes)} updates, {data.size} bytes")


if __name__ == "__main__":
    main()
