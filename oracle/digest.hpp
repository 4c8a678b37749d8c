// oracle/digest.hpp — TEST INFRASTRUCTURE ONLY (see oracle.hpp for who may load the oracle).
//
// CPU restatement of UpdateMessage.ComputeDigest (BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:32-55),
// the digest every batch of client states carries into consensus:
//
//     toSign = ArrayPool<byte>.Shared.Rent(update.Count * 32);   // :35
//     Array.Clear(toSign, 0, toSign.Length);                       // :36  (the WHOLE rented array)
//     foreach u: if (u.message is not null) copy SHA256(u.message) to toSign[32*i]   // :41-45
//     return SHA256.HashData(toSign);                              // :47  (hashes toSign.Length bytes)
//
// Two third-party pieces, absent from /root/reference (they are the .NET 6 runtime the reference
// targets, BFT-CRDT/BFT-CRDT.csproj:5):
//   * SHA256.HashData (System.Security.Cryptography, .NET 6.0; OpenSSL on Linux) = FIPS 180-4
//     SHA-256.  Restated below from the standard; pinned by the FIPS 180-4 / NIST example vectors
//     (oracle/test_kat.cpp) and against Python's hashlib in tests/test_digest.py.
//   * ArrayPool<byte>.Shared.Rent(n) (.NET 6.0 TlsOverPerCoreLockedStacksArrayPool<byte>): n == 0
//     returns the empty array; 0 < n <= 2^20 returns a pooled array of the bucket length
//     max(16, next power of two >= n) (buckets 16 << i, i < 17); n > 2^20 allocates exactly n.
//     So the second-level hash covers the digests plus zero padding up to that length.  .NET 7+
//     pools up to 2^30, which differs only above 32768 states per UpdateMessage (the batcher cuts
//     at clientBatchSize, SafeCRDTManager.cs:165-198, far below that).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle {

// FIPS 180-4 §4.2.2 constants.
inline constexpr uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

inline uint32_t sha_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// FIPS 180-4 §6.2.2: one 512-bit block into H.
inline void sha256_block(uint32_t H[8], const uint8_t blk[64]) {
    uint32_t W[64];
    for (int t = 0; t < 16; ++t)
        W[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 | (uint32_t)blk[4 * t + 2] << 8 | blk[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = sha_rotr(W[t - 15], 7) ^ sha_rotr(W[t - 15], 18) ^ (W[t - 15] >> 3);
        uint32_t s1 = sha_rotr(W[t - 2], 17) ^ sha_rotr(W[t - 2], 19) ^ (W[t - 2] >> 10);
        W[t] = W[t - 16] + s0 + W[t - 7] + s1;
    }
    uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t T1 = h + (sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[t] + W[t];
        uint32_t T2 = (sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + T2;
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// SHA256.HashData(data[0..n)) (FIPS 180-4 §5.1.1 padding, §5.3.3 initial value).
inline void sha256(const uint8_t* data, uint64_t n, uint8_t out[32]) {
    uint32_t H[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint64_t full = n / 64;
    for (uint64_t b = 0; b < full; ++b) sha256_block(H, data + 64 * b);
    uint8_t tail[128] = {0};
    uint64_t rem = n - 64 * full;
    if (rem) std::memcpy(tail, data + 64 * full, rem);
    tail[rem] = 0x80;
    uint64_t tl = rem + 9 <= 64 ? 64 : 128;
    uint64_t bits = n * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_block(H, tail);
    if (tl == 128) sha256_block(H, tail + 64);
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(H[i] >> (24 - 8 * j));
}

// ArrayPool<byte>.Shared.Rent(n).Length on .NET 6 (see the header).
inline uint64_t array_pool_rent_length(uint64_t n) {
    if (n == 0) return 0;
    if (n > (1ull << 20)) return n;
    uint64_t len = 16;
    while (len < n) len <<= 1;
    return len;
}

// UpdateMessage.ComputeDigest over update.Count payloads: msgs[i] / lens[i], null when is_null[i].
// msg_digest (optional) receives SHA256(message i) (zeros for null, as toSign holds).
inline void update_digest(uint64_t count, const uint8_t* const* msgs, const uint64_t* lens, const uint8_t* is_null, uint8_t out[32],
                          uint8_t* msg_digest = nullptr) {
    std::vector<uint8_t> toSign(array_pool_rent_length(count * 32), 0);  // Rent + Array.Clear (:35-36)
    for (uint64_t i = 0; i < count; ++i) {                               // :39-46
        if (!(is_null && is_null[i])) sha256(msgs[i], lens[i], toSign.data() + 32 * i);
        if (msg_digest) std::memcpy(msg_digest + 32 * i, toSign.data() + 32 * i, 32);
    }
    sha256(toSign.data(), toSign.size(), out);  // :47
}

}  // namespace oracle
