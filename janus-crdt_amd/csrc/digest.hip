// digest.hip — UpdateMessage digests on the device.
//
// UpdateMessage.ComputeDigest (BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:32-55) hashes every
// NetworkProtocol.message of a batch with SHA-256, writes the 32-byte digests one after another into a
// buffer rented from ArrayPool<byte>.Shared (cleared, so null messages and the bucket's tail are zero)
// and hashes the WHOLE rented buffer.  The rented length is .NET 6's bucket length: 0 for an empty
// batch, max(16, next power of two) up to 2^20 bytes, the exact length above (oracle/digest.hpp).
//
// Two kernels, both one lane per hash (SHA-256 is a serial chain per message; the parallelism is
// across messages):
//   k_sha_msgs     one lane per payload.  Payloads sit back to back at arbitrary byte offsets: a lane
//                  reads each 64-byte block through five aligned 16-byte loads (a granule is loaded
//                  only if it starts before the payload's end, so nothing outside the wave's byte
//                  range is touched) and shifts it into place with a 4-way dword select plus
//                  v_alignbyte.  The padding (0x80, zeros, bit length) is composed in registers on
//                  the last one or two blocks.  Output: the eight state words of each digest, which
//                  ARE the second level's message words (big-endian reading of the digest bytes).
//   k_sha_expand / k_sha_chain  the second level over those words (data blocks, the rented buffer's
//                  zero tail, the padding; no buffer materialised): message schedules of every block in
//                  parallel, then one lane per UpdateMessage runs only the rounds.
// The compression is fully unrolled (K as literals, the message schedule in a 16-word register ring,
// rotations as v_alignbit, three-way XORs as one v_bitop3).  VALU-bound: ≈1.5k VALU instructions per 64-byte block.
#include <algorithm>
#include <cstring>
#include <vector>

#include "jg_internal.hpp"
#include "sha256_device.hpp"

namespace {

constexpr int kBlock = 256;

using jgsha::bswap;
using jgsha::ch;
using jgsha::compress;
using jgsha::maj;
using jgsha::rotr;
using jgsha::sha_init;
using jgsha::xor3;

// An 80-byte window of a payload as five 16-byte granules; dword i of it (i constant after unrolling).
struct Win { uint4 g0, g1, g2, g3, g4; };
__device__ __forceinline__ uint32_t win_dw(const Win& w, int i) {
    const uint4 g = i < 4 ? w.g0 : i < 8 ? w.g1 : i < 12 ? w.g2 : i < 16 ? w.g3 : w.g4;
    const int c = i & 3;
    return c == 0 ? g.x : c == 1 ? g.y : c == 2 ? g.z : g.w;
}
// Granule j of the aligned window at p, or zeros when it starts at or past `end` (then granule 0, which
// holds payload bytes, is read instead: no address outside the payload's lines).
__device__ __forceinline__ uint4 ld_granule(uintptr_t p, int j, uintptr_t end) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    using G = const __attribute__((address_space(1))) v4u*;
    const uintptr_t a = p + 16 * j;
    const bool in = a < end;
    const v4u v = *(G)(in ? a : p);
    return in ? make_uint4(v.x, v.y, v.z, v.w) : make_uint4(0, 0, 0, 0);
}

// One lane per payload: D[8i..8i+8) = SHA-256 state words of payload i (zeros for a null payload);
// kBytes: the digest bytes instead (big-endian words, what SHA256.HashData returns).
template <bool kBytes>
__global__ void __launch_bounds__(kBlock) k_sha_msgs(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                     const uint8_t* __restrict__ is_null, uint64_t n, uint4* __restrict__ D) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t o0 = off[i], len = off[i + 1] - o0;
    if (is_null && is_null[i]) {
        D[2 * i] = make_uint4(0, 0, 0, 0);
        D[2 * i + 1] = make_uint4(0, 0, 0, 0);
        return;
    }
    const uintptr_t end = (uintptr_t)(bytes + o0 + len);
    uint32_t H[8];
    sha_init(H);
    const uint64_t nblk = (len + 72) >> 6;  // message + 0x80 + 8-byte length, rounded up to blocks
    // block b's five granules are loaded while block b - 1 compresses (its words are formed first): each
    // wave's own ~1.7k VALU instructions hide the load.  The 80-byte window is five uint4 values picked by
    // constant index (an array indexed through the per-lane select became a dynamic index: the compiler put
    // it in LDS, one full wait per granule), loaded through a global pointer (an address rebuilt from an
    // integer is generic: FLAT), without branches (a granule past the payload reads the block's first one
    // and is zeroed, so nothing outside the wave's byte range is touched).
    Win w;
    auto load = [&](uint64_t q0) {
        const uintptr_t p = (uintptr_t)(bytes + o0 + q0) & ~(uintptr_t)15;
        w.g0 = ld_granule(p, 0, end);
        w.g1 = ld_granule(p, 1, end);
        w.g2 = ld_granule(p, 2, end);
        w.g3 = ld_granule(p, 3, end);
        w.g4 = ld_granule(p, 4, end);
    };
    if (len > 0) load(0);
    for (uint64_t b = 0; b < nblk; ++b) {
        const uint64_t q0 = b << 6;
        uint32_t W[16];
        if (q0 < len) {
            const uint32_t s = (uint32_t)((uintptr_t)(bytes + o0 + q0) & 15);
            const bool s1 = (s >> 2) & 1, s2 = (s >> 3) & 1;
            const uint32_t sb = s & 3;
            uint32_t e[17];
#pragma unroll
            for (int k = 0; k < 17; ++k) {
                const uint32_t lo = s1 ? win_dw(w, k + 1) : win_dw(w, k);
                const uint32_t hi = s1 ? win_dw(w, k + 3) : win_dw(w, k + 2);
                e[k] = s2 ? hi : lo;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) W[k] = __builtin_amdgcn_alignbyte(e[k + 1], e[k], sb);  // bytes q0+4k.. (LE)
            if (q0 + 64 > len) {  // last data block: keep the payload's bytes, then 0x80
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int64_t r = (int64_t)len - (int64_t)(q0 + 4 * k);
                    if (r < 4) W[k] = r <= 0 ? (r == 0 ? 0x80u : 0u) : ((W[k] & ((1u << (8 * r)) - 1)) | (0x80u << (8 * r)));
                }
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) W[k] = bswap(W[k]);
            if (q0 + 64 < len) load(q0 + 64);  // the next block holds payload bytes: its granules now
        } else {  // a block of padding only: 0x80 opens it when the payload filled the previous block
#pragma unroll
            for (int k = 0; k < 16; ++k) W[k] = 0;
            if (q0 == len) W[0] = 0x80000000u;
        }
        if (b == nblk - 1) {
            W[14] = (uint32_t)(len >> 29);
            W[15] = (uint32_t)(len << 3);
        }
        compress(H, W);
    }
    if (kBytes) {
#pragma unroll
        for (int k = 0; k < 8; ++k) H[k] = bswap(H[k]);
    }
    D[2 * i] = make_uint4(H[0], H[1], H[2], H[3]);
    D[2 * i + 1] = make_uint4(H[4], H[5], H[6], H[7]);
}

__device__ __forceinline__ uint64_t rent_length(uint64_t n) {  // ArrayPool<byte>.Shared.Rent(n).Length, .NET 6
    if (n == 0) return 0;
    if (n > (1ull << 20)) return n;
    return n <= 16 ? 16 : 1ull << (64 - __clzll(n - 1));
}

// Second level, split so that the serial part is as short as possible.  Per UpdateMessage u the hashed
// buffer is D[first[u]..first[u+1]) (8 words each) followed by zeros up to the rented length L, then
// the padding: (L + 72) / 64 blocks, block b of u being global block boff[u] + b.
//   k_sha_expand  one lane per block (all updates' blocks in parallel): the block's 16 message words,
//                 the message schedule to 64 words and + K[t] -> KW[64 per block].  None of this depends
//                 on the chaining state, so it leaves the chain.
//   k_sha_chain   one lane per UpdateMessage: the 64 rounds per block on KW (next block's KW loaded
//                 while the current one compresses) — ≈940 VALU instructions per block instead of ≈1650.
__device__ __forceinline__ void update_block_words(const uint4* __restrict__ D, const uint64_t* __restrict__ first, uint64_t u, uint64_t b,
                                                   uint32_t W[16]) {
    const uint64_t m0 = first[u], cnt = first[u + 1] - m0;
    const uint64_t L = rent_length(cnt * 32);
    const uint64_t data_q = cnt * 2;  // uint4 granules of digest data
    const uint4* src = D + 2 * m0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t g = 4 * b + j;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (g < data_q) v = src[g];
        W[4 * j] = v.x; W[4 * j + 1] = v.y; W[4 * j + 2] = v.z; W[4 * j + 3] = v.w;
    }
    // L is a multiple of 32: the 0x80 byte opens a 16-byte granule of this block or the next.
    const uint64_t q0 = b << 6;
    if (L == q0) W[0] = 0x80000000u;        // (constant indices: W stays in registers)
    if (L == q0 + 32) W[8] = 0x80000000u;
    if (b == ((L + 72) >> 6) - 1) {
        W[14] = (uint32_t)(L >> 29);
        W[15] = (uint32_t)(L << 3);
    }
}

__global__ void __launch_bounds__(kBlock) k_sha_expand(const uint4* __restrict__ D, const uint64_t* __restrict__ first,
                                                       const uint64_t* __restrict__ boff, uint64_t n_upd, uint4* __restrict__ KW) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= boff[n_upd]) return;
    uint64_t lo = 0, hi = n_upd - 1;  // last u with boff[u] <= g (every update has at least one block)
    while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (boff[mid] <= g) lo = mid; else hi = mid - 1;
    }
    uint32_t W[64];
    update_block_words(D, first, lo, g - boff[lo], W);
#pragma unroll
    for (int t = 16; t < 64; ++t)
        W[t] = W[t - 16] + xor3(rotr(W[t - 15], 7), rotr(W[t - 15], 18), W[t - 15] >> 3) + W[t - 7] +
               xor3(rotr(W[t - 2], 17), rotr(W[t - 2], 19), W[t - 2] >> 10);
    constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint4* dst = KW + 16 * g;
#pragma unroll
    for (int q = 0; q < 16; ++q)
        dst[q] = make_uint4(W[4 * q] + K[4 * q], W[4 * q + 1] + K[4 * q + 1], W[4 * q + 2] + K[4 * q + 2], W[4 * q + 3] + K[4 * q + 3]);
}

#define JG_SHA_ROUND_KW(a, b, c, d, e, f, g, h, kw)                                                        \
    do {                                                                                                   \
        uint32_t t1_ = (h + (kw)) + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g);              \
        uint32_t t2_ = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);                          \
        d += t1_;                                                                                          \
        h = t1_ + t2_;                                                                                     \
    } while (0)

__device__ __forceinline__ void chain_block(uint32_t H[8], const uint4 kw[16]) {
    uint32_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
    for (int q = 0; q < 16; q += 2) {
        JG_SHA_ROUND_KW(a, bb, c, d, e, f, g, h, kw[q].x);
        JG_SHA_ROUND_KW(h, a, bb, c, d, e, f, g, kw[q].y);
        JG_SHA_ROUND_KW(g, h, a, bb, c, d, e, f, kw[q].z);
        JG_SHA_ROUND_KW(f, g, h, a, bb, c, d, e, kw[q].w);
        JG_SHA_ROUND_KW(e, f, g, h, a, bb, c, d, kw[q + 1].x);
        JG_SHA_ROUND_KW(d, e, f, g, h, a, bb, c, kw[q + 1].y);
        JG_SHA_ROUND_KW(c, d, e, f, g, h, a, bb, kw[q + 1].z);
        JG_SHA_ROUND_KW(bb, c, d, e, f, g, h, a, kw[q + 1].w);
    }
    H[0] += a; H[1] += bb; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// Unconditional (a block past the chain's end re-reads its last block): loads under a branch make the
// compiler's wait counting fall back to waiting for every load in flight.
__device__ __forceinline__ void load_kw(uint4 dst[16], const uint4* __restrict__ KW, uint64_t b, uint64_t b1) {
    const uint4* src = KW + 16 * (b < b1 ? b : b1 - 1);
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[q] = src[q];
    __builtin_amdgcn_sched_barrier(0);  // keep the loads here, ahead of the block that compresses meanwhile
}

// The lanes of a wave read 256 B each from far-apart blocks, so a block's KW arrives about one HBM round
// trip after it is requested: three blocks rotate through registers (two loads in flight while one
// block compresses), which keeps the chain on its VALU dependency path instead of the load latency.
__global__ void __launch_bounds__(kBlock) k_sha_chain(const uint4* __restrict__ KW, const uint64_t* __restrict__ boff, uint64_t n_upd,
                                                      uint4* __restrict__ out) {
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_upd) return;
    const uint64_t b0 = boff[u], b1 = boff[u + 1];
    uint32_t H[8];
    sha_init(H);
    uint4 x[16], y[16], z[16];
    load_kw(x, KW, b0, b1);
    load_kw(y, KW, b0 + 1, b1);
    for (uint64_t b = b0; b < b1; b += 3) {  // loads unconditional, compressions predicated
        load_kw(z, KW, b + 2, b1);
        chain_block(H, x);
        load_kw(x, KW, b + 3, b1);
        if (b + 1 < b1) chain_block(H, y);
        load_kw(y, KW, b + 4, b1);
        if (b + 2 < b1) chain_block(H, z);
    }
    out[2 * u] = make_uint4(bswap(H[0]), bswap(H[1]), bswap(H[2]), bswap(H[3]));
    out[2 * u + 1] = make_uint4(bswap(H[4]), bswap(H[5]), bswap(H[6]), bswap(H[7]));
}

uint32_t grid_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }
// k_sha_chain: one wave per workgroup, so the few chain waves spread over as many CUs as there are waves
constexpr uint32_t kChainBlock = 64;
uint32_t chain_grid(uint64_t n) { return (uint32_t)((n + kChainBlock - 1) / kChainBlock); }

void check_first(uint64_t n, uint64_t n_upd, const uint64_t* first) {
    JG_REQUIRE(first[0] == 0, JG_EINVAL, "update digests: first[0] must be 0");
    for (uint64_t u = 0; u < n_upd; ++u)
        JG_REQUIRE(first[u + 1] >= first[u], JG_EINVAL, "update digests: first[] decreases at update %llu", (unsigned long long)u);
    JG_REQUIRE(first[n_upd] == n, JG_EINVAL, "update digests: first[%llu] = %llu, expected the payload count %llu", (unsigned long long)n_upd,
               (unsigned long long)first[n_upd], (unsigned long long)n);
}

// boff[u] = first second-level block of update u: 32 * count bytes rounded up to the ArrayPool bucket
// (rent_length) plus the 72-byte SHA-256 tail, in 64-byte blocks.  Returns the total block count.
uint64_t chain_offsets(const uint64_t* first, uint64_t n_upd, uint64_t* boff) {
    boff[0] = 0;
    for (uint64_t u = 0; u < n_upd; ++u) {
        const uint64_t c = first[u + 1] - first[u];
        uint64_t L = c * 32;
        if (c && L <= (1ull << 20)) {
            uint64_t p = 32;
            while (p < L) p <<= 1;
            L = p;
        }
        boff[u + 1] = boff[u] + ((L + 72) >> 6);
    }
    return boff[n_upd];
}

inline uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

// The second level from per-payload digests already on the device (D: n state-word digests, zeros for null):
// update digests to the host (synchronous).
void chain_digests(jg_ctx* ctx, const uint4* D, uint64_t n, uint64_t n_upd, const uint64_t* first, uint8_t* digest) {
    if (n_upd == 0) return;
    std::vector<uint64_t> hb(2 * (n_upd + 1));
    std::memcpy(hb.data(), first, (n_upd + 1) * 8);
    const uint64_t B = chain_offsets(first, n_upd, hb.data() + n_upd + 1);
    char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, n_upd * 32 + hb.size() * 8 + B * 256 + 512));
    auto* out = reinterpret_cast<uint4*>(s);
    auto* d_first = reinterpret_cast<uint64_t*>(s + n_upd * 32);
    uint64_t* d_boff = d_first + n_upd + 1;
    auto* KW = reinterpret_cast<uint4*>(s + ((n_upd * 32 + hb.size() * 8 + 255) & ~255ull));
    hipStream_t st = ctx->stream;
    // from the context's page-locked write area when it fits (a pageable source is staged by the runtime)
    const void* src = hb.data();
    if (hb.size() * 8 <= jg::kPinBytes - jg::kPinRead) {
        void* pin = static_cast<char*>(ctx->hstat) + jg::kPinRead;
        std::memcpy(pin, hb.data(), hb.size() * 8);
        src = pin;
    }
    JG_HIP(hipMemcpyAsync(d_first, src, hb.size() * 8, hipMemcpyHostToDevice, st));
    k_sha_expand<<<grid_for(B), kBlock, 0, st>>>(D, d_first, d_boff, n_upd, KW);
    k_sha_chain<<<chain_grid(n_upd), kChainBlock, 0, st>>>(KW, d_boff, n_upd, out);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemcpyAsync(digest, out, n_upd * 32, hipMemcpyDeviceToHost, st));
    JG_HIP(hipStreamSynchronize(st));
}

__global__ void k_zero_null(uint4* D, const uint8_t* is_null, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && is_null[i]) D[2 * i] = D[2 * i + 1] = make_uint4(0, 0, 0, 0);
}

// Digest bytes <-> SHA-256 state words (big-endian words), in place, on the device.
__global__ void k_bswap_words(uint32_t* w, uint64_t n_words) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_words; i += (uint64_t)gridDim.x * kBlock) w[i] = __builtin_bswap32(w[i]);
}

// Both levels on device buffers already in place (d_bytes: payloads; d_off: n+1 offsets); results to host.
void run_digests(jg_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_off, const uint8_t* d_null, uint64_t n, uint64_t n_upd,
                 const uint64_t* first, uint8_t* msg_digest, uint8_t* digest) {
    std::vector<uint64_t> hb(2 * (n_upd + 1));  // first[] then boff[] (second-level block offsets)
    std::memcpy(hb.data(), first, (n_upd + 1) * 8);
    const uint64_t B = chain_offsets(first, n_upd, hb.data() + n_upd + 1);
    char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, n * 32 + n_upd * 32 + hb.size() * 8 + B * 256 + 512));
    auto* D = reinterpret_cast<uint4*>(s);
    auto* out = reinterpret_cast<uint4*>(s + n * 32);
    auto* d_first = reinterpret_cast<uint64_t*>(s + n * 32 + n_upd * 32);
    uint64_t* d_boff = d_first + n_upd + 1;
    auto* KW = reinterpret_cast<uint4*>(s + ((n * 32 + n_upd * 32 + hb.size() * 8 + 255) & ~255ull));
    hipStream_t st = ctx->stream;
    JG_HIP(hipMemcpyAsync(d_first, hb.data(), hb.size() * 8, hipMemcpyHostToDevice, st));
    if (n) k_sha_msgs<false><<<grid_for(n), kBlock, 0, st>>>(d_bytes, d_off, d_null, n, D);
    if (n_upd) {
        k_sha_expand<<<grid_for(B), kBlock, 0, st>>>(D, d_first, d_boff, n_upd, KW);
        k_sha_chain<<<chain_grid(n_upd), kChainBlock, 0, st>>>(KW, d_boff, n_upd, out);
    }
    JG_HIP(hipGetLastError());
    if (digest && n_upd) JG_HIP(hipMemcpyAsync(digest, out, n_upd * 32, hipMemcpyDeviceToHost, st));
    if (msg_digest && n) JG_HIP(hipMemcpyAsync(msg_digest, D, n * 32, hipMemcpyDeviceToHost, st));
    JG_HIP(hipStreamSynchronize(st));
    if (msg_digest) {  // state words -> digest bytes (big-endian)
        auto* w = reinterpret_cast<uint32_t*>(msg_digest);
        for (uint64_t k = 0; k < n * 8; ++k) w[k] = __builtin_bswap32(w[k]);
    }
}

}  // namespace

namespace jg {
// SHA-256 of n payloads already in device memory (d_bytes at d_off[i]..d_off[i+1]) into host `out` (n * 32 digest
// bytes), queued on ctx->stream: the caller's next sync covers it.  The encoders hash what they just wrote.
void sha256_device(jg_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* out) {
    if (n == 0) return;
    auto* D = static_cast<uint4*>(jg::scratch(ctx, ctx->scratch3, n * 32 + 256));
    hipStream_t st = ctx->stream;
    k_sha_msgs<false><<<grid_for(n), kBlock, 0, st>>>(d_bytes, d_off, nullptr, n, D);
    k_bswap_words<<<std::min<uint64_t>(grid_for(n * 8), 4096), kBlock, 0, st>>>(reinterpret_cast<uint32_t*>(D), n * 8);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemcpyAsync(out, D, n * 32, hipMemcpyDeviceToHost, st));
}
}  // namespace jg

extern "C" {

int jg_update_digests(jg_ctx* ctx, uint64_t n, const uint64_t* off, const uint8_t* bytes, const uint8_t* is_null, uint64_t n_updates,
                      const uint64_t* first, uint8_t* msg_digest, uint8_t* digest) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && off && first && (digest || n_updates == 0), JG_EINVAL, "jg_update_digests: NULL argument");
        JG_REQUIRE(n < 0xFFFFFFFFull * kBlock, JG_EINVAL, "jg_update_digests: too many payloads");
        JG_REQUIRE(off[0] == 0, JG_EINVAL, "jg_update_digests: off[0] must be 0");
        for (uint64_t i = 0; i < n; ++i)
            JG_REQUIRE(off[i + 1] >= off[i], JG_EINVAL, "jg_update_digests: offsets decrease at payload %llu", (unsigned long long)i);
        JG_REQUIRE(bytes || off[n] == 0, JG_EINVAL, "jg_update_digests: bytes is NULL");
        check_first(n, n_updates, first);
        jg::ensure_device(ctx);
        const uint64_t nb = off[n];
        char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch, ((nb + 15) & ~15ull) + (n + 1) * 8 + n + 256));
        auto* d_bytes = reinterpret_cast<uint8_t*>(s);
        auto* d_off = reinterpret_cast<uint64_t*>(s + ((nb + 15) & ~15ull));
        uint8_t* d_null = is_null ? reinterpret_cast<uint8_t*>(d_off + n + 1) : nullptr;
        hipStream_t st = ctx->stream;
        if (nb) JG_HIP(hipMemcpyAsync(d_bytes, bytes, nb, hipMemcpyHostToDevice, st));
        JG_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        if (is_null && n) JG_HIP(hipMemcpyAsync(d_null, is_null, n, hipMemcpyHostToDevice, st));
        run_digests(ctx, d_bytes, d_off, d_null, n, n_updates, first, msg_digest, digest);
    });
}

int jg_sha256_batch(jg_ctx* ctx, uint64_t n, const uint64_t* off, const uint8_t* bytes, uint8_t* out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && off && (out || n == 0), JG_EINVAL, "jg_sha256_batch: NULL argument");
        JG_REQUIRE(n < 0xFFFFFFFFull * kBlock, JG_EINVAL, "jg_sha256_batch: too many payloads");
        JG_REQUIRE(off[0] == 0, JG_EINVAL, "jg_sha256_batch: off[0] must be 0");
        for (uint64_t i = 0; i < n; ++i)
            JG_REQUIRE(off[i + 1] >= off[i], JG_EINVAL, "jg_sha256_batch: offsets decrease at payload %llu", (unsigned long long)i);
        JG_REQUIRE(bytes || off[n] == 0, JG_EINVAL, "jg_sha256_batch: bytes is NULL");
        if (n == 0) return;
        jg::ensure_device(ctx);
        const uint64_t nb = off[n];
        char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch, ((nb + 15) & ~15ull) + (n + 1) * 8 + n * 32 + 256));
        auto* d_bytes = reinterpret_cast<uint8_t*>(s);
        auto* d_off = reinterpret_cast<uint64_t*>(s + ((nb + 15) & ~15ull));
        auto* D = reinterpret_cast<uint4*>(s + ((((nb + 15) & ~15ull) + (n + 1) * 8 + 15) & ~15ull));
        hipStream_t st = ctx->stream;
        if (nb) JG_HIP(hipMemcpyAsync(d_bytes, bytes, nb, hipMemcpyHostToDevice, st));
        JG_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, st));
        k_sha_msgs<false><<<grid_for(n), kBlock, 0, st>>>(d_bytes, d_off, nullptr, n, D);
        k_bswap_words<<<std::min<uint64_t>(grid_for(n * 8), 4096), kBlock, 0, st>>>(reinterpret_cast<uint32_t*>(D), n * 8);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(out, D, n * 32, hipMemcpyDeviceToHost, st));
        JG_HIP(hipStreamSynchronize(st));
    });
}

int jg_update_digests_of(jg_ctx* ctx, uint64_t n, const uint8_t* msg_digest, const uint8_t* is_null, uint64_t n_updates, const uint64_t* first,
                         uint8_t* digest) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && first && (msg_digest || n == 0) && (digest || n_updates == 0), JG_EINVAL, "jg_update_digests_of: NULL argument");
        JG_REQUIRE(n < 0xFFFFFFFFull * kBlock, JG_EINVAL, "jg_update_digests_of: too many payloads");
        check_first(n, n_updates, first);
        if (n_updates == 0) return;
        jg::ensure_device(ctx);
        auto* D = static_cast<uint4*>(jg::scratch(ctx, ctx->scratch, n * 32 + n + 256));
        auto* d_null = reinterpret_cast<uint8_t*>(D + 2 * n);  // D: two uint4 per digest
        hipStream_t st = ctx->stream;
        if (n) {
            JG_HIP(hipMemcpyAsync(D, msg_digest, n * 32, hipMemcpyHostToDevice, st));
            k_bswap_words<<<std::min<uint64_t>(grid_for(n * 8), 4096), kBlock, 0, st>>>(reinterpret_cast<uint32_t*>(D), n * 8);
            if (is_null) {  // a null payload hashes as 32 zero bytes whatever its row holds
                JG_HIP(hipMemcpyAsync(d_null, is_null, n, hipMemcpyHostToDevice, st));
                k_zero_null<<<grid_for(n), kBlock, 0, st>>>(D, d_null, n);
            }
            JG_HIP(hipGetLastError());
        }
        chain_digests(ctx, D, n, n_updates, first, digest);
    });
}

int jg_wave_update_digests(const jg_wave* w, uint64_t n_updates, const uint64_t* first, uint8_t* msg_digest, uint8_t* digest) {
    return jg::guard([&] {
        auto lk_ = jg::lock(w);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(w && first && (digest || n_updates == 0), JG_EINVAL, "jg_wave_update_digests: NULL argument");
        check_first(w->n, n_updates, first);
        jg::ensure_device(w->ctx);
        run_digests(w->ctx, w->bytes.as<uint8_t>(), w->off.as<uint64_t>(), nullptr, w->n, n_updates, first, msg_digest, digest);
    });
}

int jg_waves_update_digests(const jg_wave* const* waves, uint64_t n_waves, const uint64_t* n_updates, const uint64_t* const* first,
                            uint8_t* const* digest) {
    return jg::guard([&] {
        JG_REQUIRE(n_waves == 0 || (waves && n_updates && first && digest), JG_EINVAL, "jg_waves_update_digests: NULL argument");
        if (n_waves == 0) return;
        jg_ctx* ctx = waves[0] ? waves[0]->ctx : nullptr;
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, streams)
        JG_REQUIRE(ctx, JG_EINVAL, "jg_waves_update_digests: wave 0 is NULL");
        // host metadata of every wave, [first (nu+1) | boff (nu+1)] back to back, uploaded once; the
        // digests of every wave land in one device array (one D2H at the end, no pageable copy inside the
        // pipeline that would block the host until the chain before it finished)
        std::vector<uint64_t> moff(n_waves + 1, 0), ooff(n_waves + 1, 0), blocks(n_waves);
        for (uint64_t k = 0; k < n_waves; ++k) {
            const jg_wave* w = waves[k];
            const uint64_t nu = n_updates[k];
            JG_REQUIRE(w && w->ctx == ctx, JG_EINVAL, "jg_waves_update_digests: wave %llu is NULL or on another context", (unsigned long long)k);
            JG_REQUIRE(first[k] && (digest[k] || nu == 0), JG_EINVAL, "jg_waves_update_digests: NULL first/digest for wave %llu",
                       (unsigned long long)k);
            check_first(w->n, nu, first[k]);
            moff[k + 1] = moff[k] + 2 * (nu + 1);
            ooff[k + 1] = ooff[k] + nu * 32;
        }
        std::vector<uint64_t> hm(moff[n_waves]);
        uint64_t slot = 0;  // one slot: first-level digests D then the second level's KW blocks
        for (uint64_t k = 0; k < n_waves; ++k) {
            const uint64_t nu = n_updates[k];
            std::memcpy(&hm[moff[k]], first[k], (nu + 1) * 8);
            blocks[k] = chain_offsets(first[k], nu, &hm[moff[k] + nu + 1]);
            slot = std::max(slot, align256(waves[k]->n * 32) + blocks[k] * 256);
        }
        slot = align256(slot);
        const uint64_t m_bytes = align256(hm.size() * 8), o_bytes = align256(ooff[n_waves]);
        jg::ensure_device(ctx);
        char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, m_bytes + o_bytes + 2 * slot + 256));
        auto* d_meta = reinterpret_cast<uint64_t*>(s);
        char* d_out = s + m_bytes;
        hipStream_t st = ctx->stream, sd = ctx->side, s1 = ctx->level1;
        // a failure below leaves work queued on `side` / `level1` writing the scratch slots: drain both
        // before the error leaves the call (the next user of scratch3 orders itself on `stream` only)
        struct Drain {
            hipStream_t a, b;
            bool armed = true;
            ~Drain() {
                if (!armed) return;
                (void)hipStreamSynchronize(a);
                (void)hipStreamSynchronize(b);
                (void)hipGetLastError();
            }
        } drain{sd, s1};
        JG_HIP(hipMemcpyAsync(d_meta, hm.data(), hm.size() * 8, hipMemcpyHostToDevice, st));
        JG_HIP(hipEventRecord(ctx->begun, st));  // the metadata and every earlier upload / kernel on `stream`
        JG_HIP(hipStreamWaitEvent(s1, ctx->begun, 0));
        // wave k: first level + schedules on `level1` into slot k&1 (after wave k-2's chain released it),
        // its chain on `side`; wave k+1's first level overlaps wave k's chain
        for (uint64_t k = 0; k < n_waves; ++k) {
            const jg_wave* w = waves[k];
            const uint64_t nu = n_updates[k];
            const int sl = (int)(k & 1);
            char* base = s + m_bytes + o_bytes + sl * slot;
            auto* D = reinterpret_cast<uint4*>(base);
            auto* KW = reinterpret_cast<uint4*>(base + align256(w->n * 32));
            const uint64_t* d_first = d_meta + moff[k];
            const uint64_t* d_boff = d_first + nu + 1;
            if (k >= 2) JG_HIP(hipStreamWaitEvent(s1, ctx->chain_free[sl], 0));
            if (w->n) k_sha_msgs<false><<<grid_for(w->n), kBlock, 0, s1>>>(w->bytes.as<uint8_t>(), w->off.as<uint64_t>(), nullptr, w->n, D);
            if (nu) k_sha_expand<<<grid_for(blocks[k]), kBlock, 0, s1>>>(D, d_first, d_boff, nu, KW);
            JG_HIP(hipEventRecord(ctx->level1_done[sl], s1));
            JG_HIP(hipStreamWaitEvent(sd, ctx->level1_done[sl], 0));
            if (nu) k_sha_chain<<<chain_grid(nu), kChainBlock, 0, sd>>>(KW, d_boff, nu, reinterpret_cast<uint4*>(d_out + ooff[k]));
            JG_HIP(hipEventRecord(ctx->chain_free[sl], sd));
        }
        JG_HIP(hipGetLastError());
        // the last chain (side is in order; it waited on the last first level, which waited on `level1`'s past)
        JG_HIP(hipStreamWaitEvent(st, ctx->chain_free[(n_waves - 1) & 1], 0));
        std::vector<uint8_t> out(ooff[n_waves]);
        if (!out.empty()) JG_HIP(hipMemcpyAsync(out.data(), d_out, out.size(), hipMemcpyDeviceToHost, st));
        JG_HIP(hipStreamSynchronize(st));
        drain.armed = false;  // `stream` waited on the last chain, which waited on every earlier launch
        for (uint64_t k = 0; k < n_waves; ++k)
            if (n_updates[k]) std::memcpy(digest[k], out.data() + ooff[k], n_updates[k] * 32);
    });
}

int jg_wave_sha256(const jg_wave* w, void* d_out, uint8_t async) {
    return jg::guard([&] {
        auto lk_ = jg::lock(w);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(w && (d_out || w->n == 0), JG_EINVAL, "jg_wave_sha256: NULL argument");
        jg::ensure_device(w->ctx);
        hipStream_t st = w->ctx->stream;
        if (w->n) k_sha_msgs<true><<<grid_for(w->n), kBlock, 0, st>>>(w->bytes.as<uint8_t>(), w->off.as<uint64_t>(), nullptr, w->n,
                                                                      static_cast<uint4*>(d_out));
        JG_HIP(hipGetLastError());
        if (!async) JG_HIP(hipStreamSynchronize(st));
    });
}

}  // extern "C"
