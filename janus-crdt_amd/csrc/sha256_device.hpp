// sha256_device.hpp — SHA-256 compression on one lane (FIPS 180-4 §6.2.2), shared by csrc/digest.hip
// (UpdateMessage.ComputeDigest) and tools/valu_rate.hip (its measured issue ceiling).
// Fully unrolled: K as literals, the message schedule in a 16-word register ring, rotations as
// v_alignbit_b32, three-way XORs / Ch / Maj as one v_bitop3_b32 each.  Measured issue costs on gfx950
// (tools/valu_rate.hip, profiles/r04/valu_rate.txt): v_alignbit_b32 and v_add3_u32 take ~4 cycles per
// wave64 instruction, v_bitop3_b32 ~2.5, v_add_u32 ~2 — 576 rotations and ~240 three-way adds per block
// make the block's issue time ~1.4x what 1.6k instructions at 2 cycles would be.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace jgsha {

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
// v_bitop3_b32 truth tables: bit (s0 << 2 | s1 << 1 | s2) of the immediate is the result for those input bits.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA); }
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8); }

#define JG_SHA_ROUND(a, b, c, d, e, f, g, h, k, w)                                                     \
    do {                                                                                                \
        uint32_t t1_ = (h + (k) + (w)) + xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25)) + ch(e, f, g);       \
        uint32_t t2_ = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22)) + maj(a, b, c);                         \
        d += t1_;                                                                                       \
        h = t1_ + t2_;                                                                                  \
    } while (0)

// FIPS 180-4 §6.2.2 on one block W[16] (consumed) into H[8].
__device__ __forceinline__ void compress(uint32_t H[8], uint32_t W[16]) {
    constexpr uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
    for (int t = 0; t < 64; t += 8) {
        if (t >= 16) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = (t + j) & 15;
                uint32_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
                W[i] += xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3) + W[(i + 9) & 15] + xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            }
        }
        JG_SHA_ROUND(a, b, c, d, e, f, g, h, K[t + 0], W[(t + 0) & 15]);
        JG_SHA_ROUND(h, a, b, c, d, e, f, g, K[t + 1], W[(t + 1) & 15]);
        JG_SHA_ROUND(g, h, a, b, c, d, e, f, K[t + 2], W[(t + 2) & 15]);
        JG_SHA_ROUND(f, g, h, a, b, c, d, e, K[t + 3], W[(t + 3) & 15]);
        JG_SHA_ROUND(e, f, g, h, a, b, c, d, K[t + 4], W[(t + 4) & 15]);
        JG_SHA_ROUND(d, e, f, g, h, a, b, c, K[t + 5], W[(t + 5) & 15]);
        JG_SHA_ROUND(c, d, e, f, g, h, a, b, K[t + 6], W[(t + 6) & 15]);
        JG_SHA_ROUND(b, c, d, e, f, g, h, a, K[t + 7], W[(t + 7) & 15]);
    }
    H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

__device__ __forceinline__ void sha_init(uint32_t H[8]) {
    H[0] = 0x6a09e667; H[1] = 0xbb67ae85; H[2] = 0x3c6ef372; H[3] = 0xa54ff53a;
    H[4] = 0x510e527f; H[5] = 0x9b05688c; H[6] = 0x1f83d9ab; H[7] = 0x5be0cd19;
}

}  // namespace jgsha
