// wire_cursor.hpp — device-side byte cursor over one wire payload (System.Text.Json state messages),
// shared by the PN-Counter decoder (json.hip) and the OR-Set decoder (orset_wire.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace jgw {

// Byte cursor over [p, end) with a 16-byte aligned window register: one aligned global load per 16
// bytes of payload.  The payload buffer is padded so that the last window load stays in bounds.
struct Cursor {
    const uint8_t* base;
    uint64_t p, end;
    uint64_t wbase;
    uint4 win;
    __device__ Cursor(const uint8_t* b, uint64_t beg, uint64_t e) : base(b), p(beg), end(e), wbase(~0ull), win{0, 0, 0, 0} {}
    __device__ __forceinline__ int peek() {
        if (p >= end) return -1;
        const uint64_t a = p & ~15ull;
        if (a != wbase) {
            win = *reinterpret_cast<const uint4*>(base + a);
            wbase = a;
        }
        const uint32_t k = (uint32_t)(p - a);
        const uint32_t w = k < 8 ? (k < 4 ? win.x : win.y) : (k < 12 ? win.z : win.w);
        return (int)((w >> ((k & 3) * 8)) & 0xFF);
    }
    __device__ __forceinline__ int get() {
        const int c = peek();
        if (c >= 0) ++p;
        return c;
    }
    __device__ __forceinline__ void ws() {
        for (;;) {
            const int c = peek();
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') ++p;
            else return;
        }
    }
    __device__ __forceinline__ bool expect(int ch) {
        ws();
        if (peek() != ch) return false;
        ++p;
        return true;
    }
};

__device__ __forceinline__ int hexv(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    const int l = c | 0x20;
    if (l >= 'a' && l <= 'f') return l - 'a' + 10;
    return -1;
}


// LDS written by some lanes of a wave, then read by others: order them (a group never spans waves).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---- SWAR over 4 ASCII bytes (byte 0 = the first character): 0x80 in each byte where a test holds --
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) { return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu); }
__device__ __forceinline__ uint32_t ge_bytes(uint32_t x7, uint32_t a) { return ((x7 | 0x80808080u) - a * 0x01010101u) & 0x80808080u; }
__device__ __forceinline__ uint32_t le_bytes(uint32_t x7, uint32_t b) { return ((b * 0x01010101u | 0x80808080u) - x7) & 0x80808080u; }
__device__ __forceinline__ uint32_t digit_bytes(uint32_t x) {  // '0'..'9'
    const uint32_t x7 = x & 0x7F7F7F7Fu;
    return ge_bytes(x7, 0x30) & le_bytes(x7, 0x39) & ~x;
}
__device__ __forceinline__ uint32_t bits4(uint32_t c) {  // 0x80 flags of bytes 0..3 -> bits 0..3
    return ((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u);
}
// 4 hex characters (hexv's alphabet: 0-9 a-f A-F) -> byte j = value of character j
__device__ __forceinline__ uint32_t hex4(uint32_t x, uint32_t& nib) {  // 1 if all four are hex
    const uint32_t x7 = x & 0x7F7F7F7Fu, l7 = x7 | 0x20202020u;
    const uint32_t dig = ge_bytes(x7, 0x30) & le_bytes(x7, 0x39);
    const uint32_t af = ge_bytes(l7, 0x61) & le_bytes(l7, 0x66);
    nib = (x & 0x0F0F0F0Fu) + ((af >> 7) | (af >> 4));  // + 9 per letter (no multiply: bits 0 and 3)
    return ((dig | af) & ~x & 0x80808080u) == 0x80808080u ? 1u : 0u;
}
__device__ __forceinline__ uint32_t hex_pairs(uint32_t nib) {  // byte 0 = c0 c1, byte 2 = c2 c3
    return ((nib & 0x000F000Fu) << 4) | ((nib >> 8) & 0x000F000Fu);
}
__device__ __forceinline__ uint32_t hex_be16(uint32_t nib) {  // the 4 characters as one hex number
    const uint32_t t = hex_pairs(nib);
    return ((t & 0xFFu) << 8) | (t >> 16);
}
__device__ __forceinline__ uint32_t hex_le16(uint32_t nib) {  // two hex-pair bytes, the first at the low address
    const uint32_t t = hex_pairs(nib);
    return (t & 0xFFu) | ((t >> 8) & 0xFF00u);
}

// K words of LDS bytes [q, q + 4K) at any alignment: K + 1 aligned reads, realigned in registers.
template <int K>
__device__ __forceinline__ void lds_words(const uint8_t* base, uint32_t q, uint32_t (&X)[K]) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base) + (q >> 2);
    const uint32_t sh = q & 3;
    uint32_t W[K + 1];
#pragma unroll
    for (int i = 0; i <= K; ++i) W[i] = w[i];
#pragma unroll
    for (int i = 0; i < K; ++i) X[i] = __builtin_amdgcn_alignbyte(W[i + 1], W[i], sh);
}

}  // namespace jgw
