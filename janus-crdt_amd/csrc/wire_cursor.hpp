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


// ---- JSON strings: read_string feeds each unescaped UTF-8 byte to sink.put(), sink.esc() at a backslash -------
struct GuidSink {  // Guid.Parse of the "D" form (what Guid's JSON converter accepts), C# byte order
    uint32_t k = 0, va = 0, vb = 0, vc = 0;
    unsigned long long hi = 0;
    bool bad = false;
    __device__ void esc() {}
    __device__ void put(int b) {
        if (k == 8 || k == 13 || k == 18 || k == 23) {
            bad |= b != '-';
        } else if (k < 36) {
            const int h = hexv(b);
            bad |= h < 0;
            const uint32_t x = (uint32_t)h & 15;
            if (k < 8) va = va << 4 | x;
            else if (k < 13) vb = vb << 4 | x;
            else if (k < 18) vc = vc << 4 | x;
            else {
                const uint32_t j = k < 23 ? k - 19 : k - 20;  // hex digit among the last 16
                hi |= (unsigned long long)x << (8 * (j >> 1) + ((j & 1) ? 0 : 4));
            }
        } else {
            bad = true;
        }
        ++k;
    }
    __device__ bool ok() const { return !bad && k == 36; }
    __device__ unsigned long long lo() const { return (unsigned long long)va | (unsigned long long)vb << 32 | (unsigned long long)vc << 48; }
};

__device__ __forceinline__ bool hex4(Cursor& c, uint32_t& u) {
    u = 0;
    for (int k = 0; k < 4; ++k) {
        const int h = hexv(c.get());
        if (h < 0) return false;
        u = u << 4 | (uint32_t)h;
    }
    return true;
}

template <class S> __device__ __forceinline__ void put_utf8(S& s, uint32_t u) {
    if (u < 0x80) { s.put((int)u); return; }
    if (u < 0x800) { s.put((int)(0xC0 | u >> 6)); s.put((int)(0x80 | (u & 0x3F))); return; }
    if (u < 0x10000) { s.put((int)(0xE0 | u >> 12)); s.put((int)(0x80 | (u >> 6 & 0x3F))); s.put((int)(0x80 | (u & 0x3F))); return; }
    s.put((int)(0xF0 | u >> 18)); s.put((int)(0x80 | (u >> 12 & 0x3F))); s.put((int)(0x80 | (u >> 6 & 0x3F))); s.put((int)(0x80 | (u & 0x3F)));
}

// The rest of a JSON string after its opening quote: escapes decoded (surrogate pairs joined), raw
// UTF-8 validated, control characters rejected — host/wire.cpp Scan::str.
template <class S> __device__ __forceinline__ bool read_string(Cursor& c, S& s) {
    for (;;) {
        const int ch = c.get();
        if (ch < 0) return false;
        if (ch == '"') return true;
        if (ch < 0x20) return false;
        if (ch == '\\') {
            s.esc();
            const int e = c.get();
            int out;
            switch (e) {
                case '"': out = '"'; break;
                case '\\': out = '\\'; break;
                case '/': out = '/'; break;
                case 'b': out = 8; break;
                case 'f': out = 12; break;
                case 'n': out = 10; break;
                case 'r': out = 13; break;
                case 't': out = 9; break;
                case 'u': {
                    uint32_t u;
                    if (!hex4(c, u) || (u >= 0xDC00 && u <= 0xDFFF)) return false;
                    if (u >= 0xD800 && u <= 0xDBFF) {
                        if (c.get() != '\\' || c.get() != 'u') return false;
                        uint32_t lo;
                        if (!hex4(c, lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
                        u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(s, u);
                    continue;
                }
                default: return false;
            }
            s.put(out);
            continue;
        }
        if (ch < 0x80) { s.put(ch); continue; }
        int extra;
        uint32_t cp;
        if (ch >= 0xC2 && ch <= 0xDF) { extra = 1; cp = ch & 0x1F; }
        else if (ch >= 0xE0 && ch <= 0xEF) { extra = 2; cp = ch & 0x0F; }
        else if (ch >= 0xF0 && ch <= 0xF4) { extra = 3; cp = ch & 0x07; }
        else return false;
        s.put(ch);
        for (int k = 0; k < extra; ++k) {
            const int cc = c.get();
            if (cc < 0 || (cc & 0xC0) != 0x80) return false;
            cp = cp << 6 | (uint32_t)(cc & 0x3F);
            s.put(cc);
        }
        if (extra == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
        if (extra == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
    }
}


// A string whose bytes nobody needs (a skipped member's names and values).
struct NullSink {
    __device__ void esc() {}
    __device__ void put(int) {}
};

// `lit` at the cursor (true / false / null)
__device__ __forceinline__ bool take_literal(Cursor& c, const char* lit) {
    for (; *lit; ++lit)
        if (c.get() != *lit) return false;
    return true;
}

// -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)? and no number character after it
__device__ inline bool skip_number(Cursor& c) {
    auto digits = [&c]() {
        uint32_t k = 0;
        for (int ch = c.peek(); ch >= '0' && ch <= '9'; ch = c.peek()) ++c.p, ++k;
        return k;
    };
    if (c.peek() == '-') ++c.p;
    const int d0 = c.peek();
    if (d0 < '0' || d0 > '9') return false;
    if (d0 == '0') ++c.p;
    else digits();
    if (c.peek() == '.') {
        ++c.p;
        if (!digits()) return false;
    }
    if (c.peek() == 'e' || c.peek() == 'E') {
        ++c.p;
        if (c.peek() == '+' || c.peek() == '-') ++c.p;
        if (!digits()) return false;
    }
    const int n = c.peek();
    return !((n >= '0' && n <= '9') || n == '.' || n == 'e' || n == 'E' || n == '+' || n == '-');
}

// The value of a member the message type does not have (System.Text.Json skips it; oracle/json.hpp Reader::
// skip_value): any well-formed JSON value, validated and dropped.  `depth` = containers open around it (the message
// object = 1); a container that would open level 65 fails (MaxDepth 64).  Iterative: bit k of `obj` says whether
// the k-th container open inside the value is an object (at most 63 of them).
__device__ inline bool skip_value(Cursor& c, int depth) {
    unsigned long long obj = 0;
    int n = 0;
    bool want = true;  // a value next (else: a separator or a closing bracket of the innermost container)
    for (;;) {
        c.ws();
        if (want) {
            const int ch = c.peek();
            if (ch == '{' || ch == '[') {
                if (depth + n + 1 > 64) return false;
                ++c.p;
                const bool o = ch == '{';
                obj = o ? obj | 1ull << n : obj & ~(1ull << n);
                ++n;
                c.ws();
                if (c.peek() == (o ? '}' : ']')) {
                    ++c.p;
                    --n;
                    want = false;
                } else if (o) {
                    NullSink ns;
                    if (!c.expect('"') || !read_string(c, ns) || !c.expect(':')) return false;
                }
                continue;
            }
            bool ok;
            if (ch == '"') {
                ++c.p;
                NullSink ns;
                ok = read_string(c, ns);
            } else if (ch == 't') ok = take_literal(c, "true");
            else if (ch == 'f') ok = take_literal(c, "false");
            else if (ch == 'n') ok = take_literal(c, "null");
            else ok = skip_number(c);
            if (!ok) return false;
            want = false;
            continue;
        }
        if (n == 0) return true;
        const bool o = (obj >> (n - 1)) & 1;
        const int ch = c.get();
        if (ch == ',') {
            if (o) {
                NullSink ns;
                if (!c.expect('"') || !read_string(c, ns) || !c.expect(':')) return false;
            }
            want = true;
        } else if (ch == (o ? '}' : ']')) {
            --n;
        } else {
            return false;
        }
    }
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
// hex4 without the compare: 0x80 in each byte that is not a hex digit (0 when all four are), so that the
// checks of a Guid's eight groups fold into one OR and one compare
__device__ __forceinline__ uint32_t hex4_bad(uint32_t x, uint32_t& nib) {
    const uint32_t x7 = x & 0x7F7F7F7Fu, l7 = x7 | 0x20202020u;
    const uint32_t dig = ge_bytes(x7, 0x30) & le_bytes(x7, 0x39);
    const uint32_t af = ge_bytes(l7, 0x61) & le_bytes(l7, 0x66);
    nib = (x & 0x0F0F0F0Fu) + ((af >> 7) | (af >> 4));
    return (~(dig | af) | x) & 0x80808080u;
}

// The 36-character "D" form in X[0..8] (characters 0..35, Guid.ToString() layout b3b2b1b0-b5b4-b7b6-b8b9-b10..b15)
// in C#'s byte order (lo = bytes 0..7, hi = 8..15); true iff every digit is hex and the dashes sit at 8, 13, 18,
// 23.  Digit pairs combine with one shift-or per group (byte 0 = characters 0-1, byte 2 = 2-3) and the bytes
// land in place with one v_perm per half word pair.
__device__ __forceinline__ bool guid_d(const uint32_t* X, unsigned long long& lo, unsigned long long& hi) {
    uint32_t n[8];
    const uint32_t bad = hex4_bad(X[0], n[0]) | hex4_bad(X[1], n[1]) | hex4_bad(__builtin_amdgcn_alignbyte(X[3], X[2], 1), n[2]) |
                         hex4_bad(__builtin_amdgcn_alignbyte(X[4], X[3], 2), n[3]) | hex4_bad(__builtin_amdgcn_alignbyte(X[5], X[4], 3), n[4]) |
                         hex4_bad(X[6], n[5]) | hex4_bad(X[7], n[6]) | hex4_bad(X[8], n[7]);
    // characters 8, 13, 18, 23 gathered into one word
    const uint32_t dashes = __builtin_amdgcn_perm(X[3], X[2], 0x0C0C0500u) | __builtin_amdgcn_perm(X[5], X[4], 0x07020C0Cu);
    uint32_t t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = n[i] << 4 | n[i] >> 8;  // valid only where every digit is (< 16)
    // group a big-endian into bytes 0..3, b and c big-endian into 4..5 / 6..7, the rest in text order
    lo = (unsigned long long)__builtin_amdgcn_perm(t[0], t[1], 0x04060002u) | (unsigned long long)__builtin_amdgcn_perm(t[3], t[2], 0x04060002u) << 32;
    hi = (unsigned long long)__builtin_amdgcn_perm(t[5], t[4], 0x06040200u) | (unsigned long long)__builtin_amdgcn_perm(t[7], t[6], 0x06040200u) << 32;
    return bad == 0 && dashes == 0x2D2D2D2Du;
}

// ---- quote positions of a 16-byte window -----------------------------------------------------------------
__device__ __forceinline__ uint32_t quote_flags(uint32_t x) {  // 0x80 in each byte equal to '"'
    return ~((((x & 0x7F7F7F7Fu) ^ 0x22222222u) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// 0x80 byte flags of a window's four words (bit 8k + 7 of word i) -> bit 4i + k: a 4x4 bit transpose (two delta
// swaps) and one byte gather, 17 operations instead of 31 for four bits4
__device__ __forceinline__ uint32_t flags16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3) {
    uint32_t u = f0 >> 7 | f1 >> 6 | f2 >> 5 | f3 >> 4;  // bit 8k + i
    uint32_t t = ((u >> 14) ^ u) & 0x00000C0Cu;  // swap the off-diagonal 2x2 blocks
    u ^= t ^ (t << 14);
    t = ((u >> 7) ^ u) & 0x000A000Au;  // then the off-diagonal bits inside each block: bit 8i + k
    u ^= t ^ (t << 7);
    u |= u >> 4;
    return __builtin_amdgcn_perm(u, u, 0x0C0C0200u);  // bytes 0 and 2
}
// bit j = byte j of the window is '"'
__device__ __forceinline__ uint32_t quote_mask16(uint4 v) {
    return flags16(quote_flags(v.x), quote_flags(v.y), quote_flags(v.z), quote_flags(v.w));
}

// Inclusive prefix sum over the 64 lanes of a wave: row_shr DPP moves inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry a row's total into the rows after it (no LDS, no address arithmetic; a
// __shfl_up ladder costs a ds_bpermute and ~6 VALU per step).  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t r = threadIdx.x & 15;
    uint32_t y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true); x += r >= 1 ? y : 0u;  // row_shr:1
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true); x += r >= 2 ? y : 0u;  // row_shr:2
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true); x += r >= 4 ? y : 0u;  // row_shr:4
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true); x += r >= 8 ? y : 0u;  // row_shr:8
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); x += y;  // row_bcast:15 -> rows 1, 3
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); x += y;  // row_bcast:31 -> rows 2, 3
    return x;
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

// The same from 8-byte aligned reads (base 8-byte aligned): ceil((q % 8 + 4K + 4) / 8) ds_read_b64 (twice the
// bytes per LDS cycle of ds_read2_b32, banks over 64), one mask stage for the dword offset.
template <int K>
__device__ __forceinline__ void lds_words_b64(const uint8_t* base, uint32_t q, uint32_t (&X)[K]) {
    constexpr int NQ = (7 + 4 * K + 4 + 7) / 8;
    const uint2* w = reinterpret_cast<const uint2*>(base) + (q >> 3);
    uint32_t W[2 * NQ];
#pragma unroll
    for (int b = 0; b < NQ; ++b) {
        const uint2 v = w[b];
        W[2 * b] = v.x, W[2 * b + 1] = v.y;
    }
    const uint32_t m1 = (q & 4) ? ~0u : 0u, sh = q & 3;
    uint32_t B[K + 1];
#pragma unroll
    for (int i = 0; i < K + 1; ++i) B[i] = W[i] ^ ((W[i] ^ W[i + 1]) & m1);
#pragma unroll
    for (int i = 0; i < K; ++i) X[i] = __builtin_amdgcn_alignbyte(B[i + 1], B[i], sh);
}

}  // namespace jgw
