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

}  // namespace jgw
