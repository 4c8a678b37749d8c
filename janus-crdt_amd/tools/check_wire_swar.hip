// check_wire_swar.hip — device check of the SWAR wire helpers (csrc/wire_cursor.hpp) against host formatting:
// guid_d (text -> C# byte order, validity), quote_mask16, and the DPP
// scans (wave_incl_scan, group_scan) against host prefix sums.  A tool, not part of the library.
//   hipcc -O3 --offload-arch=gfx950 -I../include -Icsrc tools/check_wire_swar.hip -o build/check_wire_swar
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "wire_cursor.hpp"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } \
    } while (0)

constexpr int kN = 4096;

__global__ void k_guid(const uint8_t* text, unsigned long long* lo, unsigned long long* hi, uint32_t* ok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kN) return;
    uint32_t X[9];
    for (int k = 0; k < 9; ++k) std::memcpy(&X[k], text + i * 36 + 4 * k, 4);
    unsigned long long l, h;
    ok[i] = jgw::guid_d(X, l, h) ? 1u : 0u;
    lo[i] = l;
    hi[i] = h;
}

__global__ void k_scans(const uint32_t* in, uint32_t* wave_out, uint32_t* g8_out, uint32_t* last8, const uint4* win, uint32_t* qmask) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t x = in[i];
    wave_out[i] = jgw::wave_incl_scan(x);
    const uint32_t g = threadIdx.x % 8, y = x;
    uint32_t s = y;
    {
        uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x111, 0xF, 0xF, true); s += g >= 1 ? t : 0u;
        t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x112, 0xF, 0xF, true); s += g >= 2 ? t : 0u;
        t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s, 0x114, 0xF, 0xF, true); s += g >= 4 ? t : 0u;
    }
    g8_out[i] = s;
    last8[i] = (uint32_t)__builtin_amdgcn_ds_swizzle((int)s, (int)((0x1Fu & ~7u) | 7u << 5));
    qmask[i] = jgw::quote_mask16(win[i]);
}

static std::string guid_str(const uint8_t* b) {  // C# Guid.ToString() of bytes in C# order
    char s[37];
    std::snprintf(s, sizeof s, "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[3], b[2], b[1], b[0], b[5], b[4], b[7],
                  b[6], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
    return s;
}

int main() {
    std::mt19937_64 rng(7);
    std::vector<uint8_t> bytes(kN * 16), text(kN * 36);
    for (auto& b : bytes) b = (uint8_t)rng();
    std::vector<uint32_t> expect_ok(kN, 1);
    for (int i = 0; i < kN; ++i) {
        std::string s = guid_str(&bytes[i * 16]);
        if (i % 7 == 3) { s[(i / 7) % 36] = "gG -:Z{"[i % 7]; expect_ok[i] = 0; }  // a bad character somewhere
        if (i % 11 == 5) for (auto& c : s) c = (char)std::toupper(c);             // uppercase: valid, decodes the same
        std::memcpy(&text[i * 36], s.data(), 36);
        if (expect_ok[i] == 0) {  // a dash replaced by '-' stays valid; a hex digit replaced by another hex digit too
            const char c = s[(i / 7) % 36];
            const int pos = (i / 7) % 36;
            const bool dash = pos == 8 || pos == 13 || pos == 18 || pos == 23;
            const bool hexc = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
            if ((dash && c == '-') || (!dash && hexc)) expect_ok[i] = 1;
        }
    }
    uint8_t* dt;
    unsigned long long *dlo, *dhi;
    uint32_t* dok;
    CK(hipMalloc(&dt, text.size()));
    CK(hipMalloc(&dlo, kN * 8));
    CK(hipMalloc(&dhi, kN * 8));
    CK(hipMalloc(&dok, kN * 4));
    CK(hipMemcpy(dt, text.data(), text.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_guid, dim3(kN / 256), dim3(256), 0, 0, dt, dlo, dhi, dok);
    CK(hipGetLastError());
    std::vector<unsigned long long> lo(kN), hi(kN);
    std::vector<uint32_t> ok(kN);
    CK(hipMemcpy(lo.data(), dlo, kN * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hi.data(), dhi, kN * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ok.data(), dok, kN * 4, hipMemcpyDeviceToHost));
    int bad_ok = 0, bad_bytes = 0;
    for (int i = 0; i < kN; ++i) {
        if (ok[i] != expect_ok[i]) ++bad_ok;
        if (!expect_ok[i]) continue;
        uint8_t got[16];
        std::memcpy(got, &lo[i], 8);
        std::memcpy(got + 8, &hi[i], 8);
        if (std::memcmp(got, &bytes[i * 16], 16) != 0) {
            if (bad_bytes++ < 3) std::printf("bytes %d: %s vs %s\n", i, guid_str(got).c_str(), guid_str(&bytes[i * 16]).c_str());
        }
    }
    std::printf("guid_d validity mismatches %d, byte mismatches %d (of %d)\n", bad_ok, bad_bytes, kN);

    // scans and quote masks
    std::vector<uint32_t> in(kN);
    std::vector<uint4> win(kN);
    for (auto& x : in) x = (uint32_t)(rng() % 17);
    for (auto& w : win) {
        uint8_t b[16];
        for (auto& c : b) { const uint64_t r = rng() % 6; c = r == 0 ? '"' : r == 1 ? 0xA2 : (uint8_t)('a' + r); }
        std::memcpy(&w, b, 16);
    }
    uint32_t *din, *dw, *dg, *dl, *dq;
    uint4* dwin;
    CK(hipMalloc(&din, kN * 4));
    CK(hipMalloc(&dw, kN * 4));
    CK(hipMalloc(&dg, kN * 4));
    CK(hipMalloc(&dl, kN * 4));
    CK(hipMalloc(&dq, kN * 4));
    CK(hipMalloc(&dwin, kN * 16));
    CK(hipMemcpy(din, in.data(), kN * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwin, win.data(), kN * 16, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_scans, dim3(kN / 256), dim3(256), 0, 0, din, dw, dg, dl, dwin, dq);
    CK(hipGetLastError());
    std::vector<uint32_t> w(kN), g8(kN), l8(kN), q(kN);
    CK(hipMemcpy(w.data(), dw, kN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(g8.data(), dg, kN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l8.data(), dl, kN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(q.data(), dq, kN * 4, hipMemcpyDeviceToHost));
    int bw = 0, bg = 0, bl = 0, bq = 0;
    for (int i = 0; i < kN; ++i) {
        uint32_t sw = 0, sg = 0, tot = 0;
        for (int j = i - i % 64; j <= i; ++j) sw += in[j];
        for (int j = i - i % 8; j <= i; ++j) sg += in[j];
        for (int j = i - i % 8; j < i - i % 8 + 8; ++j) tot += in[j];
        bw += w[i] != sw;
        bg += g8[i] != sg;
        bl += l8[i] != tot;
        uint8_t b[16];
        std::memcpy(b, &win[i], 16);
        uint32_t m = 0;
        for (int j = 0; j < 16; ++j) m |= (b[j] == '"' ? 1u : 0u) << j;
        bq += q[i] != m;
    }
    std::printf("wave scan mismatches %d, group-8 scan %d, group-8 last %d, quote masks %d (of %d)\n", bw, bg, bl, bq, kN);
    const bool pass = !bad_ok && !bad_bytes && !bw && !bg && !bl && !bq;
    std::printf("%s\n", pass ? "PASS" : "FAIL");
    return pass ? 0 : 1;
}
