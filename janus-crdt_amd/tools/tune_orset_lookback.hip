// tune_orset.hip — dev tool: interleaved timing of OR-Set union variants (workgroup size x records
// per thread) on the C3 add stream (100M + 100M records, 50 % shared), hipEvents, median of rounds.
// Every variant's output is checked against the first (count and a position-weighted checksum).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "orset_union_lookback.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31; return x;
}
__global__ void k_gen(unsigned long long* key, uint4* tag, unsigned long long n, unsigned per, unsigned u0, unsigned E, unsigned long long seed) {
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        unsigned long long g = i / per, u = u0 + i % per;
        unsigned long long h1 = mix64(seed ^ mix64(g * 256 + u + 1)), h2 = mix64(h1 + 0x9E3779B97F4A7C15ull);
        key[i] = ((g / E) << 32) | (g % E);
        unsigned long long t0 = (u << 56) | (h1 >> 8);
        tag[i] = make_uint4((unsigned)t0, (unsigned)(t0 >> 32), (unsigned)h2, (unsigned)(h2 >> 32));
    }
}
__global__ void k_sum(const unsigned long long* key, const uint4* tag, unsigned long long n, unsigned long long* out) {
    unsigned long long s = 0;
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
        s += (key[i] ^ ((unsigned long long)tag[i].x << 1) ^ ((unsigned long long)tag[i].w << 17)) * (i + 1);
    atomicAdd(out, s);
}

struct StampW {
    unsigned long long* buf;
    __device__ __forceinline__ void operator()(int i) const {
        if (threadIdx.x == 0) {
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            buf[i] = t;
        }
    }
};

// k_union with phase stamps (thread 0's view): 0 start, 1 ticket, 2 bounds, 3 staged, 4 merge-path
// search, 5 serial merge, 6 scan, 7 look-back, 8 compaction, 9 stores issued.
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_union_stamped(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                                       const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                                       const uint64_t* __restrict__ part, uint64_t n_tiles,
                                                       unsigned long long* __restrict__ ok, uint4* __restrict__ ot,
                                                       unsigned long long* status, unsigned* ticket, unsigned long long* out_count,
                                                       unsigned* err, unsigned long long* stamps) {
    using namespace jgk;
    JGK_TILE_LDS(kOB, kItems);
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t tile = s_tile;
    StampW st{stamps + (size_t)tile * 16};
    st(1);
    const TileBounds b = tile_bounds<kOB, kItems>(tile, part, na, nb);
    if (tid == 0) asm volatile("" ::"v"(b.nA), "v"(b.nB));
    st(2);
    TileRegs<kItems> r;
    tile_load<kOB, kItems>(r, b, ak, at, bk, bt, tid);
    tile_stage<kOB, kItems>(r, b, L, tid);
    __syncthreads();
    st(3);
    tile_process<kOB, kItems, StampW>(tile, b, n_tiles, L, ok, ot, status, out_count, err, tid, st);
}

struct Buf { unsigned long long* key; uint4* tag; unsigned long long n; };

int num_cus;

template <int OB, int IT, bool PP = false, int LB = 1, bool PS = false>
float run(const Buf& a, const Buf& b, Buf& o, char* ws, unsigned* err, unsigned long long* cnt, hipStream_t s, float* part_ms) {
    const unsigned long long total = a.n + b.n, tile = OB * IT, nt = (total + tile - 1) / tile;
    const size_t sb = ((nt * 8 + 16) + 255) & ~255ull;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    CK(hipMemsetAsync(ws, 0, sb, s));
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL((jgk::k_partition<OB, IT>), dim3((nt + 1 + OB - 1) / OB), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n, nt + 1,
                       (uint64_t*)(ws + sb));
    CK(hipEventRecord(e1, s));
    if constexpr (PS) {
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, jgk::k_union_ps<OB, IT, LB>, OB, 0));
        unsigned long long g = (unsigned long long)num_cus * (occ > 0 ? occ : 1);
        if (g > nt) g = nt;
        hipLaunchKernelGGL((jgk::k_union_ps<OB, IT, LB>), dim3(g), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n,
                           (const uint64_t*)(ws + sb), nt, o.key, o.tag, (unsigned long long*)ws, (unsigned*)(ws + nt * 8), cnt, err);
    } else if constexpr (PP) {
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, jgk::k_union_pp<OB, IT>, OB, 0));
        static bool said = false;
        if (!said) { std::printf("occupancy PP<%d,%d> = %d blocks/CU\n", OB, IT, occ); said = true; }
        unsigned long long g = (unsigned long long)num_cus * (occ > 0 ? occ : 1);
        if (g > nt) g = nt;
        hipLaunchKernelGGL((jgk::k_union_pp<OB, IT>), dim3(g), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n,
                           (const uint64_t*)(ws + sb), nt, o.key, o.tag, (unsigned long long*)ws, (unsigned*)(ws + nt * 8), cnt, err);
    } else {
        hipLaunchKernelGGL((jgk::k_union<OB, IT, LB>), dim3(nt), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n, (const uint64_t*)(ws + sb), nt,
                           o.key, o.tag, (unsigned long long*)ws, (unsigned*)(ws + nt * 8), cnt, err);
    }
    CK(hipEventRecord(e2, s));
    CK(hipEventSynchronize(e2));
    float p, u;
    CK(hipEventElapsedTime(&p, e0, e1)); CK(hipEventElapsedTime(&u, e1, e2));
    *part_ms = p;
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1)); CK(hipEventDestroy(e2));
    return u;
}

// Persistent variant with stamps: 1 iteration start (staged), 2 next ticket read, 3 next loads issued.
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_union_pp_stamped(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                                          const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                                          const uint64_t* __restrict__ part, uint64_t n_tiles,
                                                          unsigned long long* __restrict__ ok, uint4* __restrict__ ot,
                                                          unsigned long long* status, unsigned* ticket, unsigned long long* out_count,
                                                          unsigned* err, unsigned long long* stamps) {
    using namespace jgk;
    JGK_TILE_LDS(kOB, kItems);
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    uint64_t tile = s_tile;
    if (tile >= n_tiles) return;
    TileBounds b = tile_bounds<kOB, kItems>(tile, part, na, nb);
    TileRegs<kItems> r;
    tile_load<kOB, kItems>(r, b, ak, at, bk, bt, tid);
    for (;;) {
        StampW st{stamps + (size_t)tile * 16};
        st(1);
        tile_stage<kOB, kItems>(r, b, L, tid);
        if (tid == 0) s_tile = atomicAdd(ticket, 1u);
        __syncthreads();
        st(2);
        const uint64_t next = s_tile;
        TileBounds nb2{0, 0, 0, 0};
        if (next < n_tiles) {
            nb2 = tile_bounds<kOB, kItems>(next, part, na, nb);
            tile_load<kOB, kItems>(r, nb2, ak, at, bk, bt, tid);
        }
        st(3);
        tile_process<kOB, kItems, StampW>(tile, b, n_tiles, L, ok, ot, status, out_count, err, tid, st);
        if (next >= n_tiles) break;
        tile = next;
        b = nb2;
        __syncthreads();
    }
}

template <int OB, int IT, bool PP = false>
void run_stamped(const Buf& a, const Buf& b, Buf& o, char* ws, unsigned* err, unsigned long long* cnt, hipStream_t s) {
    const unsigned long long total = a.n + b.n, tile = OB * IT, nt = (total + tile - 1) / tile;
    const size_t sb = ((nt * 8 + 16) + 255) & ~255ull;
    unsigned long long* stamps;
    CK(hipMalloc(&stamps, nt * 16 * 8));
    CK(hipMemset(stamps, 0, nt * 16 * 8));
    CK(hipMemsetAsync(ws, 0, sb, s));
    hipLaunchKernelGGL((jgk::k_partition<OB, IT>), dim3((nt + 1 + OB - 1) / OB), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n, nt + 1,
                       (uint64_t*)(ws + sb));
    if constexpr (PP) {
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_union_pp_stamped<OB, IT>, OB, 0));
        unsigned long long g = (unsigned long long)num_cus * (occ > 0 ? occ : 1);
        hipLaunchKernelGGL((k_union_pp_stamped<OB, IT>), dim3(g), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n,
                           (const uint64_t*)(ws + sb), nt, o.key, o.tag, (unsigned long long*)ws, (unsigned*)(ws + nt * 8), cnt, err, stamps);
    } else {
        hipLaunchKernelGGL((k_union_stamped<OB, IT>), dim3(nt), dim3(OB), 0, s, a.key, a.tag, a.n, b.key, b.tag, b.n, (const uint64_t*)(ws + sb), nt,
                           o.key, o.tag, (unsigned long long*)ws, (unsigned*)(ws + nt * 8), cnt, err, stamps);
    }
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(nt * 16);
    CK(hipMemcpy(h.data(), stamps, nt * 16 * 8, hipMemcpyDeviceToHost));
    double sum[10] = {0};
    unsigned long long tmin = ~0ull, tmax = 0;
    for (unsigned long long t = 0; t < nt; ++t) {
        for (int i = 2; i < 10; ++i) sum[i] += (double)(h[t * 16 + i] - h[t * 16 + i - 1]);
        tmin = std::min(tmin, h[t * 16 + 1]); tmax = std::max(tmax, h[t * 16 + 9]);
    }
    const char* nm[10] = {"", "", PP ? "stage+ticket" : "bounds(part ld)", PP ? "next bounds+loads" : "load+stage", "mp search", "serial merge",
                          "scan", "lookback", "compact", "store issue"};
    std::printf("stamps %sOB%d IT%d (shader cycles, avg per tile):", PP ? "PP " : "", OB, IT);
    double tot = 0;
    for (int i = 2; i < 10; ++i) tot += sum[i];
    for (int i = 2; i < 10; ++i) std::printf(" %s=%.0f (%.0f%%)", nm[i], sum[i] / nt, 100 * sum[i] / tot);
    std::printf("  | per-tile total %.0f, kernel span %llu\n", tot / nt, tmax - tmin);
    CK(hipFree(stamps));
}

struct V { const char* name; float (*fn)(const Buf&, const Buf&, Buf&, char*, unsigned*, unsigned long long*, hipStream_t, float*); };

int main(int argc, char** argv) {
    const unsigned long long G = 10000000, n = G * 10;
    { hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0)); num_cus = prop.multiProcessorCount; }
    Buf a{}, b{}, o{};
    CK(hipMalloc(&a.key, n * 8)); CK(hipMalloc(&a.tag, n * 16)); CK(hipMalloc(&b.key, n * 8)); CK(hipMalloc(&b.tag, n * 16));
    CK(hipMalloc(&o.key, 2 * n * 8)); CK(hipMalloc(&o.tag, 2 * n * 16));
    a.n = b.n = n;
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, a.key, a.tag, n, 10u, 0u, 10u, 0x4A414E5553ull);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, b.key, b.tag, n, 10u, 5u, 10u, 0x4A414E5553ull);
    char* ws; CK(hipMalloc(&ws, 64 << 20));
    unsigned* err; CK(hipMalloc(&err, 4)); CK(hipMemset(err, 0, 4));
    unsigned long long *cnt, *sum; CK(hipMalloc(&cnt, 8)); CK(hipMalloc(&sum, 8));
    hipStream_t s; CK(hipStreamCreate(&s));
    CK(hipDeviceSynchronize());
    { unsigned e0; CK(hipMemcpy(&e0, err, 4, hipMemcpyDeviceToHost)); std::printf("err after init %u\n", e0); }
    std::vector<V> vs = {
        {"OB512 IT6 (prod)", run<512, 6>},
        {"OB512 IT6 NOLB", run<512, 6, false, 0>},
        {"OB256 IT8 NOLB", run<256, 8, false, 0>},
        {"OB256 IT4 NOLB", run<256, 4, false, 0>},
        {"OB512 IT4 NOLB", run<512, 4, false, 0>},
        {"OB256 IT12 NOLB", run<256, 12, false, 0>},
        {"PS OB512 IT6 LB1", run<512, 6, false, 1, true>},
        {"PS OB512 IT6 NOLB", run<512, 6, false, 0, true>},
        {"PS OB256 IT8 NOLB", run<256, 8, false, 0, true>},
    };
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    std::vector<std::vector<float>> tu(vs.size()), tp(vs.size());
    unsigned long long ref_cnt = 0, ref_sum = 0;
    for (size_t k = 0; k < vs.size(); ++k) {  // warm + check
        float p;
        vs[k].fn(a, b, o, ws, err, cnt, s, &p);
        unsigned long long c, sm = 0;
        CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
        CK(hipMemset(sum, 0, 8));
        hipLaunchKernelGGL(k_sum, dim3(2048), dim3(256), 0, 0, o.key, o.tag, c, sum);
        CK(hipMemcpy(&sm, sum, 8, hipMemcpyDeviceToHost));
        unsigned ev = 7; CK(hipMemcpy(&ev, err, 4, hipMemcpyDeviceToHost));
        if (k == 0) { ref_cnt = c; ref_sum = sm; }
        std::printf("%-20s count %llu checksum %016llx err %u %s\n", vs[k].name, c, sm, ev,
                    (c == ref_cnt && sm == ref_sum) ? "OK" : std::strstr(vs[k].name, "NOLB") ? "(timing only)" : "MISMATCH");
    }
    run_stamped<512, 6>(a, b, o, ws, err, cnt, s);

    for (int r = 0; r < rounds; ++r)
        for (size_t k = 0; k < vs.size(); ++k) { float p; tu[k].push_back(vs[k].fn(a, b, o, ws, err, cnt, s, &p)); tp[k].push_back(p); }
    const double bytes = (2.0 * n + ref_cnt) * 24;
    for (size_t k = 0; k < vs.size(); ++k) {
        auto u = tu[k], p = tp[k];
        std::sort(u.begin(), u.end()); std::sort(p.begin(), p.end());
        const double um = u[u.size() / 2], pm = p[p.size() / 2];
        std::printf("%-20s union %.3f ms (%.0f GB/s, %.1f%%)  partition %.3f ms  total %.0f GB/s\n", vs[k].name, um, bytes / (um * 1e-3) / 1e9,
                    100 * bytes / (um * 1e-3) / 8e12, pm, bytes / ((um + pm) * 1e-3) / 1e9);
    }
    return 0;
}
