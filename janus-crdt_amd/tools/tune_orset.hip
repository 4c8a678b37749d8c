// tune_orset.hip — dev tool: interleaved timing of the chunked OR-Set union (csrc/orset_union.hpp)
// on the C3 add stream (100M + 100M records, 50 % shared).  Varies the tile shape (workgroup size x
// records per thread) and the lanes per boundary of k_partition; times partition, union and finish
// separately with hipEvents (median of rounds).  Two input cases: DENSE x DENSE (a fresh batch into a
// freshly loaded store) and CHUNKED x DENSE (the store is a previous union's output, chunks 50-100 %
// full).  Every variant's output is checked against the first (count + rank-weighted checksum).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../csrc/orset_union.hpp"

#define CK(x) do { hipError_t ev_ = (x); if (ev_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(ev_)); std::exit(1); } } while (0)

// Measured and dropped (profiles/r03/tune_orset_gallop_pf.txt: 163 VGPRs leave one workgroup per CU, 38 % of peak).
// Persistent variant for DENSE inputs (slot = rank): workgroup g walks tiles g, g + G, g + 2G, ... and
// issues the loads of its next tile's records into registers right after staging the current tile in
// LDS, so they are in flight while the current tile merges, compacts and stores (the one-tile kernel
// has no load in flight during those phases; two workgroups per CU fit the LDS).  Tile bounds come one
// iteration ahead of the loads that need them.
namespace jgk {
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_union_pf(View a, View b, const uint64_t* __restrict__ part, unsigned long long* __restrict__ ok,
                                                  uint4* __restrict__ ot, uint32_t* __restrict__ oord, uint32_t b_base,
                                                  uint32_t* __restrict__ ocnt, Drop drop, uint64_t n_tiles) {
    using SH = UnionShared<kOB, kItems>;
    constexpr int kTile = SH::kTile;
    __shared__ SH sh;
    const int tid = threadIdx.x;
    const uint64_t total_in = a.n + b.n;
    const uint64_t G = gridDim.x;
    uint64_t tile = blockIdx.x;
    if (tile >= n_tiles) return;

    unsigned long long rk[kItems], rlo[kItems], rhi[kItems];
    uint32_t rord[kItems];
    unsigned long long pk = 0;
    Tag pt{0, 0};
    // loads of tile t's records (and, on thread 0, the A record before it)
    auto issue = [&](uint64_t t, uint64_t i0, uint64_t i1) {
        const uint64_t d0 = t * kTile;
        const uint64_t j0 = d0 - i0;
        const int nA = (int)(i1 - i0);
        const uint64_t d1 = d0 + kTile < total_in ? d0 + kTile : total_in;
        const int n = (int)(d1 - d0);
#pragma unroll
        for (int it = 0; it < kItems; ++it) {
            const int x = min(it * kOB + tid, n - 1);
            const bool from_a = x < nA;
            const uint64_t r = from_a ? i0 + (uint64_t)x : j0 + (uint64_t)(x - nA);
            rk[it] = __builtin_nontemporal_load((from_a ? a.key : b.key) + r);
            const Tag tg = ld_tag_nt((from_a ? a.tag : b.tag) + r);
            rlo[it] = tg.lo;
            rhi[it] = tg.hi;
            rord[it] = __builtin_nontemporal_load((from_a ? a.ord : b.ord) + r) + (from_a ? 0u : b_base);
        }
        if (tid == 0 && i0 > 0) {
            pk = a.key[i0 - 1];
            pt = ld_tag(a.tag + i0 - 1);
        }
    };
    uint64_t i0 = part[tile], i1 = part[tile + 1];
    issue(tile, i0, i1);
    uint64_t nt = tile + G;
    uint64_t n0 = nt < n_tiles ? part[nt] : 0, n1 = nt < n_tiles ? part[nt + 1] : 0;
    for (;;) {
        const uint64_t d0 = tile * kTile;
        const uint64_t d1 = d0 + kTile < total_in ? d0 + kTile : total_in;
        const int nA = (int)(i1 - i0), n = (int)(d1 - d0);
#pragma unroll
        for (int it = 0; it < kItems; ++it) {
            const int x = it * kOB + tid;
            sh.key[x] = rk[it];
            sh.tag[x] = to_u4(Tag{rlo[it], rhi[it]});
        }
        if (tid == 0) {
            sh.has_prev = i0 > 0 && !dropped(drop, pk);
            sh.prev_key = pk;
            sh.prev_tag = to_u4(pt);
        }
        uint32_t cord[kItems];
#pragma unroll
        for (int it = 0; it < kItems; ++it) cord[it] = rord[it];
        __syncthreads();
        const uint64_t cur = tile;
        const bool more = nt < n_tiles;
        if (more) {
            issue(nt, n0, n1);  // in flight during this tile's merge and stores
            i0 = n0;
            i1 = n1;
            const uint64_t nn = nt + G;
            n0 = nn < n_tiles ? part[nn] : 0;
            n1 = nn < n_tiles ? part[nn + 1] : 0;
        }
        union_tile<kOB, kItems>(sh, nA, n - nA, cur, cord, ok, ot, oord, ocnt, drop);
        if (!more) break;
        tile = nt;
        nt += G;
        __syncthreads();  // every store of this tile read its LDS before the next staging
    }
}
}  // namespace jgk

using jgk::View;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 31; return x;
}
// Same generator as jg_synth_orset (csrc/synth.hip).
__global__ void k_gen(unsigned long long* key, uint4* tag, unsigned long long n, unsigned per, unsigned u0, unsigned E, unsigned long long seed) {
    for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        unsigned long long g = i / per, u = u0 + i % per;
        unsigned long long h1 = mix64(seed ^ mix64(g * 256 + u + 1)), h2 = mix64(h1 + 0x9E3779B97F4A7C15ull);
        key[i] = ((g / E) << 32) | (g % E);
        unsigned long long t0 = (u << 56) | (h1 >> 8);
        tag[i] = make_uint4((unsigned)t0, (unsigned)(t0 >> 32), (unsigned)h2, (unsigned)(h2 >> 32));
    }
}
__global__ void k_sum(View v, const uint32_t* cnt, unsigned long long* out) {
    unsigned long long s = 0;
    const unsigned long long slots = (unsigned long long)v.nch * v.C;
    for (unsigned long long x = blockIdx.x * 256ull + threadIdx.x; x < slots; x += gridDim.x * 256ull) {
        const unsigned long long c = x / v.C, j = x - c * v.C;
        if (j < cnt[c]) s += (v.key[x] ^ ((unsigned long long)v.tag[x].x << 1) ^ ((unsigned long long)v.tag[x].w << 17)) * (v.off[c] + j + 1);
    }
    atomicAdd(out, s);
}

// A device stream with chunk metadata sized for capacity `cap_slots`.
struct Stream {
    unsigned long long* key = nullptr;
    uint4* tag = nullptr;
    uint32_t* ord = nullptr;
    uint32_t* cnt = nullptr;
    uint64_t* off = nullptr;
    uint32_t* lut = nullptr;
    unsigned long long n = 0;
    uint32_t nch = 0, C = 0, dense = 1;
    // shift: the arrays start `shift` records into their allocations (tests whether streams whose ranks
    // line up at the same large-power-of-two address offsets contend for the same HBM channels)
    void alloc(unsigned long long cap_slots, uint32_t chunk, unsigned long long shift = 0) {
        const unsigned long long ch = cap_slots / chunk + 2;
        CK(hipMalloc(&key, (ch * chunk + shift) * 8)); CK(hipMalloc(&tag, (ch * chunk + shift) * 16)); CK(hipMalloc(&ord, (ch * chunk + shift) * 4));
        key += shift; tag += shift; ord += shift;
        CK(hipMalloc(&cnt, ch * 4)); CK(hipMalloc(&off, (ch + 1) * 8)); CK(hipMalloc(&lut, (((ch * chunk) >> jgk::kQShift) + 2) * 4));
        C = chunk;
    }
    View view() const { return View{key, tag, ord, off, lut, n, nch, C, dense}; }
    void set_dense(unsigned long long nn, hipStream_t s) {
        n = nn; nch = (uint32_t)((nn + C - 1) / C); dense = 1;
        const unsigned long long nlut = (nn >> jgk::kQShift) + 2;
        hipLaunchKernelGGL(jgk::k_dense_meta, dim3(1024), dim3(256), 0, s, nn, C, nch, cnt, off, lut, nlut);
    }
};

int num_cus;
char* ws;
unsigned long long* d_cnt;
struct Times { float part, uni, fin; };

template <int OB, int IT, int L>
Times run(Stream& a, Stream& b, Stream& o, hipStream_t s) {
    constexpr int T = OB * IT;
    const unsigned long long total = a.n + b.n, nt = (total + T - 1) / T;
    uint64_t* part = (uint64_t*)ws;
    uint32_t* pch = (uint32_t*)(ws + (((nt + 1) * 8 + 255) & ~255ull));
    hipEvent_t e[4];
    for (auto& x : e) CK(hipEventCreate(&x));
    const View va = a.view(), vb = b.view();
    CK(hipEventRecord(e[0], s));
    hipLaunchKernelGGL((jgk::k_partition<T, L>), dim3((unsigned)(((nt + 1) * L + 255) / 256)), dim3(256), 0, s, va, vb, nt + 1, part, pch);
    CK(hipEventRecord(e[1], s));
    hipLaunchKernelGGL((jgk::k_union<OB, IT>), dim3((unsigned)nt), dim3(OB), 0, s, va, vb, part, pch, o.key, o.tag, o.ord, (uint32_t)a.n, o.cnt,
                       jgk::Drop{nullptr, 0});
    CK(hipEventRecord(e[2], s));
    hipLaunchKernelGGL(jgk::k_finish, dim3((unsigned)((nt + 1023) / 1024)), dim3(1024), 0, s, o.cnt, (uint32_t)nt, o.off, o.lut,
                       (total >> jgk::kQShift) + 2, d_cnt);
    CK(hipEventRecord(e[3], s));
    CK(hipEventSynchronize(e[3]));
    CK(hipGetLastError());
    Times t;
    CK(hipEventElapsedTime(&t.part, e[0], e[1])); CK(hipEventElapsedTime(&t.uni, e[1], e[2])); CK(hipEventElapsedTime(&t.fin, e[2], e[3]));
    for (auto& x : e) CK(hipEventDestroy(x));
    CK(hipMemcpy(&o.n, d_cnt, 8, hipMemcpyDeviceToHost));
    o.nch = (uint32_t)nt; o.C = T; o.dense = 0;
    return t;
}

// MODE bit 0: k_partition_gallop instead of k_partition; bit 1: persistent k_union_pf (dense inputs) with
// PF workgroups per CU.
template <int MODE, int PF>
Times run2(Stream& a, Stream& b, Stream& o, hipStream_t s) {
    constexpr int OB = 512, IT = 6, T = OB * IT;
    const unsigned long long total = a.n + b.n, nt = (total + T - 1) / T;
    uint64_t* part = (uint64_t*)ws;
    uint32_t* pch = (uint32_t*)(ws + (((nt + 1) * 8 + 255) & ~255ull));
    hipEvent_t e[4];
    for (auto& x : e) CK(hipEventCreate(&x));
    const View va = a.view(), vb = b.view();
    CK(hipEventRecord(e[0], s));
    if (MODE & 1) hipLaunchKernelGGL((jgk::k_partition_gallop<T>), dim3((unsigned)((nt + 1 + 255) / 256)), dim3(256), 0, s, va, vb, nt + 1, part, pch);
    else hipLaunchKernelGGL((jgk::k_partition<T, 1>), dim3((unsigned)((nt + 1 + 255) / 256)), dim3(256), 0, s, va, vb, nt + 1, part, pch);
    CK(hipEventRecord(e[1], s));
    if ((MODE & 2) && a.dense && b.dense) {
        const unsigned g = (unsigned)std::min<unsigned long long>(nt, (unsigned long long)num_cus * PF);
        hipLaunchKernelGGL((jgk::k_union_pf<OB, IT>), dim3(g), dim3(OB), 0, s, va, vb, part, o.key, o.tag, o.ord, (uint32_t)a.n, o.cnt,
                           jgk::Drop{nullptr, 0}, nt);
    } else {
        hipLaunchKernelGGL((jgk::k_union<OB, IT>), dim3((unsigned)nt), dim3(OB), 0, s, va, vb, part, pch, o.key, o.tag, o.ord, (uint32_t)a.n, o.cnt,
                           jgk::Drop{nullptr, 0});
    }
    CK(hipEventRecord(e[2], s));
    hipLaunchKernelGGL(jgk::k_finish, dim3((unsigned)((nt + 1023) / 1024)), dim3(1024), 0, s, o.cnt, (uint32_t)nt, o.off, o.lut,
                       (total >> jgk::kQShift) + 2, d_cnt);
    CK(hipEventRecord(e[3], s));
    CK(hipEventSynchronize(e[3]));
    CK(hipGetLastError());
    Times t;
    CK(hipEventElapsedTime(&t.part, e[0], e[1])); CK(hipEventElapsedTime(&t.uni, e[1], e[2])); CK(hipEventElapsedTime(&t.fin, e[2], e[3]));
    for (auto& x : e) CK(hipEventDestroy(x));
    CK(hipMemcpy(&o.n, d_cnt, 8, hipMemcpyDeviceToHost));
    o.nch = (uint32_t)nt; o.C = T; o.dense = 0;
    return t;
}

struct Var { const char* name; Times (*fn)(Stream&, Stream&, Stream&, hipStream_t); };

unsigned long long checksum(const Stream& o) {
    unsigned long long* d; CK(hipMalloc(&d, 8)); CK(hipMemset(d, 0, 8));
    hipLaunchKernelGGL(k_sum, dim3(2048), dim3(256), 0, 0, o.view(), o.cnt, d);
    unsigned long long h; CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost)); CK(hipFree(d));
    return h;
}

void bench(const char* title, Stream& a, Stream& b, Stream& o, hipStream_t s, const std::vector<Var>& vs, int rounds) {
    std::printf("== %s: |A| %llu (%s), |B| %llu (%s)\n", title, a.n, a.dense ? "dense" : "chunked", b.n, b.dense ? "dense" : "chunked");
    unsigned long long rc = 0, rs = 0;
    for (size_t k = 0; k < vs.size(); ++k) {
        vs[k].fn(a, b, o, s);
        const unsigned long long c = o.n, sm = checksum(o);
        if (k == 0) { rc = c; rs = sm; }
        std::printf("%-24s count %llu checksum %016llx %s\n", vs[k].name, c, sm, c == rc && sm == rs ? "OK" : "MISMATCH");
    }
    std::vector<std::vector<Times>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t k = 0; k < vs.size(); ++k) t[k].push_back(vs[k].fn(a, b, o, s));
    const double bytes = (double)(a.n + b.n + rc) * 28;  // key 8 + tag 16 + ord 4
    for (size_t k = 0; k < vs.size(); ++k) {
        auto med = [&](float Times::*f) { std::vector<float> x; for (auto& y : t[k]) x.push_back(y.*f); std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        const double p = med(&Times::part), u = med(&Times::uni), f = med(&Times::fin);
        std::printf("%-24s partition %.3f  union %.3f (%.0f GB/s, %.1f%%)  finish %.3f  | all %.3f ms = %.0f GB/s\n", vs[k].name, p, u,
                    bytes / (u * 1e-3) / 1e9, 100 * bytes / (u * 1e-3) / 8e12, f, p + u + f, bytes / ((p + u + f) * 1e-3) / 1e9);
    }
}

int main(int argc, char** argv) {
    const unsigned long long G = 10000000, n = G * 10;
    { hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0)); num_cus = prop.multiProcessorCount; }
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    hipStream_t s; CK(hipStreamCreate(&s));
    CK(hipMalloc(&ws, 64 << 20));
    CK(hipMalloc(&d_cnt, 8));
    Stream a, b, o, o2;
    a.alloc(n, 3072); b.alloc(n, 3072); o.alloc(2 * n + 8192, 1024); o2.alloc(3 * n + 8192, 1024);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, a.key, a.tag, n, 10u, 0u, 10u, 0x4A414E5553ull);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, b.key, b.tag, n, 10u, 5u, 10u, 0x4A414E5553ull);
    a.set_dense(n, s);
    b.set_dense(n, s);
    CK(hipStreamSynchronize(s));

    const std::vector<Var> shapes = {
        {"OB512 IT6 L1 (prod)", run<512, 6, 1>}, {"gallop", run2<1, 2>}, {"OB512 IT6 L1 (prod) again", run<512, 6, 1>},
    };
    bench("dense x dense (C3 adds)", a, b, o, s, shapes, rounds);
    {  // the same inputs with B's arrays (and then the output's) started at odd record offsets
        Stream bs, os_;
        bs.alloc(n, 3072, 1573);
        os_.alloc(2 * n + 8192, 1024, 777);
        hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, bs.key, bs.tag, n, 10u, 5u, 10u, 0x4A414E5553ull);
        bs.set_dense(n, s);
        CK(hipStreamSynchronize(s));
        const std::vector<Var> pv = {{"prod", run<512, 6, 1>}, {"prod again", run<512, 6, 1>}};
        bench("dense x dense, B shifted 1573 records", a, bs, o, s, pv, rounds);
        bench("dense x dense, B shifted 1573, out 777", a, bs, os_, s, pv, rounds);
        bench("dense x dense, unshifted (control)", a, b, o, s, pv, rounds);
    }

    // chunked store: A' = A u B from the production shape, then A' u B2 with B2 a fresh dense batch
    run<512, 6, 1>(a, b, o, s);
    Stream b2;
    b2.alloc(n, 3072);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, b2.key, b2.tag, n, 10u, 10u, 10u, 0x4A414E5553ull);
    b2.set_dense(n, s);
    CK(hipStreamSynchronize(s));
    const std::vector<Var> ch = {
        {"OB512 IT6 L1 (prod)", run<512, 6, 1>}, {"gallop", run2<1, 2>},
    };
    // the C3 tombstone stream: 20M + 20M records (u in [0, 2) and [1, 3)), dense x dense
    Stream ra, rb, ro;
    const unsigned long long nr = G * 2;
    ra.alloc(nr, 3072); rb.alloc(nr, 3072); ro.alloc(2 * nr + 8192, 1024);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, ra.key, ra.tag, nr, 2u, 0u, 10u, 0x52454Dull);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, rb.key, rb.tag, nr, 2u, 1u, 10u, 0x52454Dull);
    ra.set_dense(nr, s);
    rb.set_dense(nr, s);
    CK(hipStreamSynchronize(s));
    const std::vector<Var> tv = {
        {"OB512 IT6 L1 (prod)", run<512, 6, 1>}, {"gallop", run2<1, 2>}, {"pf 2/CU", run2<2, 2>}, {"gallop+pf 2/CU", run2<3, 2>},
    };
    bench("dense x dense (C3 tombstones)", ra, rb, ro, s, tv, rounds);
    bench("chunked x dense (store = previous union output)", o, b2, o2, s, ch, rounds);
    return 0;
}
