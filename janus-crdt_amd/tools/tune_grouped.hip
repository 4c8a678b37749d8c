// tune_grouped.hip — dev tool: indexed PN-Counter merge variants (exchange / merge_rows with key indices)
// on the bench's exchange shape: 1M received rows x 64 replicas int64 into a 2M-key store, keys uniform
// (39 % of rows share their key with another row) or a permutation (every key once).  Interleaved
// rounds, hipEvents around each variant's whole launch sequence, median; checksums must agree.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tune_grouped tune_grouped.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
struct I64x2 { long long x, y; };
__device__ __forceinline__ uint4 vmax8(uint4 a, uint4 b) {
    I64x2 p = __builtin_bit_cast(I64x2, a), q = __builtin_bit_cast(I64x2, b);
    I64x2 r{p.x > q.x ? p.x : q.x, p.y > q.y ? p.y : q.y};
    return __builtin_bit_cast(uint4, r);
}
__device__ __forceinline__ uint4 ntl(const uint4* p) { return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p))); }
__device__ __forceinline__ void nts(uint4* p, uint4 v) { __builtin_nontemporal_store(__builtin_bit_cast(v4u, v), reinterpret_cast<v4u*>(p)); }

constexpr uint32_t kNil = 0xFFFFFFFFu;
constexpr int R = 64, NV = R * 8 / 16;  // 32 vectors per array row

// COUNT: also count each key's rows (round-2 first cut: a key seen once skips the next[] read)
template <bool COUNT>
__global__ void k_link(const uint32_t* keys, uint64_t n, uint32_t* claim, uint32_t* head, uint32_t* next) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t k = keys[i];
        if (COUNT) atomicAdd(claim + k, 1u);
        next[i] = atomicExch(head + k, (uint32_t)i);
    }
}
template <bool COUNT>
__global__ void k_reset(const uint32_t* keys, uint64_t n, uint32_t* claim, uint32_t* head) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        if (COUNT) claim[keys[i]] = 0;
        head[keys[i]] = kNil;
    }
}

// one wave per row, U rows in flight; list heads fold their keys' rows.  COUNT: the lead test and the
// walk use the occurrence count; otherwise (production, csrc/pnc.hip) the head alone decides.
template <int U, bool NTS, bool COUNT>
__global__ __launch_bounds__(256) void k_grouped(long long* AP, long long* AN, const long long* BP, const long long* BN, const uint32_t* keys,
                                                 const uint32_t* claim, const uint32_t* head, const uint32_t* next, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * 256) >> 6;
    for (uint64_t m0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U; m0 < n; m0 += nw * U) {
        uint64_t key[U];
        uint32_t cnt[U];
        bool lead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t m = m0 + u;
            key[u] = m < n ? keys[m] : 0;
            if (COUNT) {
                cnt[u] = m < n ? claim[key[u]] : 0;
                lead[u] = cnt[u] == 1 || (cnt[u] >= 2 && head[key[u]] == (uint32_t)m);
            } else {
                cnt[u] = 2;
                lead[u] = m < n && head[key[u]] == (uint32_t)m;
            }
        }
        const bool isP = lane < NV;
        const uint32_t w = isP ? lane : lane - NV;
        const long long* B = isP ? BP : BN;
        long long* A = isP ? AP : AN;
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lead[u]) {
                b[u] = ntl(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!lead[u]) continue;
            a[u] = vmax8(a[u], b[u]);
            for (uint32_t cur = cnt[u] == 1 ? kNil : next[m0 + u]; cur != kNil;) {
                const uint4 bb = ntl(reinterpret_cast<const uint4*>(B + (uint64_t)cur * R) + w);
                const uint32_t nx = next[cur];
                a[u] = vmax8(a[u], bb);
                cur = nx;
            }
            uint4* dst = reinterpret_cast<uint4*>(A + key[u] * R) + w;
            if (NTS) nts(dst, a[u]);
            else *dst = a[u];
        }
    }
}

// pipelined head-only: the next iteration's keys and list heads are loaded while this iteration's rows
// fold (the keys -> head -> rows chain otherwise leaves a wave with nothing in flight for two round trips)
template <int U>
__global__ __launch_bounds__(256) void k_grouped_pipe(long long* AP, long long* AN, const long long* BP, const long long* BN,
                                                      const uint32_t* keys, const uint32_t* head, const uint32_t* next, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t step = (((uint64_t)gridDim.x * 256) >> 6) * U;
    const bool isP = lane < NV;
    const uint32_t w = isP ? lane : lane - NV;
    const long long* B = isP ? BP : BN;
    long long* A = isP ? AP : AN;
    uint64_t m0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U;
    uint64_t key[U];
    bool lead[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        key[u] = m0 + u < n ? keys[m0 + u] : 0;
        lead[u] = m0 + u < n && head[key[u]] == (uint32_t)(m0 + u);
    }
    for (; m0 < n; m0 += step) {
        uint4 a[U], b[U];
        uint32_t nx0[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lead[u]) {
                b[u] = ntl(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
                nx0[u] = next[m0 + u];
            }
        const uint64_t m1 = m0 + step;
        uint64_t nkey[U];
        bool nlead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) nkey[u] = m1 + u < n ? keys[m1 + u] : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) nlead[u] = m1 + u < n && head[nkey[u]] == (uint32_t)(m1 + u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!lead[u]) continue;
            a[u] = vmax8(a[u], b[u]);
            for (uint32_t cur = nx0[u]; cur != kNil;) {
                const uint4 bb = ntl(reinterpret_cast<const uint4*>(B + (uint64_t)cur * R) + w);
                const uint32_t nx = next[cur];
                a[u] = vmax8(a[u], bb);
                cur = nx;
            }
            *(reinterpret_cast<uint4*>(A + key[u] * R) + w) = a[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) { key[u] = nkey[u]; lead[u] = nlead[u]; }
    }
}

// lead flags from a pass of their own (head[key] == m, then head reset), so the merge's chain is
// (keys, flag) -> rows: one dependent round trip fewer per iteration
__global__ void k_lead(const uint32_t* keys, uint64_t n, const uint32_t* head, uint8_t* lead) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        lead[i] = head[keys[i]] == (uint32_t)i;
}
template <int U>
__global__ __launch_bounds__(256) void k_grouped_flag(long long* AP, long long* AN, const long long* BP, const long long* BN,
                                                      const uint32_t* keys, const uint8_t* leadf, const uint32_t* next, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * 256) >> 6;
    const bool isP = lane < NV;
    const uint32_t w = isP ? lane : lane - NV;
    const long long* B = isP ? BP : BN;
    long long* A = isP ? AP : AN;
    for (uint64_t m0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U; m0 < n; m0 += nw * U) {
        uint64_t key[U];
        bool lead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            key[u] = m0 + u < n ? keys[m0 + u] : 0;
            lead[u] = m0 + u < n && leadf[m0 + u];
        }
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lead[u]) {
                b[u] = ntl(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!lead[u]) continue;
            a[u] = vmax8(a[u], b[u]);
            for (uint32_t cur = next[m0 + u]; cur != kNil;) {
                const uint4 bb = ntl(reinterpret_cast<const uint4*>(B + (uint64_t)cur * R) + w);
                const uint32_t nx = next[cur];
                a[u] = vmax8(a[u], bb);
                cur = nx;
            }
            *(reinterpret_cast<uint4*>(A + key[u] * R) + w) = a[u];
        }
    }
}

// sort-based: rows sorted by key (sk, sr); one wave per sorted position, U in flight; a segment head
// folds its segment's rows (independent loads, no pointer chase)
template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_sorted(long long* AP, long long* AN, const long long* BP, const long long* BN, const uint32_t* sk,
                                                const uint32_t* sr, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * 256) >> 6;
    const bool isP = lane < NV;
    const uint32_t w = isP ? lane : lane - NV;
    const long long* B = isP ? BP : BN;
    long long* A = isP ? AP : AN;
    for (uint64_t i0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U; i0 < n; i0 += nw * U) {
        uint32_t key[U];
        bool headp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + u;
            key[u] = i < n ? sk[i] : 0;
            headp[u] = i < n && (i == 0 || sk[i - 1] != key[u]);
        }
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (headp[u]) {
                b[u] = ntl(reinterpret_cast<const uint4*>(B + (uint64_t)sr[i0 + u] * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + (uint64_t)key[u] * R) + w);
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!headp[u]) continue;
            a[u] = vmax8(a[u], b[u]);
            for (uint64_t j = i0 + u + 1; j < n && sk[j] == key[u]; ++j)
                a[u] = vmax8(a[u], ntl(reinterpret_cast<const uint4*>(B + (uint64_t)sr[j] * R) + w));
            uint4* dst = reinterpret_cast<uint4*>(A + (uint64_t)key[u] * R) + w;
            if (NTS) nts(dst, a[u]);
            else *dst = a[u];
        }
    }
}

// Generation-tagged heads: head64[key] = gen << 32 | row, so a head left from an earlier batch reads as
// empty and no reset write is needed (the lead's head[key] = kNil store was one random write per
// distinct key).
__global__ void k_link_gen(const uint32_t* keys, uint64_t n, unsigned long long* head64, uint32_t* next, unsigned long long gen) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const unsigned long long old = atomicExch(head64 + keys[i], gen << 32 | i);
        next[i] = (old >> 32) == gen ? (uint32_t)old : kNil;
    }
}
template <int U>
__global__ __launch_bounds__(256) void k_grouped_gen(long long* AP, long long* AN, const long long* BP, const long long* BN, const uint32_t* keys,
                                                     const unsigned long long* head64, const uint32_t* next, uint64_t n, unsigned long long gen) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * 256) >> 6;
    const bool isP = lane < NV;
    const uint32_t w = isP ? lane : lane - NV;
    const long long* B = isP ? BP : BN;
    long long* A = isP ? AP : AN;
    for (uint64_t m0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U; m0 < n; m0 += nw * U) {
        uint64_t key[U];
        bool lead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t m = m0 + u;
            key[u] = m < n ? keys[m] : 0;
            lead[u] = m < n && head64[key[u]] == (gen << 32 | m);
        }
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lead[u]) {
                b[u] = ntl(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!lead[u]) continue;
            a[u] = vmax8(a[u], b[u]);
            for (uint32_t cur = next[m0 + u]; cur != kNil;) {
                const uint4 bb = ntl(reinterpret_cast<const uint4*>(B + (uint64_t)cur * R) + w);
                const uint32_t nx = next[cur];
                a[u] = vmax8(a[u], bb);
                cur = nx;
            }
            *(reinterpret_cast<uint4*>(A + key[u] * R) + w) = a[u];
        }
    }
}

// Ceilings of the access pattern (not merges): each lead row (precomputed flags) reads its B row and its
// key's A row and writes the A row back (RMW = 0) — the grouped merge minus its list walks — or only
// gathers the A row into a sequential output (RMW = 1, the guide's "random whole-row gather").
template <int U, int KIND>
__global__ __launch_bounds__(256) void k_ceiling(long long* AP, long long* AN, const long long* BP, const long long* BN, const uint32_t* keys,
                                                 const uint8_t* leadf, uint64_t n, long long* OP, long long* ON) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = ((uint64_t)gridDim.x * 256) >> 6;
    const bool isP = lane < NV;
    const uint32_t w = isP ? lane : lane - NV;
    const long long* B = isP ? BP : BN;
    long long* A = isP ? AP : AN;
    long long* O = isP ? OP : ON;
    for (uint64_t m0 = (((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6) * U; m0 < n; m0 += nw * U) {
        uint64_t key[U];
        bool lead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            key[u] = m0 + u < n ? keys[m0 + u] : 0;
            lead[u] = m0 + u < n && leadf[m0 + u];
        }
        uint4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lead[u]) {
                if (KIND == 0) b[u] = ntl(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!lead[u]) continue;
            if (KIND == 0) *(reinterpret_cast<uint4*>(A + key[u] * R) + w) = vmax8(a[u], b[u]);
            else nts(reinterpret_cast<uint4*>(O + (m0 + u) * R) + w, a[u]);
        }
    }
}

__global__ void k_sum(const unsigned long long* a, uint64_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) s += a[i] * (i | 1);
    atomicAdd(out, s);
}

int main() {
    const uint64_t n_keys = 2000000, n = 1000000, cells = n_keys * R;
    long long *AP, *AN, *BP, *BN, *A0P, *A0N;
    CK(hipMalloc(&AP, cells * 8)); CK(hipMalloc(&AN, cells * 8)); CK(hipMalloc(&A0P, cells * 8)); CK(hipMalloc(&A0N, cells * 8));
    CK(hipMalloc(&BP, n * R * 8)); CK(hipMalloc(&BN, n * R * 8));
    {
        std::mt19937_64 g(1);
        std::vector<long long> h(cells);
        for (auto& x : h) x = (long long)(g() % 1000000);
        CK(hipMemcpy(A0P, h.data(), cells * 8, hipMemcpyHostToDevice));
        for (auto& x : h) x = (long long)(g() % 1000000);
        CK(hipMemcpy(A0N, h.data(), cells * 8, hipMemcpyHostToDevice));
        h.resize(n * R);
        for (auto& x : h) x = (long long)(g() % 1000000);
        CK(hipMemcpy(BP, h.data(), n * R * 8, hipMemcpyHostToDevice));
        for (auto& x : h) x = (long long)(g() % 1000000);
        CK(hipMemcpy(BN, h.data(), n * R * 8, hipMemcpyHostToDevice));
    }
    uint32_t *keys, *claim, *head, *next, *sk, *sr, *rows;
    CK(hipMalloc(&keys, n * 4)); CK(hipMalloc(&claim, n_keys * 4)); CK(hipMalloc(&head, n_keys * 4)); CK(hipMalloc(&next, n * 4));
    CK(hipMalloc(&sk, n * 4)); CK(hipMalloc(&sr, n * 4)); CK(hipMalloc(&rows, n * 4));
    CK(hipMemset(claim, 0, n_keys * 4)); CK(hipMemset(head, 0xFF, n_keys * 4));
    std::vector<uint32_t> hr(n);
    for (uint64_t i = 0; i < n; ++i) hr[i] = (uint32_t)i;
    CK(hipMemcpy(rows, hr.data(), n * 4, hipMemcpyHostToDevice));
    size_t temp = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, keys, sk, rows, sr, (int)n, 0, 21));
    void* dtemp;
    CK(hipMalloc(&dtemp, temp));
    unsigned long long* dsum;
    CK(hipMalloc(&dsum, 8));
    int num_cus = 256;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned gk = 4096;
    auto grid = [&](int U) { uint64_t g = (n + U - 1) / U * 64 / 256; return (unsigned)std::min<uint64_t>(g, (uint64_t)num_cus * 16); };

    // kind: 0 head-only U4 (production), 1 head-only U8, 2 count+head U4, 3 sorted U4, 4 sorted U8, 5 sorted U4 nt-store
    struct Var { const char* name; int kind; };
    const Var vars[] = {{"head-only U4", 0}, {"head-only U8", 1}, {"count+head U4", 2}, {"sorted U4", 3}, {"sorted U8", 4}, {"sorted U4 nt-store", 5},
                        {"pipelined U4", 6}, {"pipelined U2", 7}, {"lead-flag U4", 8}, {"head-only U4 32/CU", 9},
                        {"head-only U4 nt-store", 10}, {"head-only U2 nt-store", 11}, {"ceiling: lead RMW, no lists", 12},
                        {"ceiling: lead A gather only", 13}, {"gen-tagged heads U4", 14}};
    constexpr int kVars = 15;
    unsigned long long* head64;
    CK(hipMalloc(&head64, n_keys * 8));
    CK(hipMemset(head64, 0, n_keys * 8));
    unsigned long long gen = 0;
    uint8_t* leadf;
    CK(hipMalloc(&leadf, n));
    long long *OP, *ON;  // gather-only ceiling's output
    CK(hipMalloc(&OP, n * R * 8)); CK(hipMalloc(&ON, n * R * 8));
    for (int dist = 0; dist < 2; ++dist) {
        std::vector<uint32_t> hk(n);
        std::mt19937_64 g(7 + dist);
        if (dist == 0) for (auto& k : hk) k = (uint32_t)(g() % n_keys);
        else {
            std::vector<uint32_t> p(n_keys);
            for (uint64_t i = 0; i < n_keys; ++i) p[i] = (uint32_t)i;
            std::shuffle(p.begin(), p.end(), g);
            for (uint64_t i = 0; i < n; ++i) hk[i] = p[i];
        }
        CK(hipMemcpy(keys, hk.data(), n * 4, hipMemcpyHostToDevice));
        std::printf("== keys %s\n", dist == 0 ? "uniform over 2M (39%% of rows repeat a key)" : "a permutation (every key once)");
        std::vector<std::vector<float>> t(kVars);
        std::vector<unsigned long long> chk(kVars);
        for (int round = 0; round < 7; ++round)
            for (const Var& v : vars) {
                CK(hipMemcpy(AP, A0P, cells * 8, hipMemcpyDeviceToDevice));
                CK(hipMemcpy(AN, A0N, cells * 8, hipMemcpyDeviceToDevice));
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, 0));
                if (v.kind <= 1) {
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    if (v.kind == 0) hipLaunchKernelGGL((k_grouped<4, false, false>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    if (v.kind == 1) hipLaunchKernelGGL((k_grouped<8, false, false>), dim3(grid(8)), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else if (v.kind == 2) {
                    hipLaunchKernelGGL(k_link<true>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    hipLaunchKernelGGL((k_grouped<4, false, true>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    hipLaunchKernelGGL(k_reset<true>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else if (v.kind == 6 || v.kind == 7) {
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    if (v.kind == 6) hipLaunchKernelGGL((k_grouped_pipe<4>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, head, next, n);
                    else hipLaunchKernelGGL((k_grouped_pipe<2>), dim3(grid(2)), dim3(256), 0, 0, AP, AN, BP, BN, keys, head, next, n);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else if (v.kind == 8) {
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    hipLaunchKernelGGL(k_lead, dim3(gk), dim3(256), 0, 0, keys, n, head, leadf);
                    hipLaunchKernelGGL((k_grouped_flag<4>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, leadf, next, n);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else if (v.kind == 10 || v.kind == 11) {
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    if (v.kind == 10) hipLaunchKernelGGL((k_grouped<4, true, false>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    else hipLaunchKernelGGL((k_grouped<2, true, false>), dim3(grid(2)), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else if (v.kind == 14) {
                    ++gen;
                    hipLaunchKernelGGL(k_link_gen, dim3(gk), dim3(256), 0, 0, keys, n, head64, next, gen);
                    hipLaunchKernelGGL((k_grouped_gen<4>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, head64, next, n, gen);
                } else if (v.kind == 12 || v.kind == 13) {  // flags computed outside the timed region
                    CK(hipEventRecord(e1, 0));
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    hipLaunchKernelGGL(k_lead, dim3(gk), dim3(256), 0, 0, keys, n, head, leadf);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(e0, 0));
                    if (v.kind == 12) hipLaunchKernelGGL((k_ceiling<4, 0>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, leadf, n, A0P, A0N);
                    else hipLaunchKernelGGL((k_ceiling<4, 1>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, keys, leadf, n, OP, ON);
                } else if (v.kind == 9) {
                    hipLaunchKernelGGL(k_link<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head, next);
                    const unsigned g9 = (unsigned)std::min<uint64_t>((n + 3) / 4 * 64 / 256, (uint64_t)num_cus * 32);
                    hipLaunchKernelGGL((k_grouped<4, false, false>), dim3(g9), dim3(256), 0, 0, AP, AN, BP, BN, keys, claim, head, next, n);
                    hipLaunchKernelGGL(k_reset<false>, dim3(gk), dim3(256), 0, 0, keys, n, claim, head);
                } else {
                    CK(hipcub::DeviceRadixSort::SortPairs(dtemp, temp, keys, sk, rows, sr, (int)n, 0, 21));
                    if (v.kind == 3) hipLaunchKernelGGL((k_sorted<4, false>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, sk, sr, n);
                    if (v.kind == 4) hipLaunchKernelGGL((k_sorted<8, false>), dim3(grid(8)), dim3(256), 0, 0, AP, AN, BP, BN, sk, sr, n);
                    if (v.kind == 5) hipLaunchKernelGGL((k_sorted<4, true>), dim3(grid(4)), dim3(256), 0, 0, AP, AN, BP, BN, sk, sr, n);
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipGetLastError());
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                t[v.kind].push_back(ms);
                CK(hipMemset(dsum, 0, 8));
                hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, (const unsigned long long*)AP, cells, dsum);
                hipLaunchKernelGGL(k_sum, dim3(4096), dim3(256), 0, 0, (const unsigned long long*)AN, cells, dsum);
                CK(hipMemcpy(&chk[v.kind], dsum, 8, hipMemcpyDeviceToHost));
            }
        for (const Var& v : vars) {
            auto x = t[v.kind];
            std::sort(x.begin(), x.end());
            const bool ceil = v.kind >= 12;
            std::printf("%-28s median %.3f ms  min %.3f  %s %016llx%s\n", v.name, x[x.size() / 2], x[0], ceil ? "(no merge) sum" : "checksum", chk[v.kind],
                        ceil || chk[v.kind] == chk[0] ? "" : "  MISMATCH");
        }
    }
    return 0;
}
