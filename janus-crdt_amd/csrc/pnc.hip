// pnc.hip — PN-Counter store and kernels (gfx950, wave64, no MFMA: integer bandwidth work).
//
// Layout in HBM: P and N are row-major [n_keys x R] arrays of the store's width (int32 = the
// reference's `int`, int64 = the BASELINE variant).  Row = interned key, column = interned replica.
//
// Kernels and their roofline (HBM):
//   k_merge_dense    A = max(A, B) over identity rows.  Reads A.P A.N B.P B.N, writes A.P A.N:
//                    6 x elem_bytes per cell (48 B at int64).  One 16-B vector per array per lane,
//                    non-temporal.  This is PNCounter.Merge (PNCounters.cs:131-144).
//   k_merge_indexed  scatter-max of received rows into their keys (atomicMax: rows may repeat a
//                    key inside one committed batch, SafeCRDTManager.cs:122-146).
//   k_apply_ops      Increment/Decrement (PNCounters.cs:97-112): wrapping atomic adds.
//   k_values         PNCounter.Get (PNCounters.cs:87-90): one wave per key, exact prefix sums in
//                    column order to reproduce the checked LINQ Sum's OverflowException.
#include <cstdlib>

#include "jg_internal.hpp"

namespace {

constexpr int kBlock = 256;

struct I64x2 { long long x, y; };
struct I32x4 { int x, y, z, w; };

template <int EB> __device__ __forceinline__ uint4 vmax(uint4 a, uint4 b);
template <> __device__ __forceinline__ uint4 vmax<8>(uint4 a, uint4 b) {
    I64x2 p = __builtin_bit_cast(I64x2, a), q = __builtin_bit_cast(I64x2, b);
    I64x2 r{p.x > q.x ? p.x : q.x, p.y > q.y ? p.y : q.y};
    return __builtin_bit_cast(uint4, r);
}
template <> __device__ __forceinline__ uint4 vmax<4>(uint4 a, uint4 b) {
    I32x4 p = __builtin_bit_cast(I32x4, a), q = __builtin_bit_cast(I32x4, b);
    I32x4 r{max(p.x, q.x), max(p.y, q.y), max(p.z, q.z), max(p.w, q.w)};
    return __builtin_bit_cast(uint4, r);
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load(const uint4* p) {
    return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)));
}
__device__ __forceinline__ void nt_store(uint4* p, uint4 v) {
    __builtin_nontemporal_store(__builtin_bit_cast(v4u, v), reinterpret_cast<v4u*>(p));
}

template <int EB> struct Elem;
template <> struct Elem<4> { using T = int; };
template <> struct Elem<8> { using T = long long; };

// Dense merge: nv 16-byte vectors per array, one vector of each array per lane, plus `tail` trailing
// cells (< 16 B) done by block 0.  Measured on MI355X against grid-stride / multi-vector-per-lane /
// block-chunk variants (tools/tune_pnc.hip, profiles/r01/tune_pnc_*.txt): a flat grid with one
// vector per lane and non-temporal loads/stores (every byte is touched once) was fastest.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_merge_dense(uint4* __restrict__ AP, uint4* __restrict__ AN,
                                                        const uint4* __restrict__ BP, const uint4* __restrict__ BN,
                                                        uint64_t nv, uint32_t tail) {
    using T = typename Elem<EB>::T;
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < nv) {
        const uint4 ap = nt_load(AP + i), bp = nt_load(BP + i), an = nt_load(AN + i), bn = nt_load(BN + i);
        nt_store(AP + i, vmax<EB>(ap, bp));
        nt_store(AN + i, vmax<EB>(an, bn));
    }
    if (blockIdx.x == 0 && threadIdx.x < tail) {
        T* ap = reinterpret_cast<T*>(AP + nv) + threadIdx.x;
        T* an = reinterpret_cast<T*>(AN + nv) + threadIdx.x;
        const T bp = reinterpret_cast<const T*>(BP + nv)[threadIdx.x];
        const T bn = reinterpret_cast<const T*>(BN + nv)[threadIdx.x];
        *ap = *ap > bp ? *ap : bp;
        *an = *an > bn ? *an : bn;
    }
}

// Scatter-max: cell (m, c) of the received rows into row keys[m].  ABSENT cells are skipped.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_merge_indexed(typename Elem<EB>::T* __restrict__ AP, typename Elem<EB>::T* __restrict__ AN,
                                                          const typename Elem<EB>::T* __restrict__ BP,
                                                          const typename Elem<EB>::T* __restrict__ BN,
                                                          const uint32_t* __restrict__ keys, uint64_t n_rows, uint32_t R) {
    using T = typename Elem<EB>::T;
    const T absent = EB == 4 ? (T)INT32_MIN : (T)INT64_MIN;
    const uint64_t n = n_rows * R;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t m = i / R, c = i - m * R;
        const uint64_t at = (uint64_t)keys[m] * R + c;
        const T p = BP[i], q = BN[i];
        if (p != absent) atomicMax(AP + at, p);
        if (q != absent) atomicMax(AN + at, q);
    }
}

// The same scatter-max with one wave per received row (lanes over columns): no 64-bit division per
// cell, coalesced row loads and row-contiguous atomics.  Used when a row fills most of a wave (R >= 32).
template <int EB>
__global__ __launch_bounds__(kBlock) void k_merge_indexed_rows(typename Elem<EB>::T* __restrict__ AP, typename Elem<EB>::T* __restrict__ AN,
                                                               const typename Elem<EB>::T* __restrict__ BP,
                                                               const typename Elem<EB>::T* __restrict__ BN,
                                                               const uint32_t* __restrict__ keys, uint64_t n_rows, uint32_t R) {
    using T = typename Elem<EB>::T;
    const T absent = EB == 4 ? (T)INT32_MIN : (T)INT64_MIN;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n_waves = ((uint64_t)gridDim.x * kBlock) >> 6;
    for (uint64_t m = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; m < n_rows; m += n_waves) {
        const uint64_t at = (uint64_t)keys[m] * R, src = m * R;
        for (uint32_t c = lane; c < R; c += 64) {
            const T p = BP[src + c], q = BN[src + c];
            if (p != absent) atomicMax(AP + at + c, p);
            if (q != absent) atomicMax(AN + at + c, q);
        }
    }
}

// Duplicate-aware scatter-max with no atomics on the data, two passes over the batch's keys (a committed
// wave folds several states of one key, SafeCRDTManager.cs:122-146).  Pass 1 (k_group_link) links each
// key's rows into a list: next[m] = the key's previous head, head[key] = gen << 32 | m (one atomicExch per
// row).  Pass 2 (k_merge_grouped): the head row of every key loads its A row once, max-folds every B row of
// the key in registers — each B row's load issued together with its next[] link, so a key held k times
// costs k - 1 dependent hops — and stores A once; the other rows of the key do nothing.  Heads carry the
// batch's generation: a head left by an earlier batch reads as empty, so nothing resets them (the list
// head's `head[key] = kNil` store was one more random write per distinct key: 0.578 -> 0.566 ms per 1M rows,
// tools/tune_grouped.hip).  Atomics ran at ~1.3 TB/s of added bytes on MI355X against ~6 TB/s for plain
// stores (MI355X_MICROARCH.md, atomics table), and random 4-B atomics ~17x slower again: a per-cell
// atomicMax for repeated keys (39 % of the rows of a uniform batch of n rows over 2n keys) and an
// occurrence count per row both measured slower (tools/tune_grouped.hip).  ABSENT (the
// width's minimum) needs no test: max(a, ABSENT) = a.
constexpr uint32_t kNil = 0xFFFFFFFFu;

__global__ __launch_bounds__(kBlock) void k_group_link(const uint32_t* __restrict__ keys, uint64_t n, unsigned long long* __restrict__ head,
                                                       uint32_t* __restrict__ next, unsigned long long gen) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const unsigned long long old = atomicExch(head + keys[i], gen << 32 | i);
        next[i] = (old >> 32) == gen ? (uint32_t)old : kNil;
    }
}

// One wave per received row, U rows in flight; the row (R x EB bytes) is a whole number of 16-B vectors
// and each lane owns the same vector slot(s) of every row it touches.
template <int EB, int U>
__global__ __launch_bounds__(kBlock) void k_merge_grouped(typename Elem<EB>::T* __restrict__ AP, typename Elem<EB>::T* __restrict__ AN,
                                                          const typename Elem<EB>::T* __restrict__ BP,
                                                          const typename Elem<EB>::T* __restrict__ BN, const uint32_t* __restrict__ keys,
                                                          const unsigned long long* __restrict__ head, const uint32_t* __restrict__ next,
                                                          uint64_t n_rows, uint32_t R, unsigned long long gen) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nv = R * EB / 16;  // vectors per array row
    const uint64_t n_waves = ((uint64_t)gridDim.x * kBlock) >> 6;
    for (uint64_t m0 = (((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6) * U; m0 < n_rows; m0 += n_waves * U) {
        uint64_t key[U];
        bool lead[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t m = m0 + u;
            key[u] = m < n_rows ? keys[m] : 0;
            lead[u] = m < n_rows && head[key[u]] == (gen << 32 | m);
        }
        for (uint32_t v = lane; v < 2 * nv; v += 64) {
            const bool isP = v < nv;
            const uint32_t w = isP ? v : v - nv;
            const auto* B = isP ? BP : BN;
            auto* A = isP ? AP : AN;
            uint4 a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (lead[u]) {
                    b[u] = nt_load(reinterpret_cast<const uint4*>(B + (m0 + u) * R) + w);
                    a[u] = *(reinterpret_cast<const uint4*>(A + key[u] * R) + w);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!lead[u]) continue;
                a[u] = vmax<EB>(a[u], b[u]);
                uint64_t hops = 0;  // a list holds at most n_rows - 1 more rows: a bound every walk reaches
                for (uint32_t cur = next[m0 + u]; cur != kNil && ++hops < n_rows;) {  // the key's other rows
                    const uint4 bb = nt_load(reinterpret_cast<const uint4*>(B + (uint64_t)cur * R) + w);
                    const uint32_t nx = next[cur];
                    a[u] = vmax<EB>(a[u], bb);
                    cur = nx;
                }
                *(reinterpret_cast<uint4*>(A + key[u] * R) + w) = a[u];
            }
        }
    }
}

// Row copy (write: keys on the destination side; read: keys on the source side).
template <int EB>
__global__ __launch_bounds__(kBlock) void k_rows_copy(typename Elem<EB>::T* __restrict__ dst, const typename Elem<EB>::T* __restrict__ src,
                                                      const uint32_t* __restrict__ keys, uint64_t n_rows, uint32_t R, int scatter) {
    const uint64_t n = n_rows * R;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t m = i / R, c = i - m * R;
        const uint64_t at = (uint64_t)keys[m] * R + c;
        if (scatter) dst[at] = src[i];
        else dst[i] = src[at];
    }
}

// Increment / Decrement: unchecked '+=' == wrapping add; order-free, so atomics are exact.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_ops(typename Elem<EB>::T* __restrict__ P, typename Elem<EB>::T* __restrict__ N,
                                                      const uint32_t* __restrict__ key, const uint32_t* __restrict__ col,
                                                      const long long* __restrict__ delta, const uint8_t* __restrict__ is_n,
                                                      uint64_t n_ops, uint32_t R) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n_ops; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t at = (uint64_t)key[i] * R + col[i];
        auto* base = is_n[i] ? N : P;
        if constexpr (EB == 4) atomicAdd(reinterpret_cast<unsigned int*>(base + at), (unsigned int)delta[i]);
        else atomicAdd(reinterpret_cast<unsigned long long*>(base + at), (unsigned long long)delta[i]);
    }
}

// ---- PNCounter.Get: checked Sum in column order -------------------------------------------------
template <int EB> struct Acc;
template <> struct Acc<4> { using T = long long; };  // 64 x 2^31 fits easily
template <> struct Acc<8> { using T = __int128; };   // exact for any 64-bit prefix

__device__ __forceinline__ long long shfl_up_acc(long long v, int d) { return __shfl_up(v, d, 64); }
__device__ __forceinline__ __int128 shfl_up_acc(__int128 v, int d) {
    long long lo = (long long)v, hi = (long long)(v >> 64);
    lo = __shfl_up(lo, d, 64);
    hi = __shfl_up(hi, d, 64);
    return ((__int128)hi << 64) | (unsigned long long)lo;
}
__device__ __forceinline__ long long shfl_acc(long long v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ __int128 shfl_acc(__int128 v, int src) {
    long long lo = (long long)v, hi = (long long)(v >> 64);
    lo = __shfl(lo, src, 64);
    hi = __shfl(hi, src, 64);
    return ((__int128)hi << 64) | (unsigned long long)lo;
}

// Returns the exact sum of row[0..R); sets `of` if any prefix leaves T's range.
template <int EB>
__device__ __forceinline__ typename Acc<EB>::T checked_row_sum(const typename Elem<EB>::T* row, uint32_t R, int lane, bool& of) {
    using T = typename Elem<EB>::T;
    using A = typename Acc<EB>::T;
    const A lo = EB == 4 ? (A)INT32_MIN : (A)INT64_MIN;
    const A hi = EB == 4 ? (A)INT32_MAX : (A)INT64_MAX;
    A carry = 0;
    for (uint32_t c0 = 0; c0 < R; c0 += 64) {
        A x = (c0 + lane < R) ? (A)row[c0 + lane] : (A)0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            A y = shfl_up_acc(x, d);
            if (lane >= d) x += y;
        }
        const A pre = carry + x;
        of |= __any(pre < lo || pre > hi) != 0;
        carry = shfl_acc(pre, 63);
    }
    (void)sizeof(T);
    return carry;
}

template <int EB>
__global__ __launch_bounds__(kBlock) void k_values(const typename Elem<EB>::T* __restrict__ P, const typename Elem<EB>::T* __restrict__ N,
                                                   uint32_t R, const uint32_t* __restrict__ keys, uint64_t n,
                                                   long long* __restrict__ out, uint8_t* __restrict__ ovf) {
    using T = typename Elem<EB>::T;
    using UT = std::make_unsigned_t<T>;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * kBlock) >> 6;
    for (uint64_t q = wave; q < n; q += n_waves) {
        const uint64_t k = keys ? keys[q] : q;
        bool of = false;
        const auto sp = checked_row_sum<EB>(P + k * R, R, lane, of);
        const auto sn = checked_row_sum<EB>(N + k * R, R, lane, of);
        if (lane == 0) {
            // ΣP and ΣN are in range when !of; '-' is unchecked: wrap at the width.
            const T v = (T)((UT)(T)sp - (UT)(T)sn);
            out[q] = of ? 0 : (long long)v;
            ovf[q] = of ? 1 : 0;
        }
    }
}

unsigned grid_for(jg_ctx* ctx, uint64_t work_items, unsigned per_cu = 8) {
    uint64_t g = (work_items + kBlock - 1) / kBlock;
    const uint64_t cap = (uint64_t)ctx->num_cus * per_cu;
    if (g > cap) g = cap;
    return g == 0 ? 1u : (unsigned)g;
}

void check_store(const jg_pnc* p, const char* fn) {
    JG_REQUIRE(p, JG_EINVAL, "%s: store is NULL", fn);
}

void check_keys(const uint32_t* k, uint64_t n, uint64_t n_keys, const char* fn) {
    for (uint64_t i = 0; i < n; ++i)
        JG_REQUIRE(k[i] < n_keys, JG_EINVAL, "%s: key_idx[%llu] = %u out of range (n_keys %llu)", fn,
                   (unsigned long long)i, k[i], (unsigned long long)n_keys);
}

// Upload key indices (validated) to ctx scratch.
uint32_t* upload_keys(jg_ctx* ctx, const uint32_t* key_idx, uint64_t n, uint64_t n_keys, const char* fn) {
    check_keys(key_idx, n, n_keys, fn);
    auto* d = static_cast<uint32_t*>(jg::scratch(ctx, ctx->scratch, n * 4));
    JG_HIP(hipMemcpyAsync(d, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
    return d;
}

void launch_merge_dense(jg_ctx* ctx, uint32_t eb, void* AP, void* AN, const void* BP, const void* BN, uint64_t n_cells) {
    const uint64_t bytes = n_cells * eb;
    const uint64_t nv = bytes / 16;
    const uint32_t tail = (uint32_t)((bytes - nv * 16) / eb);
    const uint64_t blocks = (nv + kBlock - 1) / kBlock;
    JG_REQUIRE(blocks < 0xFFFFFFFFull, JG_EINVAL, "merge: %llu cells exceed one launch", (unsigned long long)n_cells);
    const unsigned grid = blocks ? (unsigned)blocks : 1u;
    if (eb == 8)
        hipLaunchKernelGGL(k_merge_dense<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (uint4*)AP, (uint4*)AN, (const uint4*)BP,
                           (const uint4*)BN, nv, tail);
    else
        hipLaunchKernelGGL(k_merge_dense<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (uint4*)AP, (uint4*)AN, (const uint4*)BP,
                           (const uint4*)BN, nv, tail);
    JG_HIP(hipGetLastError());
}

// The store's per-key list heads (generation-tagged) and a next[] link per received row (grown to the
// largest batch); gen = this batch's generation.
struct Groups { unsigned long long* head; uint32_t* next; unsigned long long gen; };

void launch_merge_indexed(jg_ctx* ctx, uint32_t eb, void* AP, void* AN, const void* BP, const void* BN, const uint32_t* keys,
                          uint64_t n_rows, uint32_t R, const Groups* g = nullptr) {
    if (g && R >= 32 && ((uint64_t)R * eb) % 16 == 0) {
        JG_REQUIRE(n_rows < kNil, JG_EINVAL, "merge: %llu rows exceed one grouped launch", (unsigned long long)n_rows);
        const unsigned gk = grid_for(ctx, n_rows, 16);
        hipLaunchKernelGGL(k_group_link, dim3(gk), dim3(kBlock), 0, ctx->stream, keys, n_rows, g->head, g->next, g->gen);
        constexpr int U = 4;  // rows in flight per wave (U = 8 measured slower, tools/tune_grouped.hip)
        const unsigned grid = grid_for(ctx, (n_rows + U - 1) / U * 64, 16);
        if (eb == 8)
            hipLaunchKernelGGL((k_merge_grouped<8, U>), dim3(grid), dim3(kBlock), 0, ctx->stream, (long long*)AP, (long long*)AN,
                               (const long long*)BP, (const long long*)BN, keys, g->head, g->next, n_rows, R, g->gen);
        else
            hipLaunchKernelGGL((k_merge_grouped<4, U>), dim3(grid), dim3(kBlock), 0, ctx->stream, (int*)AP, (int*)AN, (const int*)BP,
                               (const int*)BN, keys, g->head, g->next, n_rows, R, g->gen);
        JG_HIP(hipGetLastError());
        return;
    }
    if (R >= 32) {
        const unsigned grid = grid_for(ctx, n_rows * 64, 16);
        if (eb == 8)
            hipLaunchKernelGGL(k_merge_indexed_rows<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (long long*)AP, (long long*)AN,
                               (const long long*)BP, (const long long*)BN, keys, n_rows, R);
        else
            hipLaunchKernelGGL(k_merge_indexed_rows<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (int*)AP, (int*)AN, (const int*)BP,
                               (const int*)BN, keys, n_rows, R);
        JG_HIP(hipGetLastError());
        return;
    }
    const unsigned grid = grid_for(ctx, n_rows * R, 16);
    if (eb == 8)
        hipLaunchKernelGGL(k_merge_indexed<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (long long*)AP, (long long*)AN,
                           (const long long*)BP, (const long long*)BN, keys, n_rows, R);
    else
        hipLaunchKernelGGL(k_merge_indexed<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (int*)AP, (int*)AN, (const int*)BP,
                           (const int*)BN, keys, n_rows, R);
    JG_HIP(hipGetLastError());
}

// The store's group state for a batch of n_rows (allocated on first use; each grouped merge takes the next
// generation, and the heads are cleared once every 2^32 - 1 batches).  nullptr when rows are too narrow
// for the vector path.
const Groups* groups_of(jg_pnc* p, uint64_t n_rows, Groups& g) {
    if (p->R < 32 || ((uint64_t)p->R * p->eb) % 16 != 0) return nullptr;
    if (!p->head.p || p->head_gen == 0xFFFFFFFFull) {
        const bool first = !p->head.p;
        if (first) p->head.alloc(p->n_keys * 8);
        JG_HIP(hipMemsetAsync(p->head.p, 0, p->n_keys * 8, p->ctx->stream));
        p->head_gen = 0;
        // JANUS_TEST_HEAD_GEN: a new store's first generation (tests run batches across the wrap)
        const char* e = first ? std::getenv("JANUS_TEST_HEAD_GEN") : nullptr;
        // clamped below 2^32 - 1: the increment below then gives 1 .. 2^32 - 1, never 0 or 2^32 (a generation
        // whose low 32 bits read 0 would make every head look old)
        if (e) p->head_gen = std::min<unsigned long long>(std::strtoull(e, nullptr, 10), 0xFFFFFFFEull);
    }
    ++p->head_gen;
    if (p->next.bytes < n_rows * 4) {
        JG_HIP(hipStreamSynchronize(p->ctx->stream));  // an earlier launch may still read the old links
        p->next.alloc(n_rows * 4 + n_rows);
    }
    g = Groups{p->head.as<unsigned long long>(), p->next.as<uint32_t>(), p->head_gen};
    return &g;
}

void launch_rows_copy(jg_ctx* ctx, uint32_t eb, void* dst, const void* src, const uint32_t* keys, uint64_t n_rows, uint32_t R,
                      int scatter) {
    const unsigned grid = grid_for(ctx, n_rows * R, 16);
    if (eb == 8)
        hipLaunchKernelGGL(k_rows_copy<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (long long*)dst, (const long long*)src, keys,
                           n_rows, R, scatter);
    else
        hipLaunchKernelGGL(k_rows_copy<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (int*)dst, (const int*)src, keys, n_rows, R,
                           scatter);
    JG_HIP(hipGetLastError());
}

}  // namespace

void jg::pnc_merge_indexed(jg_pnc* p, const void* BP, const void* BN, const uint32_t* d_keys, uint64_t n_rows) {
    Groups g;
    launch_merge_indexed(p->ctx, p->eb, p->P.p, p->N.p, BP, BN, d_keys, n_rows, p->R, groups_of(p, n_rows, g));
}

extern "C" {

int jg_pnc_create(jg_ctx* ctx, uint64_t n_keys, uint32_t n_replicas, uint32_t elem_bytes, jg_pnc** out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_pnc_create: NULL argument");
        JG_REQUIRE(elem_bytes == 4 || elem_bytes == 8, JG_EINVAL, "jg_pnc_create: elem_bytes must be 4 or 8");
        JG_REQUIRE(n_replicas > 0 && n_keys > 0, JG_EINVAL, "jg_pnc_create: empty shape");
        JG_REQUIRE(n_keys <= 0xFFFFFFFFull, JG_EINVAL, "jg_pnc_create: key_idx is 32-bit");
        jg::ensure_device(ctx);
        auto* p = new jg_pnc();
        p->ctx = ctx; p->n_keys = n_keys; p->R = n_replicas; p->eb = elem_bytes;
        try {
            const size_t bytes = (size_t)n_keys * n_replicas * elem_bytes;
            p->P.alloc(bytes);
            p->N.alloc(bytes);
            JG_HIP(hipMemsetAsync(p->P.p, 0, bytes, ctx->stream));  // PNCounter(): every replica absent = 0
            JG_HIP(hipMemsetAsync(p->N.p, 0, bytes, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
        } catch (...) {
            delete p;
            throw;
        }
        *out = p;
    });
}

int jg_pnc_destroy(jg_pnc* p) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_destroy");
        if (!p) return;
        jg::ensure_device(p->ctx);
        JG_HIP(hipStreamSynchronize(p->ctx->stream));
        delete p;
    });
}

int jg_pnc_write_rows(jg_pnc* p, const uint32_t* key_idx, uint64_t n_rows, const void* P, const void* N) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_write_rows");
        check_store(p, "jg_pnc_write_rows");
        JG_REQUIRE(P && N, JG_EINVAL, "jg_pnc_write_rows: NULL rows");
        if (n_rows == 0) return;
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const size_t bytes = (size_t)n_rows * p->R * p->eb;
        if (!key_idx) {
            JG_REQUIRE(n_rows <= p->n_keys, JG_EINVAL, "jg_pnc_write_rows: %llu rows > n_keys", (unsigned long long)n_rows);
            JG_HIP(hipMemcpyAsync(p->P.p, P, bytes, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync(p->N.p, N, bytes, hipMemcpyHostToDevice, ctx->stream));
        } else {
            const uint32_t* dk = upload_keys(ctx, key_idx, n_rows, p->n_keys, "jg_pnc_write_rows");
            void* st = jg::scratch(ctx, ctx->scratch2, 2 * bytes);
            JG_HIP(hipMemcpyAsync(st, P, bytes, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync((char*)st + bytes, N, bytes, hipMemcpyHostToDevice, ctx->stream));
            launch_rows_copy(ctx, p->eb, p->P.p, st, dk, n_rows, p->R, 1);
            launch_rows_copy(ctx, p->eb, p->N.p, (char*)st + bytes, dk, n_rows, p->R, 1);
        }
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_read_rows(jg_pnc* p, const uint32_t* key_idx, uint64_t n_rows, void* P, void* N) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        check_store(p, "jg_pnc_read_rows");
        JG_REQUIRE(P && N, JG_EINVAL, "jg_pnc_read_rows: NULL rows");
        if (n_rows == 0) return;
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const size_t bytes = (size_t)n_rows * p->R * p->eb;
        if (!key_idx) {
            JG_REQUIRE(n_rows <= p->n_keys, JG_EINVAL, "jg_pnc_read_rows: %llu rows > n_keys", (unsigned long long)n_rows);
            JG_HIP(hipMemcpyAsync(P, p->P.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipMemcpyAsync(N, p->N.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
        } else {
            const uint32_t* dk = upload_keys(ctx, key_idx, n_rows, p->n_keys, "jg_pnc_read_rows");
            void* st = jg::scratch(ctx, ctx->scratch2, 2 * bytes);
            launch_rows_copy(ctx, p->eb, st, p->P.p, dk, n_rows, p->R, 0);
            launch_rows_copy(ctx, p->eb, (char*)st + bytes, p->N.p, dk, n_rows, p->R, 0);
            JG_HIP(hipMemcpyAsync(P, st, bytes, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipMemcpyAsync(N, (char*)st + bytes, bytes, hipMemcpyDeviceToHost, ctx->stream));
        }
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_merge_rows(jg_pnc* p, const uint32_t* key_idx, uint64_t n_rows, const void* P, const void* N) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_merge_rows");
        check_store(p, "jg_pnc_merge_rows");
        JG_REQUIRE(P && N, JG_EINVAL, "jg_pnc_merge_rows: NULL rows");
        if (n_rows == 0) return;
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const size_t bytes = (size_t)n_rows * p->R * p->eb;
        const uint32_t* dk = nullptr;
        if (key_idx) dk = upload_keys(ctx, key_idx, n_rows, p->n_keys, "jg_pnc_merge_rows");
        else JG_REQUIRE(n_rows <= p->n_keys, JG_EINVAL, "jg_pnc_merge_rows: %llu rows > n_keys", (unsigned long long)n_rows);
        void* st = jg::scratch(ctx, ctx->scratch2, 2 * bytes);
        JG_HIP(hipMemcpyAsync(st, P, bytes, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync((char*)st + bytes, N, bytes, hipMemcpyHostToDevice, ctx->stream));
        Groups g;
        if (dk) launch_merge_indexed(ctx, p->eb, p->P.p, p->N.p, st, (char*)st + bytes, dk, n_rows, p->R, groups_of(p, n_rows, g));
        else launch_merge_dense(ctx, p->eb, p->P.p, p->N.p, st, (char*)st + bytes, n_rows * p->R);
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_apply_ops(jg_pnc* p, uint64_t n_ops, const uint32_t* key, const uint32_t* col, const int64_t* delta, const uint8_t* is_n) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_apply_ops");
        check_store(p, "jg_pnc_apply_ops");
        if (n_ops == 0) return;
        JG_REQUIRE(key && col && delta && is_n, JG_EINVAL, "jg_pnc_apply_ops: NULL argument");
        for (uint64_t i = 0; i < n_ops; ++i)
            JG_REQUIRE(key[i] < p->n_keys && col[i] < p->R, JG_EINVAL, "jg_pnc_apply_ops: op %llu addresses (%u,%u) outside the store",
                       (unsigned long long)i, key[i], col[i]);
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch2, n_ops * 17 + 64));
        uint32_t* dkey = (uint32_t*)st;
        uint32_t* dcol = (uint32_t*)(st + n_ops * 4);
        long long* ddel = (long long*)(st + ((n_ops * 8 + 15) & ~15ull));
        uint8_t* dn = (uint8_t*)(ddel + n_ops);
        JG_HIP(hipMemcpyAsync(dkey, key, n_ops * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(dcol, col, n_ops * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(ddel, delta, n_ops * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(dn, is_n, n_ops, hipMemcpyHostToDevice, ctx->stream));
        const unsigned grid = grid_for(ctx, n_ops, 16);
        if (p->eb == 8)
            hipLaunchKernelGGL(k_apply_ops<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (long long*)p->P.p, (long long*)p->N.p, dkey,
                               dcol, ddel, dn, n_ops, p->R);
        else
            hipLaunchKernelGGL(k_apply_ops<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (int*)p->P.p, (int*)p->N.p, dkey, dcol, ddel,
                               dn, n_ops, p->R);
        JG_HIP(hipGetLastError());
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_values(jg_pnc* p, const uint32_t* key_idx, uint64_t n, int64_t* out, uint8_t* overflow) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        check_store(p, "jg_pnc_values");
        JG_REQUIRE(out && overflow, JG_EINVAL, "jg_pnc_values: NULL output");
        if (n == 0) return;
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const uint32_t* dk = nullptr;
        if (key_idx) dk = upload_keys(ctx, key_idx, n, p->n_keys, "jg_pnc_values");
        else JG_REQUIRE(n <= p->n_keys, JG_EINVAL, "jg_pnc_values: %llu keys > n_keys", (unsigned long long)n);
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch2, n * 9 + 64));
        long long* dout = (long long*)st;
        uint8_t* dovf = (uint8_t*)(st + n * 8);
        const unsigned grid = grid_for(ctx, n * 64, 16);
        if (p->eb == 8)
            hipLaunchKernelGGL(k_values<8>, dim3(grid), dim3(kBlock), 0, ctx->stream, (const long long*)p->P.p, (const long long*)p->N.p,
                               p->R, dk, n, dout, dovf);
        else
            hipLaunchKernelGGL(k_values<4>, dim3(grid), dim3(kBlock), 0, ctx->stream, (const int*)p->P.p, (const int*)p->N.p, p->R, dk,
                               n, dout, dovf);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(overflow, dovf, n, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_rows_create(jg_ctx* ctx, uint64_t n_rows, uint32_t n_replicas, uint32_t elem_bytes, jg_rows** out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_rows_create: NULL argument");
        JG_REQUIRE(elem_bytes == 4 || elem_bytes == 8, JG_EINVAL, "jg_rows_create: elem_bytes must be 4 or 8");
        JG_REQUIRE(n_rows > 0 && n_replicas > 0, JG_EINVAL, "jg_rows_create: empty shape");
        jg::ensure_device(ctx);
        auto* r = new jg_rows();
        r->ctx = ctx; r->n_rows = n_rows; r->R = n_replicas; r->eb = elem_bytes;
        try {
            const size_t bytes = (size_t)n_rows * n_replicas * elem_bytes;
            r->P.alloc(bytes);
            r->N.alloc(bytes);
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
    });
}

int jg_rows_destroy(jg_rows* r) {
    return jg::guard([&] {
        auto lk_ = jg::lock(r);  // calls on one context are serialised (shared scratch, stream)
        if (!r) return;
        jg::ensure_device(r->ctx);
        JG_HIP(hipStreamSynchronize(r->ctx->stream));
        delete r;
    });
}

int jg_rows_upload(jg_rows* r, const uint32_t* key_idx, const void* P, const void* N) {
    return jg::guard([&] {
        auto lk_ = jg::lock(r);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(r && P && N, JG_EINVAL, "jg_rows_upload: NULL argument");
        jg_ctx* ctx = r->ctx;
        jg::ensure_device(ctx);
        const size_t bytes = (size_t)r->n_rows * r->R * r->eb;
        JG_HIP(hipMemcpyAsync(r->P.p, P, bytes, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(r->N.p, N, bytes, hipMemcpyHostToDevice, ctx->stream));
        if (key_idx) {
            uint32_t mx = 0;
            for (uint64_t i = 0; i < r->n_rows; ++i) mx = key_idx[i] > mx ? key_idx[i] : mx;
            r->max_key = mx;
            if (r->keys.bytes < r->n_rows * 4) r->keys.alloc(r->n_rows * 4);
            JG_HIP(hipMemcpyAsync(r->keys.p, key_idx, r->n_rows * 4, hipMemcpyHostToDevice, ctx->stream));
            r->has_keys = true;
        } else {
            r->has_keys = false;
        }
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_merge_batch(jg_pnc* p, const jg_rows* r, int async) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_merge_batch");
        check_store(p, "jg_pnc_merge_batch");
        JG_REQUIRE(r, JG_EINVAL, "jg_pnc_merge_batch: rows is NULL");
        JG_REQUIRE(r->ctx == p->ctx, JG_EINVAL, "jg_pnc_merge_batch: rows and store belong to different contexts");
        JG_REQUIRE(r->R == p->R && r->eb == p->eb, JG_ETYPE, "jg_pnc_merge_batch: row shape (%u x %uB) != store (%u x %uB)", r->R, r->eb,
                   p->R, p->eb);
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        if (r->has_keys) {
            JG_REQUIRE(r->max_key < p->n_keys, JG_EINVAL, "jg_pnc_merge_batch: batch addresses key %u >= n_keys %llu", r->max_key,
                       (unsigned long long)p->n_keys);
            Groups g;
            launch_merge_indexed(ctx, p->eb, p->P.p, p->N.p, r->P.p, r->N.p, r->keys.as<uint32_t>(), r->n_rows, p->R, groups_of(p, r->n_rows, g));
        } else {
            JG_REQUIRE(r->n_rows <= p->n_keys, JG_EINVAL, "jg_pnc_merge_batch: identity batch of %llu rows > n_keys",
                       (unsigned long long)r->n_rows);
            launch_merge_dense(ctx, p->eb, p->P.p, p->N.p, r->P.p, r->N.p, r->n_rows * p->R);
        }
        if (!async) JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

}  // extern "C"
