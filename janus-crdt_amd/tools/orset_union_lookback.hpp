// orset_union.hpp — OR-Set stream-union kernels (merge path + decoupled look-back), templated on
// the workgroup size and records per thread so the production build (orset.hip) and the tuning tool
// (tools/tune_orset.hip) compile the same code.  See orset.hip for the algorithm summary.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace jgk {


constexpr unsigned long long kFlagAgg = 1ull << 62;
constexpr unsigned long long kFlagIncl = 2ull << 62;
constexpr unsigned long long kValMask = (1ull << 62) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

struct Tag { unsigned long long lo, hi; };

__device__ __forceinline__ Tag ld_tag(const uint4* p) { return __builtin_bit_cast(Tag, *p); }
__device__ __forceinline__ uint4 to_u4(Tag t) { return __builtin_bit_cast(uint4, t); }

// Branch-free lexicographic compare on (key, tag.lo, tag.hi), unsigned.
__device__ __forceinline__ bool rec_lt(unsigned long long ka, Tag ta, unsigned long long kb, Tag tb) {
    return (ka < kb) | ((ka == kb) & ((ta.lo < tb.lo) | ((ta.lo == tb.lo) & (ta.hi < tb.hi))));
}
__device__ __forceinline__ bool rec_eq(unsigned long long ka, Tag ta, unsigned long long kb, Tag tb) {
    return (ka == kb) & (ta.lo == tb.lo) & (ta.hi == tb.hi);
}

// Merge-path split for diagonal d over (a, b): number of A records among the first d merged.
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_partition(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                                   const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                                   uint64_t n_parts, uint64_t* __restrict__ part) {
    constexpr int kTile = kOB * kItems;
    const uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x;
    if (i >= n_parts) return;
    const uint64_t total = na + nb;
    const uint64_t d = i * kTile < total ? i * kTile : total;
    uint64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const unsigned long long ka = ak[mid], kb = bk[d - 1 - mid];
        bool a_le_b;  // a[mid] <= b[d-1-mid]  -> take more from A
        if (ka != kb) a_le_b = ka < kb;
        else a_le_b = !rec_lt(kb, ld_tag(bt + d - 1 - mid), ka, ld_tag(at + mid));
        if (a_le_b) lo = mid + 1;
        else hi = mid;
    }
    part[i] = lo;
}

// Wave 0 of a tile: sum the counts of all earlier tiles (decoupled look-back).  kLB windows of 64
// predecessors are fetched per round trip (one status word per lane and window); a window is only
// re-polled while some of its tiles have not published yet.
template <int kLB>
__device__ inline unsigned long long lookback(unsigned long long* status, long long tile, int lane, unsigned* err) {
    unsigned long long excl = 0;
    long long base = tile - 1;
    unsigned spins = 0;
    for (;;) {
        unsigned long long w[kLB];
#pragma unroll
        for (int j = 0; j < kLB; ++j) {
            const long long idx = base - 64 * j - lane;
            w[j] = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
        }
#pragma unroll
        for (int j = 0; j < kLB; ++j) {
            const long long idx = base - 64 * j - lane;
            while (!__all((w[j] >> 62) != 0)) {
                if (++spins > kSpinLimit) {  // wave-uniform: give up, flag the call, let the grid drain
                    if (lane == 0) atomicOr(err, 1u);
                    w[j] = kFlagIncl;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                w[j] = idx >= 0 ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
            }
            const unsigned long long incl = __ballot((w[j] >> 62) == 2);
            const int first = incl ? __ffsll((long long)incl) - 1 : 64;
            unsigned long long v = lane <= first ? (w[j] & kValMask) : 0ull;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            excl += v;
            if (incl) return excl;
        }
        base -= 64 * kLB;
    }
}

// ---- one tile of the union, split into phases so the one-shot and the persistent kernels share it ----
struct TileBounds {
    uint64_t i0, j0;  // first A / B record of the tile
    int nA, nB;       // records of A / B in the tile
};

template <int kOB, int kItems>
__device__ __forceinline__ TileBounds tile_bounds(uint64_t tile, const uint64_t* __restrict__ part, uint64_t na, uint64_t nb) {
    constexpr uint64_t kTile = (uint64_t)kOB * kItems;
    const uint64_t total = na + nb;
    const uint64_t d0 = tile * kTile;
    const uint64_t d1 = d0 + kTile < total ? d0 + kTile : total;
    const uint64_t i0 = part[tile], i1 = part[tile + 1];
    TileBounds b;
    b.i0 = i0;
    b.j0 = d0 - i0;
    b.nA = (int)(i1 - i0);
    b.nB = (int)((d1 - i1) - b.j0);
    return b;
}

// A tile's records held in registers between the global loads and the LDS writes (scalar arrays:
// they stay in VGPRs; arrays of uint4 went to scratch).
template <int kItems>
struct TileRegs {
    unsigned long long k[kItems], lo[kItems], hi[kItems];
    unsigned long long pk, plo, phi;  // A record before the tile (thread 0 only)
};

// Issue every global load of the tile (unconditional: index clamped into the tile, n >= 1).
template <int kOB, int kItems>
__device__ __forceinline__ void tile_load(TileRegs<kItems>& r, const TileBounds& b, const unsigned long long* __restrict__ ak,
                                          const uint4* __restrict__ at, const unsigned long long* __restrict__ bk,
                                          const uint4* __restrict__ bt, int tid) {
    const int n = b.nA + b.nB;
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
        const int x = min(it * kOB + tid, n - 1);
        const bool from_a = x < b.nA;
        const uint64_t gi = from_a ? b.i0 + (uint64_t)x : b.j0 + (uint64_t)(x - b.nA);
        r.k[it] = (from_a ? ak : bk)[gi];
        const Tag t = ld_tag((from_a ? at : bt) + gi);
        r.lo[it] = t.lo;
        r.hi[it] = t.hi;
    }
    if (tid == 0 && b.i0 > 0) {
        r.pk = ak[b.i0 - 1];
        const Tag t = ld_tag(at + b.i0 - 1);
        r.plo = t.lo;
        r.phi = t.hi;
    }
}

// Set-indexed drop bitmap (ORSet.Clear applied inside a batch of ops): A-side records whose set bit
// is 1 are removed from the union.  nullptr = keep everything.
__device__ __forceinline__ bool dropped(const unsigned* drop, unsigned long long key) {
    if (!drop) return false;
    const unsigned set = (unsigned)(key >> 32);
    return (drop[set >> 5] >> (set & 31)) & 1u;
}

struct TileLds {
    unsigned long long* key;
    uint4* tag;
    unsigned long long* prev_key;
    uint4* prev_tag;
    int* has_prev;
    unsigned long long* excl;
    int* wsum;
};

template <int kOB, int kItems>
__device__ __forceinline__ void tile_stage(const TileRegs<kItems>& r, const TileBounds& b, const TileLds& L, int tid,
                                           const unsigned* drop = nullptr) {
#pragma unroll
    for (int it = 0; it < kItems; ++it) {  // slots >= n get a duplicate; never read
        const int x = it * kOB + tid;
        L.key[x] = r.k[it];
        L.tag[x] = to_u4(Tag{r.lo[it], r.hi[it]});
    }
    if (tid == 0) {
        *L.has_prev = b.i0 > 0 && !dropped(drop, r.pk);
        if (b.i0 > 0) { *L.prev_key = r.pk; *L.prev_tag = to_u4(Tag{r.plo, r.phi}); }
    }
}

struct NoStamp {
    __device__ __forceinline__ void operator()(int) const {}
};

// Merge, de-duplicate, scan, look back, compact and store one staged tile.  Called by the whole
// workgroup after a barrier that follows tile_stage; ends with the LDS image read for the stores.
// `stamp(i)` marks phase boundaries in the diagnostic build (tools/tune_orset.hip); a no-op here.
template <int kOB, int kItems, class Stamp = NoStamp, int kLB = 1>
__device__ __forceinline__ void tile_process(uint64_t tile, const TileBounds& b, uint64_t n_tiles, const TileLds& L,
                                             unsigned long long* __restrict__ ok, uint4* __restrict__ ot, unsigned long long* status,
                                             unsigned long long* out_count, unsigned* err, int tid, const Stamp& stamp = Stamp(),
                                             const unsigned* drop = nullptr) {
    const int lane = tid & 63, wid = tid >> 6;
    const int nA = b.nA, nB = b.nB, n = nA + nB;
    unsigned long long* s_key = L.key;
    uint4* s_tag = L.tag;

    // ---- per-thread merge path + serial merge of kItems outputs ----
    const int diag = min(tid * kItems, n);
    int lo = diag > nB ? diag - nB : 0, hi = min(diag, nA);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int bj = nA + diag - 1 - mid;
        const bool a_le_b = !rec_lt(s_key[bj], __builtin_bit_cast(Tag, s_tag[bj]), s_key[mid], __builtin_bit_cast(Tag, s_tag[mid]));
        if (a_le_b) lo = mid + 1;
        else hi = mid;
    }
    stamp(4);
    int ai = lo, bi = diag - lo;
    bool hp;
    unsigned long long pk;
    Tag pt;
    // hp: the A record just before the next B record in merged order exists and survives the drop
    // filter (a B record can only equal that one, since A and B are strictly increasing).
    if (ai > 0) { pk = s_key[ai - 1]; pt = __builtin_bit_cast(Tag, s_tag[ai - 1]); hp = !dropped(drop, pk); }
    else { hp = *L.has_prev != 0; pk = *L.prev_key; pt = __builtin_bit_cast(Tag, *L.prev_tag); }

    const int my_n = n - diag < kItems ? n - diag : kItems;
    unsigned long long ka = 0, kb = 0;
    Tag ta{0, 0}, tb{0, 0};
    if (ai < nA) { ka = s_key[ai]; ta = __builtin_bit_cast(Tag, s_tag[ai]); }
    if (bi < nB) { kb = s_key[nA + bi]; tb = __builtin_bit_cast(Tag, s_tag[nA + bi]); }
    int src[kItems];
    unsigned keep = 0;
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
        src[it] = 0;
        if (it < my_n) {
            const bool take_a = ai < nA && (bi >= nB || !rec_lt(kb, tb, ka, ta));
            if (take_a) {
                src[it] = ai;
                hp = !dropped(drop, ka);
                if (hp) keep |= 1u << it;
                pk = ka; pt = ta;
                ++ai;
                if (ai < nA) { ka = s_key[ai]; ta = __builtin_bit_cast(Tag, s_tag[ai]); }
            } else {
                src[it] = nA + bi;
                if (!(hp && rec_eq(pk, pt, kb, tb))) keep |= 1u << it;
                ++bi;
                if (bi < nB) { kb = s_key[nA + bi]; tb = __builtin_bit_cast(Tag, s_tag[nA + bi]); }
            }
        }
    }

    stamp(5);
    // ---- block scan of kept counts ----
    const int cnt = __popc(keep);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    if (lane == 63) L.wsum[wid] = incl;
    __syncthreads();
    int wbase = 0, block_total = 0;
#pragma unroll
    for (int w = 0; w < kOB / 64; ++w) {
        const int v = L.wsum[w];
        if (w < wid) wbase += v;
        block_total += v;
    }
    const int my_off = wbase + incl - cnt;
    stamp(6);

    // ---- publish and look back (wave 0) ----
    if (kLB == 0) {  // chunked-output experiment (tools/): tile t owns output slots [t*kTile, t*kTile + total)
        if (tid == 0) *L.excl = tile * (unsigned long long)(kOB * kItems);
    } else if (wid == 0) {
        unsigned long long excl = 0;
        if (tile == 0) {
            if (lane == 0) __hip_atomic_store(status, kFlagIncl | (unsigned long long)block_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(status + tile, kFlagAgg | (unsigned long long)block_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            excl = lookback<(kLB > 0 ? kLB : 1)>(status, (long long)tile, lane, err);
            if (lane == 0)
                __hip_atomic_store(status + tile, kFlagIncl | (excl + (unsigned long long)block_total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            *L.excl = excl;
            if (tile == n_tiles - 1) *out_count = excl + (unsigned long long)block_total;
        }
    }

    stamp(7);
    // ---- gather kept records, compact through LDS, store coalesced ----
    unsigned long long rk[kItems], rlo[kItems], rhi[kItems];
#pragma unroll
    for (int it = 0; it < kItems; ++it) {  // src[it] is a valid LDS index even for dropped items
        rk[it] = s_key[src[it]];
        const Tag t = __builtin_bit_cast(Tag, s_tag[src[it]]);
        rlo[it] = t.lo;
        rhi[it] = t.hi;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
        if (keep & (1u << it)) {
            const int o = my_off + __popc(keep & ((1u << it) - 1u));
            s_key[o] = rk[it];
            s_tag[o] = to_u4(Tag{rlo[it], rhi[it]});
        }
    }
    __syncthreads();
    stamp(8);
    const unsigned long long base = *L.excl;
    for (int x = tid; x < block_total; x += kOB) {
        ok[base + x] = s_key[x];
        ot[base + x] = s_tag[x];
    }
    stamp(9);
}

#define JGK_TILE_LDS(kOB, kItems)                                                                          \
    __shared__ unsigned long long s_key[(kOB) * (kItems)];                                                 \
    __shared__ uint4 s_tag[(kOB) * (kItems)];                                                              \
    __shared__ unsigned long long s_prev_key, s_excl;                                                      \
    __shared__ uint4 s_prev_tag;                                                                           \
    __shared__ int s_has_prev;                                                                             \
    __shared__ unsigned s_tile;                                                                            \
    __shared__ int s_wsum[(kOB) / 64];                                                                     \
    const TileLds L{s_key, s_tag, &s_prev_key, &s_prev_tag, &s_has_prev, &s_excl, s_wsum}

// One tile per workgroup; grid = n_tiles.  Tickets (not blockIdx) order the tiles, so a tile only
// ever waits for tiles already owned by running workgroups.
template <int kOB, int kItems, int kLB = 1>
__global__ __launch_bounds__(kOB) void k_union(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                               const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                               const uint64_t* __restrict__ part, uint64_t n_tiles,
                                               unsigned long long* __restrict__ ok, uint4* __restrict__ ot,
                                               unsigned long long* status, unsigned* ticket, unsigned long long* out_count,
                                               unsigned* err, const unsigned* __restrict__ drop = nullptr) {
    JGK_TILE_LDS(kOB, kItems);
    const int tid = threadIdx.x;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t tile = s_tile;
    const TileBounds b = tile_bounds<kOB, kItems>(tile, part, na, nb);
    TileRegs<kItems> r;
    tile_load<kOB, kItems>(r, b, ak, at, bk, bt, tid);
    tile_stage<kOB, kItems>(r, b, L, tid, drop);
    __syncthreads();
    tile_process<kOB, kItems, NoStamp, kLB>(tile, b, n_tiles, L, ok, ot, status, out_count, err, tid, NoStamp(), drop);
}

// Persistent variant: each workgroup loops over tickets and loads tile t+1 into registers while it
// merges tile t.  A workgroup takes ticket t+1 before finishing t; the smallest unfinished tile is
// always some workgroup's current tile, which waits only on finished ones, so progress holds.
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_union_pp(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                                  const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                                  const uint64_t* __restrict__ part, uint64_t n_tiles,
                                                  unsigned long long* __restrict__ ok, uint4* __restrict__ ot,
                                                  unsigned long long* status, unsigned* ticket, unsigned long long* out_count,
                                                  unsigned* err) {
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
        tile_stage<kOB, kItems>(r, b, L, tid);
        if (tid == 0) s_tile = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint64_t next = s_tile;
        TileBounds nb2{0, 0, 0, 0};
        if (next < n_tiles) {
            nb2 = tile_bounds<kOB, kItems>(next, part, na, nb);
            tile_load<kOB, kItems>(r, nb2, ak, at, bk, bt, tid);
        }
        tile_process<kOB, kItems>(tile, b, n_tiles, L, ok, ot, status, out_count, err, tid);
        if (next >= n_tiles) break;
        tile = next;
        b = nb2;
        __syncthreads();  // every wave's stores read the LDS image before it is restaged
    }
}

// Persistent, statically assigned variant: workgroup b owns tiles b, b+G, b+2G, ... (G = grid) and
// loads its next tile into registers while it merges the current one.  Tile t only waits on
// lower tiles, all owned by co-resident workgroups that process theirs in increasing order, so
// the grid MUST be fully resident (G <= resident workgroups); the bounded spin flags a violation.
template <int kOB, int kItems, int kLB = 1>
__global__ __launch_bounds__(kOB) void k_union_ps(const unsigned long long* __restrict__ ak, const uint4* __restrict__ at, uint64_t na,
                                                  const unsigned long long* __restrict__ bk, const uint4* __restrict__ bt, uint64_t nb,
                                                  const uint64_t* __restrict__ part, uint64_t n_tiles,
                                                  unsigned long long* __restrict__ ok, uint4* __restrict__ ot,
                                                  unsigned long long* status, unsigned* ticket, unsigned long long* out_count,
                                                  unsigned* err) {
    JGK_TILE_LDS(kOB, kItems);
    (void)ticket;
    (void)s_tile;
    const int tid = threadIdx.x;
    uint64_t tile = blockIdx.x;
    if (tile >= n_tiles) return;
    TileBounds b = tile_bounds<kOB, kItems>(tile, part, na, nb);
    TileRegs<kItems> r;
    tile_load<kOB, kItems>(r, b, ak, at, bk, bt, tid);
    for (;;) {
        tile_stage<kOB, kItems>(r, b, L, tid);
        __syncthreads();
        const uint64_t next = tile + gridDim.x;
        TileBounds nb2{0, 0, 0, 0};
        if (next < n_tiles) {
            nb2 = tile_bounds<kOB, kItems>(next, part, na, nb);
            tile_load<kOB, kItems>(r, nb2, ak, at, bk, bt, tid);
        }
        tile_process<kOB, kItems, NoStamp, kLB>(tile, b, n_tiles, L, ok, ot, status, out_count, err, tid);
        if (next >= n_tiles) break;
        tile = next;
        b = nb2;
        __syncthreads();  // every wave's stores read the LDS image before it is restaged
    }
}

}  // namespace jgk
