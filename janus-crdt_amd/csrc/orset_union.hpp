// orset_union.hpp — OR-Set record streams in the CHUNKED layout, and their union kernels.
//
// A stream is sorted strictly increasing by (key, tag.lo, tag.hi) in RANK space, stored in chunks of
// C slots: chunk c holds ranks [off[c], off[c+1]) in slots [c*C, c*C + cnt[c]).  A union tile writes
// its output straight into its own chunk, so no workgroup ever waits on another: the contiguous
// layout needed a decoupled look-back that measured 32-36 % of every tile and 57 % more kernel time
// (the look-back tool was removed in round 2; DESIGN.md §4 keeps its numbers).  Readers translate rank -> slot with a lookup table:
// lut[q] = the last chunk starting at or before rank q * 512, so the chunk of rank r lies in
// [lut[r >> 9], lut[(r >> 9) + 1]] — usually one candidate, a short binary search when a Clear left
// empty chunks behind.
//
// Templated on the workgroup size and records per thread so the production build (orset.hip) and
// the tuning tool (tools/tune_orset.hip) compile the same code.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace jgk {

constexpr int kQShift = 9;  // LUT granularity: one entry per 512 ranks

struct Tag { unsigned long long lo, hi; };

__device__ __forceinline__ Tag ld_tag(const uint4* p) { return __builtin_bit_cast(Tag, *p); }
typedef unsigned int nt_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Tag ld_tag_nt(const uint4* p) {
    return __builtin_bit_cast(Tag, __builtin_nontemporal_load(reinterpret_cast<const nt_v4u*>(p)));
}
// Streams' records read through global-address-space pointers: a pointer picked per lane between two
// streams is otherwise generic (a FLAT load, which also counts on lgkmcnt).
template <class T>
using gptr = const __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr<T> as_global(const T* p) { return (gptr<T>)p; }
__device__ __forceinline__ Tag ld_tag_nt(gptr<uint4> p) {
    return __builtin_bit_cast(Tag, __builtin_nontemporal_load((gptr<nt_v4u>)p));
}
__device__ __forceinline__ void st_tag_nt(uint4* p, uint4 v) {
    __builtin_nontemporal_store(__builtin_bit_cast(nt_v4u, v), reinterpret_cast<nt_v4u*>(p));
}
__device__ __forceinline__ uint4 to_u4(Tag t) { return __builtin_bit_cast(uint4, t); }

// Branch-free lexicographic compare on (key, tag.lo, tag.hi), unsigned.
__device__ __forceinline__ bool rec_lt(unsigned long long ka, Tag ta, unsigned long long kb, Tag tb) {
    return (ka < kb) | ((ka == kb) & ((ta.lo < tb.lo) | ((ta.lo == tb.lo) & (ta.hi < tb.hi))));
}
__device__ __forceinline__ bool rec_eq(unsigned long long ka, Tag ta, unsigned long long kb, Tag tb) {
    return (ka == kb) & (ta.lo == tb.lo) & (ta.hi == tb.hi);
}

// Read view of one chunked stream (plain pointers: passed by value to kernels).
struct View {
    const unsigned long long* key;
    const uint4* tag;
    const uint32_t* ord;  // arrival ordinals (jg_tagrec.ord); only the union reads them
    const uint64_t* off;  // [nch + 1]
    const uint32_t* lut;  // [(n >> kQShift) + 2]
    uint64_t n;
    uint32_t nch;
    uint32_t C;
    uint32_t dense;  // 1: off[c] = c*C (slot = rank), set for uploaded and generated streams
};

__device__ __forceinline__ uint32_t chunk_of(const View& v, uint64_t r) {  // r < n: the last chunk with off <= r
    if (v.dense) return (uint32_t)(r / v.C);
    const uint64_t q = r >> kQShift;
    uint32_t lo = v.lut[q], hi = v.lut[q + 1];
    while (lo < hi) {
        const uint32_t m = (lo + hi + 1) >> 1;
        if (v.off[m] <= r) lo = m;
        else hi = m - 1;
    }
    return lo;
}
__device__ __forceinline__ uint64_t slot_of(const View& v, uint64_t r) {
    if (v.dense) return r;
    const uint32_t c = chunk_of(v, r);
    return (uint64_t)c * v.C + (r - v.off[c]);
}

// Set-indexed drop bitmap (ORSet.Clear applied inside a batch of ops): A-side records whose set bit
// is 1 are removed from the union; sets past the bitmap's `words` are kept.  nullptr = keep all.
struct Drop {
    const unsigned* bits;
    uint32_t words;
};
__device__ __forceinline__ bool dropped(const Drop& d, unsigned long long key) {
    const unsigned set = (unsigned)(key >> 32);
    return d.bits && (set >> 5) < d.words && ((d.bits[set >> 5] >> (set & 31)) & 1u);
}

// Merge-path split of output tile boundary w (diagonal d = w*C in merged order): the number of A
// records among the first d (A first on ties).  C must be a multiple of 512 (aligned coarse probes).  L lanes cooperate on one boundary with an
// (L+1)-ary search (L = 1: plain binary search); tags are read only when keys tie.  Also records
// the chunk holding the first A and B rank of the tile (saves the tile one dependent lookup).
// Boundary w of (a, b) on the L lanes of its group (gl = this lane's index in the group); every lane of the
// wave calls it (ballots), inactive groups with w >= n_parts.
template <int C, int L>
__device__ __forceinline__ void lanes_split(const View& a, const View& b, uint64_t n_parts, uint64_t* __restrict__ part,
                                            uint32_t* __restrict__ pchunk, uint64_t w, int gl) {
    static_assert(L >= 1 && L <= 64 && 64 % L == 0, "lanes per boundary must divide the wave");
    static_assert(C % 512 == 0, "tile boundaries on 512-rank multiples");
    const int gbase = (int)(threadIdx.x & 63) - gl;  // first lane of this boundary's group
    const uint64_t total = a.n + b.n;
    const bool active = w < n_parts;
    const uint64_t d = !active ? 0 : w * C < total ? w * C : total;
    uint64_t lo = d > b.n ? d - b.n : 0, hi = d < a.n ? d : a.n;
    if (!active) hi = lo;
    while (__ballot(lo < hi)) {  // invariant: A[m] <= B[d-1-m] holds for m < split, fails from split on
        const uint64_t W = hi - lo;
        const bool valid = lo < hi;
        bool fail = false;
        uint64_t m = lo + ((uint64_t)(gl + 1) * W) / (L + 1);
        // wide ranges probe 512-aligned A ranks only (m stays in (lo, hi): W / 2 >= 512); d is a multiple
        // of C = 6 * 512, so the B rank d - 1 - m is 511 mod 512 too: every boundary's coarse probes hit
        // the same n / 512 lines of each stream (L2 / MALL reuse across boundaries)
        if (L == 1 && W > 1024) m &= ~511ull;
        if (valid) {
            const uint64_t sa = slot_of(a, m), sb = slot_of(b, d - 1 - m);
            const unsigned long long ka = a.key[sa], kb = b.key[sb];
            fail = ka != kb ? kb < ka : rec_lt(kb, ld_tag(b.tag + sb), ka, ld_tag(a.tag + sa));
        }
        const unsigned long long fm = __ballot(fail);
        const unsigned long long mine = L == 64 ? fm : (fm >> gbase) & ((1ull << (L & 63)) - 1);
        if (valid) {
            if (L == 1) {
                if (mine == 0) lo = m + 1;
                else hi = m;
            } else if (mine == 0) {
                lo = lo + ((uint64_t)L * W) / (L + 1) + 1;
            } else {
                const uint64_t k = (uint64_t)(__ffsll((long long)mine) - 1);
                const uint64_t nlo = k > 0 ? lo + (k * W) / (L + 1) + 1 : lo;
                hi = lo + ((k + 1) * W) / (L + 1);
                lo = nlo;
            }
        }
    }
    if (active && gl == 0) {
        const uint64_t i = lo, j = d - lo;
        part[w] = i;
        pchunk[2 * w] = i < a.n ? chunk_of(a, i) : a.nch;
        pchunk[2 * w + 1] = j < b.n ? chunk_of(b, j) : b.nch;
    }
}

template <int C, int L>
__global__ __launch_bounds__(256) void k_partition(View a, View b, uint64_t n_parts, uint64_t* __restrict__ part,
                                                   uint32_t* __restrict__ pchunk) {
    const uint64_t gt = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    lanes_split<C, L>(a, b, n_parts, part, pchunk, gt / L, (int)(gt % L));
}

// Merge-path predicate at split candidate m of diagonal d: A[m] <= B[d-1-m] (A first on ties).
__device__ __forceinline__ bool mp_le(const View& a, const View& b, uint64_t d, uint64_t m) {
    const uint64_t sa = slot_of(a, m), sb = slot_of(b, d - 1 - m);
    const unsigned long long ka = a.key[sa], kb = b.key[sb];
    return !(ka != kb ? kb < ka : rec_lt(kb, ld_tag(b.tag + sb), ka, ld_tag(a.tag + sa)));
}

// k_partition from a guess: the split of diagonal d is first guessed in proportion (d * |A| / total),
// then bracketed by probes at distances 1, 2, 4, ... <= kGallop from the guess, then binary-searched
// inside the bracket (or inside what is left of the range when the gallop did not close it, with
// k_partition's 512-aligned wide probes).  Exact for any input; streams that interleave evenly need
// about 2 log2(|split - guess|) dependent probes instead of log2(min(|A|, |B|)).
template <int C>
__device__ __forceinline__ void gallop_split(const View& a, const View& b, uint64_t w, uint64_t* __restrict__ part, uint32_t* __restrict__ pchunk) {
    constexpr uint64_t kGallop = 1024;
    const uint64_t total = a.n + b.n;
    const uint64_t d = w * C < total ? w * C : total;
    uint64_t lo = d > b.n ? d - b.n : 0, hi = d < a.n ? d : a.n;  // the split lies in [lo, hi]
    if (lo < hi) {
        uint64_t g = (uint64_t)((double)d * (double)a.n / (double)total);
        g = g < lo ? lo : g >= hi ? hi - 1 : g;
        if (mp_le(a, b, d, g)) {  // split > g
            lo = g + 1;
            for (uint64_t step = 1; step <= kGallop; step <<= 1) {
                const uint64_t m = g + step;
                if (m >= hi) break;
                if (mp_le(a, b, d, m)) lo = m + 1;
                else { hi = m; break; }
            }
        } else {  // split <= g
            hi = g;
            for (uint64_t step = 1; step <= kGallop && step <= g - lo; step <<= 1) {
                const uint64_t m = g - step;
                if (mp_le(a, b, d, m)) { lo = m + 1; break; }
                hi = m;
            }
        }
        while (lo < hi) {
            const uint64_t W = hi - lo;
            uint64_t m = lo + W / 2;
            if (W > 1024) m &= ~511ull;  // wide leftovers: k_partition's shared 512-aligned probes
            if (mp_le(a, b, d, m)) lo = m + 1;
            else hi = m;
        }
    }
    part[w] = lo;
    const uint64_t j = d - lo;
    pchunk[2 * w] = lo < a.n ? chunk_of(a, lo) : a.nch;
    pchunk[2 * w + 1] = j < b.n ? chunk_of(b, j) : b.nch;
}

// One union's tile boundaries: n_parts = tiles + 1 (none for an empty union).
struct PartJob {
    View a, b;
    uint64_t n_parts;
    uint64_t* part;
    uint32_t* pchunk;
};

template <int C>
__global__ __launch_bounds__(256) void k_partition_gallop(View a, View b, uint64_t n_parts, uint64_t* __restrict__ part,
                                                          uint32_t* __restrict__ pchunk) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w < n_parts) gallop_split<C>(a, b, w, part, pchunk);
}

// Both streams' boundaries (adds, tombstones) in one launch: the two searches are latency-bound and
// overlap instead of running back to back.
template <int C>
__global__ __launch_bounds__(256) void k_partition_gallop2(PartJob j0, PartJob j1) {
    const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (w < j0.n_parts) gallop_split<C>(j0.a, j0.b, w, j0.part, j0.pchunk);
    else if (w - j0.n_parts < j1.n_parts) gallop_split<C>(j1.a, j1.b, w - j0.n_parts, j1.part, j1.pchunk);
}

// Both streams' boundaries, L lanes per boundary ((L+1)-ary search: each round's L probes are independent).
// For a union of few tiles (a committed wave into a store: a few hundred boundaries) the gallop's chain of
// dependent probes — each a chunk lookup, a key and maybe a tag, ~16 probes — is the whole kernel (46 us);
// 64 lanes per boundary take ~4 rounds.  Many boundaries (C3: 10^5) keep the gallop (one lane each).
template <int C, int L>
__global__ __launch_bounds__(256) void k_partition_lanes2(PartJob j0, PartJob j1) {
    const uint64_t gt = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t w = gt / L;
    const int gl = (int)(gt % L);
    if (w < j0.n_parts) lanes_split<C, L>(j0.a, j0.b, j0.n_parts, j0.part, j0.pchunk, w, gl);
    else lanes_split<C, L>(j1.a, j1.b, j1.n_parts, j1.part, j1.pchunk, w - j0.n_parts, gl);  // (w past both: inactive)
}

// LDS of one union tile.
template <int kOB, int kItems>
struct UnionShared {
    static constexpr int kTile = kOB * kItems;
    static constexpr int kSeg = 64;  // chunks a tile's A (or B) range may span before the slow path
    unsigned long long key[kTile];
    uint4 tag[kTile];
    uint64_t off[2][kSeg + 1];  // chunk boundaries around the A (0) and B (1) ranges
    unsigned long long prev_key;
    uint4 prev_tag;
    int has_prev;
    int wsum[kOB / 64];
};

// Merge, compaction and stores of one tile whose records are staged in LDS (A ranks [0, nA), B ranks
// [nA, n)), with their ordinals in registers (staging index it * kOB + tid) and the A record before the
// tile in sh.prev_*.  Ordinals: an A record keeps its ord, a B record arrives with b_base added (b_base
// = A's next: a tag new to A's HashSet is appended after every tag A holds, in B's order — UnionWith /
// the copy constructor, ORSet.cs:255-282).  A B record equal to an A record is dropped, so the A
// record's ord stays.  Ends with every LDS read done (the caller may restage after a barrier).
template <int kOB, int kItems>
__device__ __forceinline__ void union_tile(UnionShared<kOB, kItems>& sh, int nA, int nB, uint64_t tile, const uint32_t (&rord)[kItems],
                                           unsigned long long* __restrict__ ok, uint4* __restrict__ ot, uint32_t* __restrict__ oord,
                                           uint32_t* __restrict__ ocnt, const Drop& drop) {
    constexpr int kTile = kOB * kItems;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = nA + nB;
    unsigned long long* s_key = sh.key;
    uint4* s_tag = sh.tag;

    // ---- per-thread merge path + serial merge of kItems outputs ----
    // The search compares keys and reads the two 16-B tags from LDS only when the keys tie (LDS
    // bandwidth, not HBM, bounded this phase when every probe read both tags).
    const int diag = min(tid * kItems, n);
    int lo = diag > nB ? diag - nB : 0, hi = min(diag, nA);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const int bj = nA + diag - 1 - mid;
        const unsigned long long kb_ = s_key[bj], ka_ = s_key[mid];
        bool b_lt_a;
        if (kb_ != ka_) b_lt_a = kb_ < ka_;
        else {
            const Tag tb_ = __builtin_bit_cast(Tag, s_tag[bj]), ta_ = __builtin_bit_cast(Tag, s_tag[mid]);
            b_lt_a = (tb_.lo < ta_.lo) | ((tb_.lo == ta_.lo) & (tb_.hi < ta_.hi));
        }
        if (!b_lt_a) lo = mid + 1;
        else hi = mid;
    }
    int ai = lo, bi = diag - lo;
    // hp: the A record just before the next B record in merged order exists and survives the drop
    // filter (a B record can only equal that one, since A and B are strictly increasing).
    bool hp;
    unsigned long long pk;
    Tag pt;
    if (ai > 0) { pk = s_key[ai - 1]; pt = __builtin_bit_cast(Tag, s_tag[ai - 1]); hp = !dropped(drop, pk); }
    else { hp = sh.has_prev != 0; pk = sh.prev_key; pt = __builtin_bit_cast(Tag, sh.prev_tag); }

    const int my_n = n - diag < kItems ? n - diag : kItems;
    unsigned long long ka = 0, kb = 0;
    Tag ta{0, 0}, tb{0, 0};
    if (ai < nA) { ka = s_key[ai]; ta = __builtin_bit_cast(Tag, s_tag[ai]); }
    if (bi < nB) { kb = s_key[nA + bi]; tb = __builtin_bit_cast(Tag, s_tag[nA + bi]); }
    // the merged records stay in registers for the compaction (no second LDS gather); src = staging index
    unsigned long long rk[kItems], rlo[kItems], rhi[kItems];
    int src[kItems];
    unsigned keep = 0;
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
        rk[it] = 0; rlo[it] = 0; rhi[it] = 0; src[it] = 0;
        if (it < my_n) {
            const bool take_a = ai < nA && (bi >= nB || !rec_lt(kb, tb, ka, ta));
            src[it] = take_a ? ai : nA + bi;
            if (take_a) {
                rk[it] = ka; rlo[it] = ta.lo; rhi[it] = ta.hi;
                hp = !dropped(drop, ka);
                if (hp) keep |= 1u << it;
                pk = ka; pt = ta;
                ++ai;
                if (ai < nA) { ka = s_key[ai]; ta = __builtin_bit_cast(Tag, s_tag[ai]); }
            } else {
                rk[it] = kb; rlo[it] = tb.lo; rhi[it] = tb.hi;
                if (!(hp && rec_eq(pk, pt, kb, tb))) keep |= 1u << it;
                ++bi;
                if (bi < nB) { kb = s_key[nA + bi]; tb = __builtin_bit_cast(Tag, s_tag[nA + bi]); }
            }
        }
    }

    // ---- block scan of kept counts (its barrier also ends every thread's LDS reads of the merge) ----
    const int cnt = __popc(keep);
    int incl = cnt;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const int y = __shfl_up(incl, dd, 64);
        if (lane >= dd) incl += y;
    }
    if (lane == 63) sh.wsum[wid] = incl;
    __syncthreads();
    int wbase = 0, block_total = 0;
#pragma unroll
    for (int w = 0; w < kOB / 64; ++w) {
        const int v = sh.wsum[w];
        if (w < wid) wbase += v;
        block_total += v;
    }
    const int my_off = wbase + incl - cnt;
    const uint64_t base = tile * (uint64_t)kTile;

    // ---- ordinals: registers -> LDS by staging index -> each kept output's ord -> compacted, stored ----
    // (the scan's barrier ended every merge-phase LDS read; the key area is free, then the tag area)
    uint32_t* s_ord_in = reinterpret_cast<uint32_t*>(s_tag);  // 12 KB of the tag area
    uint32_t* s_ord_out = reinterpret_cast<uint32_t*>(s_key);  // 12 KB of the key area
#pragma unroll
    for (int it = 0; it < kItems; ++it) s_ord_in[it * kOB + tid] = rord[it];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; ++it)
        if (keep & (1u << it)) s_ord_out[my_off + __popc(keep & ((1u << it) - 1u))] = s_ord_in[src[it]];
    __syncthreads();
    for (int x = tid; x < block_total; x += kOB) __builtin_nontemporal_store(s_ord_out[x], oord + base + x);
    __syncthreads();

    // ---- compact the kept records through LDS, store coalesced into this tile's chunk ----
#pragma unroll
    for (int it = 0; it < kItems; ++it) {
        if (keep & (1u << it)) {
            const int o = my_off + __popc(keep & ((1u << it) - 1u));
            s_key[o] = rk[it];
            s_tag[o] = to_u4(Tag{rlo[it], rhi[it]});
        }
    }
    __syncthreads();
    for (int x = tid; x < block_total; x += kOB) {  // written once, read by a later launch: non-temporal
        __builtin_nontemporal_store(s_key[x], ok + base + x);
        st_tag_nt(ot + base + x, s_tag[x]);
    }
    if (tid == 0) ocnt[tile] = (uint32_t)block_total;
}

// One tile: A ranks [i0, i1), B ranks [j0, j1) -> chunk `tile` of the output (capacity kOB*kItems).
template <int kOB, int kItems>
__global__ __launch_bounds__(kOB) void k_union(View a, View b, const uint64_t* __restrict__ part, const uint32_t* __restrict__ pchunk,
                                               unsigned long long* __restrict__ ok, uint4* __restrict__ ot, uint32_t* __restrict__ oord,
                                               uint32_t b_base, uint32_t* __restrict__ ocnt, Drop drop) {
    using SH = UnionShared<kOB, kItems>;
    constexpr int kTile = SH::kTile, kSeg = SH::kSeg;
    __shared__ SH sh;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t tile = blockIdx.x;
    const uint64_t total_in = a.n + b.n;
    const uint64_t d0 = tile * kTile;
    const uint64_t d1 = d0 + kTile < total_in ? d0 + kTile : total_in;
    const uint64_t i0 = part[tile], i1 = part[tile + 1];
    const uint64_t j0 = d0 - i0, j1 = d1 - i1;
    const int nA = (int)(i1 - i0), nB = (int)(j1 - j0), n = nA + nB;
    const uint32_t ca = pchunk[2 * tile], cb = pchunk[2 * tile + 1];

    // ---- chunk boundaries around the tile's A and B ranges (waves 0 and 1) ----
    if (wid == 0) {
        const uint32_t c = ca + lane;
        sh.off[0][lane] = c <= a.nch ? a.off[c] : a.n;
        if (lane == 0) sh.off[0][kSeg] = ca + kSeg <= a.nch ? a.off[ca + kSeg] : a.n;
    } else if (wid == 1) {
        const uint32_t c = cb + lane;
        sh.off[1][lane] = c <= b.nch ? b.off[c] : b.n;
        if (lane == 0) sh.off[1][kSeg] = cb + kSeg <= b.nch ? b.off[cb + kSeg] : b.n;
    }
    __syncthreads();

    // ---- stage the tile in LDS; every load issued before the first LDS write ----
    // The ordinals stay in registers (staging index x = it * kOB + tid): keys + tags fill the LDS of two
    // workgroups per CU, so ords only pass through LDS after the merge (union_tile).
    uint32_t rord[kItems];
    {
        unsigned long long rk[kItems], rlo[kItems], rhi[kItems];  // scalar arrays: stay in VGPRs
#pragma unroll
        for (int it = 0; it < kItems; ++it) {
            const int x = min(it * kOB + tid, n - 1);  // clamped: unconditional loads (n >= 1)
            const bool from_a = x < nA;
            const uint64_t r = from_a ? i0 + (uint64_t)x : j0 + (uint64_t)(x - nA);
            const int side = from_a ? 0 : 1;
            int s = 0;
            while (s < kSeg && sh.off[side][s + 1] <= r) ++s;
            uint64_t slot;
            if (s < kSeg) slot = (uint64_t)((from_a ? ca : cb) + s) * (uint64_t)(from_a ? a.C : b.C) + (r - sh.off[side][s]);
            else slot = from_a ? slot_of(a, r) : slot_of(b, r);  // > 64 tiny chunks under one tile (drop-filtered input); not
                                                                 // slot_of(from_a ? a : b, r), which copies both Views to scratch
            rk[it] = __builtin_nontemporal_load(as_global(from_a ? a.key : b.key) + slot);  // each record is read once
            const Tag t = ld_tag_nt(as_global(from_a ? a.tag : b.tag) + slot);
            rlo[it] = t.lo;
            rhi[it] = t.hi;
            rord[it] = __builtin_nontemporal_load(as_global(from_a ? a.ord : b.ord) + slot) + (from_a ? 0u : b_base);
        }
        unsigned long long pk = 0;
        Tag pt{0, 0};
        if (tid == 0 && i0 > 0) {  // the A record before the tile (duplicate check at the seam)
            const uint64_t ps = slot_of(a, i0 - 1);
            pk = a.key[ps];
            pt = ld_tag(a.tag + ps);
        }
#pragma unroll
        for (int it = 0; it < kItems; ++it) {  // slots >= n get a duplicate; never read
            const int x = it * kOB + tid;
            sh.key[x] = rk[it];
            sh.tag[x] = to_u4(Tag{rlo[it], rhi[it]});
        }
        if (tid == 0) {
            sh.has_prev = i0 > 0 && !dropped(drop, pk);
            sh.prev_key = pk;
            sh.prev_tag = to_u4(pt);
        }
    }
    __syncthreads();
    union_tile<kOB, kItems>(sh, nA, nB, tile, rord, ok, ot, oord, ocnt, drop);
}

// After a union: off = exclusive scan of the tiles' counts (off[nch] = *total = the record count)
// and the rank -> chunk table, in ceil(nch / 1024) workgroups.  Each workgroup sums the counts before
// its 1024 chunks itself (coalesced 16-B loads, 16 in flight per thread: a one-count-per-iteration
// loop was a chain of up to 64 dependent L2 round trips, 26 us per C3 add union), so no workgroup
// waits on another.  lut[q] = the chunk holding rank q*512; entries past the last record name the
// last chunk (nlut = (n_bound >> kQShift) + 2 for a bound n_bound >= n).
struct FinishJob {
    const uint32_t* cnt;  // 16-B aligned
    uint32_t nch;
    uint64_t* off;
    uint32_t* lut;
    uint64_t nlut;
    unsigned long long* total;
};
__host__ __device__ inline unsigned finish_blocks(uint32_t nch) { return (nch + 1023) / 1024; }

__device__ __forceinline__ void finish_block(const FinishJob& j, uint32_t blk, uint32_t nblk) {
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_base, s_n;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t c0 = blk * 1024u;  // a multiple of 4
    uint64_t pre = 0;
    {
        const uint4* c4 = reinterpret_cast<const uint4*>(j.cnt);
        const uint32_t n4 = c0 / 4;
#pragma unroll 16
        for (uint32_t i = tid; i < n4; i += 1024) {
            const uint4 v = c4[i];
            pre += (uint64_t)v.x + v.y + v.z + v.w;
        }
    }
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) pre += __shfl_xor(pre, dd, 64);
    if (lane == 0) s_w[wid] = pre;
    __syncthreads();
    if (tid == 0) {
        uint64_t t = 0;
        for (int w = 0; w < 16; ++w) t += s_w[w];
        s_base = t;
    }
    __syncthreads();
    const uint32_t nch = j.nch;
    const uint32_t c = c0 + tid;
    const uint64_t v = c < nch ? j.cnt[c] : 0;
    uint64_t incl = v;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const uint64_t y = __shfl_up(incl, dd, 64);
        if (lane >= dd) incl += y;
    }
    if (lane == 63) s_w[wid] = incl;  // s_w reuse: every thread read it before the barrier above
    __syncthreads();
    uint64_t wb = s_base;
    for (int w = 0; w < wid; ++w) wb += s_w[w];
    const uint64_t o = wb + incl - v;
    if (c < nch) {
        j.off[c] = o;
        constexpr uint64_t Q = 1ull << kQShift;
        for (uint64_t q = (o + Q - 1) >> kQShift; (q << kQShift) < o + v; ++q) j.lut[q] = c;
    }
    if (c + 1 == nch) {  // the last chunk's thread: totals
        j.off[nch] = o + v;
        *j.total = o + v;
    }
    if (blk == nblk - 1) {  // tail of the table: ranks at or past the end
        __syncthreads();
        if (c + 1 == nch) s_n = o + v;
        __syncthreads();
        const uint64_t n = s_n;
        for (uint64_t q = ((n + (1ull << kQShift) - 1) >> kQShift) + tid; q < j.nlut; q += 1024) j.lut[q] = nch - 1;
    }
}

__global__ __launch_bounds__(1024) void k_finish(const uint32_t* __restrict__ cnt, uint32_t nch, uint64_t* __restrict__ off,
                                                 uint32_t* __restrict__ lut, uint64_t nlut, unsigned long long* __restrict__ total) {
    finish_block(FinishJob{cnt, nch, off, lut, nlut, total}, blockIdx.x, gridDim.x);
}

// Both streams' finishes in one launch: blocks [0, nb0) finish j0, the rest j1 (nch > 0 for each).
__global__ __launch_bounds__(1024) void k_finish2(FinishJob j0, FinishJob j1) {
    const uint32_t nb0 = finish_blocks(j0.nch);
    if (blockIdx.x < nb0) finish_block(j0, blockIdx.x, nb0);
    else finish_block(j1, blockIdx.x - nb0, gridDim.x - nb0);
}

// Metadata of a dense stream: chunk c = ranks [c*C, min((c+1)*C, n)).
__global__ __launch_bounds__(256) void k_dense_meta(uint64_t n, uint32_t C, uint32_t nch, uint32_t* __restrict__ cnt, uint64_t* __restrict__ off,
                                                    uint32_t* __restrict__ lut, uint64_t nlut) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c <= nch; c += stride) {
        const uint64_t o = c * C < n ? c * C : n;
        off[c] = o;
        if (c < nch) cnt[c] = (uint32_t)((c + 1) * C < n ? C : n - o);
    }
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < nlut; q += stride) {
        const uint64_t c = (q << kQShift) / C;
        lut[q] = (uint32_t)(c < nch ? c : (nch ? nch - 1 : 0));
    }
}

}  // namespace jgk
