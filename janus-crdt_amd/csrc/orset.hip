// orset.hip — OR-Set store and kernels (gfx950, wave64; integer/byte work, no MFMA).
//
// Layout in HBM: two record streams per store (adds, tombstones), each structure-of-arrays
//   key : uint64  = set << 32 | elem          (elem 0xFFFFFFFF = C# null)
//   tag : 16 B    = the Guid, as {lo, hi} little-endian words
// sorted strictly increasing by (key, tag.lo, tag.hi) in rank order, stored in the chunked layout
// of orset_union.hpp (chunk = one union tile of kChunk slots).  A (set, elem)'s HashSet<Guid> is the
// run of its records; Dictionary membership of elem = the run being non-empty.
//
// ORSet.Merge (ORSet.cs:253-283) over a keyspace of sets = per-stream sorted set UNION:
//   k_partition_gallop2 : merge-path split of every tile boundary of both streams in one launch (a
//                 guess in proportion, galloped and binary-searched from there, one thread each).
//   k_union     : one tile per workgroup.  Stage the tile's slices of A and B in LDS, merge (A first
//                 on ties), drop a B record equal to the A record before it in merged order (the only
//                 way a duplicate can appear, since each input is duplicate-free), compact through a
//                 block scan, write the tile into ITS OWN output chunk.  No inter-workgroup traffic.
//   k_finish2   : both outputs' chunk offsets and rank -> chunk tables (one small launch).
//   Roofline: HBM.  Reads 28 B per input record, writes 28 B per output record (key, tag, ord).
// ORSet.Contains (ORSet.cs:204-237): k_contains, binary search of each queried key in both streams
// (rank space), then SetEquals of the two sorted runs.
#include <cstring>
#include <hipcub/hipcub.hpp>

#include <chrono>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <set>
#include <unordered_map>
#include <vector>

#include "host_pool.hpp"
#include "jg_internal.hpp"
#include "orset_union.hpp"

namespace {

// Tile shape chosen by measurement (tools/tune_orset.hip; profiles/r01/tune_orset_*.txt):
// 512 x 6 = 3072 records per tile, 74 KB LDS, 2 workgroups per CU.
constexpr int kOB = 512;   // threads per workgroup
constexpr int kItems = 6;  // records per thread per tile
constexpr int kTile = kOB * kItems;
static_assert(kTile == (int)kChunk, "a union tile fills exactly one stream chunk");
constexpr uint64_t kFewParts = 4096;  // tile boundaries below which the union's partition takes 64 lanes each

using jgk::Tag;
using jgk::ld_tag;
using jgk::to_u4;
using jgk::rec_lt;
using jgk::View;

View view(const jg_stream_soa& s) {
    return View{s.key.as<unsigned long long>(), s.tag.as<uint4>(), s.ord.as<uint32_t>(), s.off.as<uint64_t>(), s.lut.as<uint32_t>(), s.n, s.nch,
                kChunk, s.dense ? 1u : 0u};
}

// Ords are 32-bit on the device: a union's output needs A.next + B.next below this (renumber() first
// otherwise).  Tests lower it (JANUS_TEST_ORD_LIMIT) to exercise the renumbering.
uint64_t ord_limit() {
    const char* e = std::getenv("JANUS_TEST_ORD_LIMIT");
    const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
    return v > 0 && v < 0xFFFFFFFFull ? v : 0xFFFFFFFFull;
}

// Strictly increasing check of a DENSE stream: err |= 1 at the first non-increasing neighbour pair.
__global__ __launch_bounds__(kOB) void k_check_sorted(const unsigned long long* __restrict__ k, const uint4* __restrict__ t, uint64_t n,
                                                      unsigned* err) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i + 1 < n; i += (uint64_t)gridDim.x * kOB) {
        if (!rec_lt(k[i], ld_tag(t + i), k[i + 1], ld_tag(t + i + 1))) atomicOr(err, 1u);
    }
}

// Largest ord + 1 over the block into span[0]: one atomicMax per block at the end of its grid-stride
// loop (span zeroed by the caller).  Every thread of the block calls it once.
__device__ __forceinline__ void block_span(unsigned long long v, unsigned long long* span) {
    __shared__ unsigned long long wmax[kOB / 64];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(v, d, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kOB / 64; ++w) v = wmax[w] > v ? wmax[w] : v;
        if (v) atomicMax(span, v);
    }
}

// Host AoS records -> dense SoA stream; err |= 2 for an ord >= 2^32, span[0] = largest ord + 1.
__global__ __launch_bounds__(kOB) void k_unpack(const jg_tagrec* __restrict__ in, uint64_t n, unsigned long long* __restrict__ k,
                                                uint4* __restrict__ t, uint32_t* __restrict__ o, unsigned* err, unsigned long long* span) {
    unsigned long long mx = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        const jg_tagrec r = in[i];
        k[i] = r.key;
        t[i] = to_u4(Tag{r.tag_lo, r.tag_hi});
        if (r.ord > 0xFFFFFFFFull) atomicOr(err, 2u);
        o[i] = (uint32_t)r.ord;
        mx = std::max<unsigned long long>(mx, (unsigned long long)(uint32_t)r.ord + 1ull);
    }
    block_span(mx, span);
}

__global__ __launch_bounds__(kOB) void k_ord_span(const uint32_t* __restrict__ o, uint64_t n, unsigned long long* span) {
    unsigned long long mx = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB)
        mx = std::max<unsigned long long>(mx, (unsigned long long)o[i] + 1ull);
    block_span(mx, span);
}

// Renumbering (order kept): ranks -> (ord, rank) pairs, sorted by ord (stable: ties stay in rank =
// (key, tag) order), then ord[slot of sorted[i].rank] = i.
__global__ __launch_bounds__(kOB) void k_ord_by_rank(View v, const uint32_t* __restrict__ cnt, uint32_t* __restrict__ ko, uint32_t* __restrict__ vr) {
    const uint64_t slots = (uint64_t)v.nch * v.C;
    for (uint64_t x = (uint64_t)blockIdx.x * kOB + threadIdx.x; x < slots; x += (uint64_t)gridDim.x * kOB) {
        const uint64_t c = x / v.C, j = x - c * v.C;
        if (j < cnt[c]) {
            const uint64_t r = v.off[c] + j;
            ko[r] = v.ord[x];
            vr[r] = (uint32_t)r;
        }
    }
}
__global__ __launch_bounds__(kOB) void k_ord_scatter(View v, uint32_t* __restrict__ ord, const uint32_t* __restrict__ sr, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) ord[jgk::slot_of(v, sr[i])] = (uint32_t)i;
}
// Chunked SoA stream -> AoS records in rank order (walks slots; skips each chunk's unused tail).
__global__ __launch_bounds__(kOB) void k_pack(View v, const uint32_t* __restrict__ cnt, jg_tagrec* __restrict__ out) {
    const uint64_t slots = (uint64_t)v.nch * v.C;
    for (uint64_t x = (uint64_t)blockIdx.x * kOB + threadIdx.x; x < slots; x += (uint64_t)gridDim.x * kOB) {
        const uint64_t c = x / v.C, j = x - c * v.C;
        if (j < cnt[c]) {
            const Tag g = ld_tag(v.tag + x);
            out[v.off[c] + j] = jg_tagrec{v.key[x], g.lo, g.hi, v.ord[x]};
        }
    }
}

__device__ __forceinline__ unsigned long long key_at(const View& v, uint64_t r) { return v.key[jgk::slot_of(v, r)]; }
__device__ __forceinline__ uint64_t lower_key(const View& v, unsigned long long q) {
    uint64_t lo = 0, hi = v.n;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (key_at(v, m) < q) lo = m + 1; else hi = m; }
    return lo;
}
__device__ __forceinline__ uint64_t upper_key(const View& v, unsigned long long q) {
    uint64_t lo = 0, hi = v.n;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (key_at(v, m) <= q) lo = m + 1; else hi = m; }
    return lo;
}

__global__ __launch_bounds__(kOB) void k_contains(View a, View r, const unsigned long long* __restrict__ q, uint64_t nq, uint8_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long key = q[i];
        const uint64_t a0 = lower_key(a, key), a1 = upper_key(a, key);
        const uint64_t r0 = lower_key(r, key), r1 = upper_key(r, key);
        const uint64_t ca = a1 - a0, cr = r1 - r0;
        bool same = ca == cr;
        for (uint64_t j = 0; same && j < ca; ++j) {
            const Tag x = ld_tag(a.tag + jgk::slot_of(a, a0 + j)), y = ld_tag(r.tag + jgk::slot_of(r, r0 + j));
            same = x.lo == y.lo && x.hi == y.hi;
        }
        bool present;
        if ((unsigned)key == JG_NULL_ELEM) present = !same;  // !nullRemoveGuid.SetEquals(nullAddGuid)
        else present = ca > 0 && (cr == 0 || !same);        // add key, and not in removeSet or !SetEquals
        out[i] = present ? 1 : 0;
    }
}

// ORSet.LookupAll (ORSet.cs:204-227) per queried set.  Elements of a set are walked in ascending
// elem id — the host interns elements in first-insertion order of the add Dictionary, so this is the
// Dictionary's enumeration order — and emitted in the reference's three groups: present elements
// with no removeSet entry (addSet.Keys.Except(removeSet.Keys)), then present elements with one
// (the join where !SetEquals), then null if !SetEquals(nullRemoveGuid, nullAddGuid).
// pass 0: cnt[i] = the set's member count; pass 1: write members at out + off[i].
__device__ __forceinline__ bool runs_equal(const View& a, uint64_t a0, uint64_t a1, const View& r, uint64_t r0, uint64_t r1) {
    if (a1 - a0 != r1 - r0) return false;
    for (uint64_t j = 0; j < a1 - a0; ++j) {
        const Tag x = ld_tag(a.tag + jgk::slot_of(a, a0 + j)), y = ld_tag(r.tag + jgk::slot_of(r, r0 + j));
        if (x.lo != y.lo || x.hi != y.hi) return false;
    }
    return true;
}

template <int PASS>
__global__ __launch_bounds__(kOB) void k_lookup_all(View a, View r, const uint32_t* __restrict__ sets, uint64_t n,
                                                    uint64_t* __restrict__ cnt_off, uint32_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long base = (unsigned long long)sets[i] << 32, nullk = base | JG_NULL_ELEM;
        const uint64_t a_end = lower_key(a, nullk), r_beg = lower_key(r, base), r_end = lower_key(r, nullk);
        uint64_t w = PASS ? cnt_off[i] : 0;
        for (int group = 0; group < 2; ++group) {
            uint64_t x = lower_key(a, base), y = r_beg;
            while (x < a_end) {
                const unsigned long long k = key_at(a, x);
                uint64_t x1 = x + 1;
                while (x1 < a_end && key_at(a, x1) == k) ++x1;
                while (y < r_end && key_at(r, y) < k) ++y;
                uint64_t y1 = y;
                while (y1 < r_end && key_at(r, y1) == k) ++y1;
                const bool has_rem = y1 > y;
                if (has_rem == (group == 1) && (!has_rem || !runs_equal(a, x, x1, r, y, y1))) {
                    if (PASS) out[w] = (uint32_t)k;
                    ++w;
                }
                x = x1;
                y = y1;
            }
        }
        // null: present iff the null tag sets differ
        const uint64_t na1 = upper_key(a, nullk), nr1 = upper_key(r, nullk);
        if (!runs_equal(a, a_end, na1, r, r_end, nr1)) {
            if (PASS) out[w] = JG_NULL_ELEM;
            ++w;
        }
        if (!PASS) cnt_off[i] = w;
    }
}

// Rank bounds of each queried key's run in both streams: out[4i..4i+3] = a0, a1, r0, r1.
__global__ __launch_bounds__(kOB) void k_runs(View a, View r, const unsigned long long* __restrict__ q, uint64_t nq, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long key = q[i];
        out[4 * i + 0] = lower_key(a, key);
        out[4 * i + 1] = upper_key(a, key);
        out[4 * i + 2] = lower_key(r, key);
        out[4 * i + 3] = upper_key(r, key);
    }
}

// Rank bounds of whole sets (every element, null included): out[4i..4i+3] = a0, a1, r0, r1 of set[i].
__global__ __launch_bounds__(kOB) void k_set_runs(View a, View r, const uint32_t* __restrict__ sets, uint64_t n, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long base = (unsigned long long)sets[i] << 32;
        const bool last = sets[i] == 0xFFFFFFFFu;
        out[4 * i + 0] = lower_key(a, base);
        out[4 * i + 1] = last ? a.n : lower_key(a, base + (1ull << 32));
        out[4 * i + 2] = lower_key(r, base);
        out[4 * i + 3] = last ? r.n : lower_key(r, base + (1ull << 32));
    }
}

// Copy rank ranges [src_off[i], src_off[i] + len[i]) of a stream to dst[dst_off[i] ...] as AoS records.
__global__ __launch_bounds__(kOB) void k_gather_ranges(View v, const uint64_t* __restrict__ src_off, const uint64_t* __restrict__ len,
                                                       const uint64_t* __restrict__ dst_off, uint64_t n, jg_tagrec* __restrict__ dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        for (uint64_t j = 0; j < len[i]; ++j) {
            const uint64_t x = jgk::slot_of(v, src_off[i] + j);
            const Tag g = ld_tag(v.tag + x);
            dst[dst_off[i] + j] = jg_tagrec{v.key[x], g.lo, g.hi, v.ord[x]};
        }
    }
}

// jg::orset_gather_sets: per query q and side, the record count of its set's run (bounds from k_set_runs).
__global__ void k_raw_counts(const uint64_t* __restrict__ bounds, uint64_t n, unsigned long long* __restrict__ cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * n) cnt[i] = bounds[2 * i + 1] - bounds[2 * i];
    if (i == 2 * n) cnt[i] = 0;
}

// Every record of the queried runs, query by query (add side, then tombstones), in store order: key, tag, ord,
// query << 1 | side, and whether it lies below the query's ord limit for that side (lim NULL: all do).
__global__ __launch_bounds__(kOB) void k_gather_raw(View a, View r, const uint64_t* __restrict__ bounds, const unsigned long long* __restrict__ roff,
                                                    uint64_t n, uint64_t R, const unsigned long long* __restrict__ lim, unsigned long long* __restrict__ key,
                                                    unsigned long long* __restrict__ tlo, unsigned long long* __restrict__ thi, uint32_t* __restrict__ ord,
                                                    uint32_t* __restrict__ qs, uint8_t* __restrict__ keep) {
    for (uint64_t j = (uint64_t)blockIdx.x * kOB + threadIdx.x; j < R; j += (uint64_t)gridDim.x * kOB) {
        uint64_t lo = 0, hi = 2 * n;  // the last segment whose offset is <= j
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (roff[mid] <= j) lo = mid;
            else hi = mid;
        }
        const View& v = (lo & 1) ? r : a;
        const uint64_t x = jgk::slot_of(v, bounds[2 * lo] + (j - roff[lo]));
        const Tag g = ld_tag(v.tag + x);
        const uint32_t o = v.ord[x];
        key[j] = v.key[x];
        tlo[j] = g.lo;
        thi[j] = g.hi;
        ord[j] = o;
        qs[j] = (uint32_t)lo;
        keep[j] = !lim || o < lim[lo];
    }
}

unsigned grid_for(jg_ctx* ctx, uint64_t items, unsigned per_cu = 8) {
    uint64_t g = (items + kOB - 1) / kOB;
    const uint64_t cap = (uint64_t)ctx->num_cus * per_cu;
    if (g > cap) g = cap;
    return g == 0 ? 1u : (unsigned)g;
}

uint64_t tiles_for(uint64_t records) { return (records + kTile - 1) / kTile; }

// Workspace of one union: [part (n_tiles+1) x 8 | pad][pchunk 2 (n_tiles+1) x 4 | pad].
size_t union_ws_bytes(uint64_t total) {
    const uint64_t p = tiles_for(total) + 1;
    return ((p * 8 + 255) & ~(size_t)255) + ((p * 8 + 255) & ~(size_t)255);
}

// Renumber a stream's ords to 0..n-1 in the same order (ties keep rank order); next = n.  Synchronous
// on ctx->stream; needs the stream's count (no pending union).
void renumber(jg_ctx* ctx, jg_stream_soa& s) {
    if (s.n == 0) { s.next = 0; return; }
    JG_REQUIRE(s.n < 0xFFFFFFFFull, JG_ESTATE, "OR-Set stream of %llu records exceeds the 32-bit ordinal range", (unsigned long long)s.n);
    const uint64_t n = s.n;
    jg::DevBuf buf;
    size_t temp = 0;
    uint32_t* nul = nullptr;
    JG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, nul, nul, nul, nul, (int)n, 0, 32, ctx->stream));
    const size_t a4 = (n * 4 + 255) & ~(size_t)255;
    buf.alloc(4 * a4 + temp + 256);
    auto* k0 = buf.as<uint32_t>();
    auto* v0 = reinterpret_cast<uint32_t*>(buf.as<char>() + a4);
    auto* k1 = reinterpret_cast<uint32_t*>(buf.as<char>() + 2 * a4);
    auto* v1 = reinterpret_cast<uint32_t*>(buf.as<char>() + 3 * a4);
    void* tmp = buf.as<char>() + 4 * a4;
    const View v = view(s);
    hipLaunchKernelGGL(k_ord_by_rank, dim3(grid_for(ctx, (uint64_t)s.nch * kChunk, 16)), dim3(kOB), 0, ctx->stream, v, s.cnt.as<uint32_t>(), k0, v0);
    JG_HIP(hipGetLastError());
    JG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, temp, k0, k1, v0, v1, (int)n, 0, 32, ctx->stream));
    hipLaunchKernelGGL(k_ord_scatter, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, v, s.ord.as<uint32_t>(), v1, n);
    JG_HIP(hipGetLastError());
    JG_HIP(hipStreamSynchronize(ctx->stream));
    s.next = n;
}

// Make room for out = a ∪ b: out's ords reach a.next + b.next.
void ensure_ord_room(jg_ctx* ctx, jg_stream_soa& a, jg_stream_soa& b) {
    if (a.next + b.next <= ord_limit()) return;
    renumber(ctx, a);
    if (a.next + b.next > ord_limit()) renumber(ctx, b);
    JG_REQUIRE(a.next + b.next <= ord_limit(), JG_ESTATE, "OR-Set union of %llu + %llu records exceeds the 32-bit ordinal range",
               (unsigned long long)a.n, (unsigned long long)b.n);
}

// One stream's union into `out` (chunk capacity ensured here), launched in three steps shared with the
// store's other stream: boundaries (k_partition_gallop2, both streams), the tiles (k_union, per stream),
// offsets + rank table (k_finish2, both streams).  Async on ctx->stream; the output record count lands
// in *d_count (device) and out.n is left for sync_counts.  Ords: see k_union (the caller ensured
// a.next + b.next fits, ensure_ord_room).
struct UnionLaunch {
    View va{}, vb{};
    jg_stream_soa* out = nullptr;
    uint64_t total = 0, n_tiles = 0;
    uint64_t* part = nullptr;
    uint32_t* pchunk = nullptr;
    unsigned long long* d_count = nullptr;
    uint32_t b_base = 0;
    jgk::PartJob part_job() const { return jgk::PartJob{va, vb, n_tiles ? n_tiles + 1 : 0, part, pchunk}; }
    jgk::FinishJob finish_job() const {
        return jgk::FinishJob{out->cnt.as<uint32_t>(), (uint32_t)n_tiles, out->off.as<uint64_t>(), out->lut.as<uint32_t>(),
                              (total >> jgk::kQShift) + 2, d_count};
    }
};

UnionLaunch prepare_union(jg_ctx* ctx, const jg_stream_soa& a, const jg_stream_soa& b, jg_stream_soa& out, unsigned long long* d_count,
                          char* ws) {
    UnionLaunch u;
    u.total = a.n + b.n;
    out.reserve_records(u.total);
    out.next = a.next + b.next;
    u.out = &out;
    u.d_count = d_count;
    u.b_base = (uint32_t)a.next;
    if (u.total == 0) {
        jg::set_dense(ctx, out, 0);
        JG_HIP(hipMemsetAsync(d_count, 0, sizeof(unsigned long long), ctx->stream));
        return u;
    }
    u.n_tiles = tiles_for(u.total);
    JG_REQUIRE(u.n_tiles < 0xFFFFFFFFull, JG_EINVAL, "union: %llu records exceed the chunk index range", (unsigned long long)u.total);
    u.part = reinterpret_cast<uint64_t*>(ws);
    u.pchunk = reinterpret_cast<uint32_t*>(ws + (((u.n_tiles + 1) * 8 + 255) & ~(size_t)255));
    u.va = view(a);
    u.vb = view(b);
    return u;
}

void launch_tiles(jg_ctx* ctx, UnionLaunch& u, jgk::Drop drop) {
    if (u.n_tiles == 0) return;
    jg_stream_soa& out = *u.out;
    hipLaunchKernelGGL((jgk::k_union<kOB, kItems>), dim3((unsigned)u.n_tiles), dim3(kOB), 0, ctx->stream, u.va, u.vb, u.part, u.pchunk,
                       out.key.as<unsigned long long>(), out.tag.as<uint4>(), out.ord.as<uint32_t>(), u.b_base, out.cnt.as<uint32_t>(), drop);
    JG_HIP(hipGetLastError());
    out.nch = (uint32_t)u.n_tiles;
    out.dense = false;
}

// Union of both streams of two stores into `oa`/`orr`; counts to counted->counts.  Stream counts must
// be current (no pending union on a or b).
void union_store(jg_ctx* ctx, jg_orset* a, jg_orset* b, jg_stream_soa& oa, jg_stream_soa& orr, jg_orset* counted,
                 jgk::Drop drop = {nullptr, 0}) {
    ensure_ord_room(ctx, a->add, b->add);
    ensure_ord_room(ctx, a->rem, b->rem);
    unsigned long long* d = counted->counts.as<unsigned long long>();
    const size_t ws_add = union_ws_bytes(a->add.n + b->add.n);
    char* ws = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, ws_add + union_ws_bytes(a->rem.n + b->rem.n)));
    UnionLaunch ua = prepare_union(ctx, a->add, b->add, oa, d, ws);
    UnionLaunch ur = prepare_union(ctx, a->rem, b->rem, orr, d + 1, ws + ws_add);
    const jgk::PartJob pa = ua.part_job(), pr = ur.part_job();
    const uint64_t parts = pa.n_parts + pr.n_parts;
    if (parts) {
        if (parts <= kFewParts)  // a wave into a store: latency of the search, not throughput (orset_union.hpp)
            hipLaunchKernelGGL((jgk::k_partition_lanes2<kTile, 64>), dim3((unsigned)((parts * 64 + 255) / 256)), dim3(256), 0, ctx->stream, pa, pr);
        else
            hipLaunchKernelGGL((jgk::k_partition_gallop2<kTile>), dim3((unsigned)((parts + 255) / 256)), dim3(256), 0, ctx->stream, pa, pr);
        JG_HIP(hipGetLastError());
    }
    launch_tiles(ctx, ua, drop);
    launch_tiles(ctx, ur, drop);
    if (ua.n_tiles && ur.n_tiles) {
        hipLaunchKernelGGL(jgk::k_finish2, dim3(jgk::finish_blocks((uint32_t)ua.n_tiles) + jgk::finish_blocks((uint32_t)ur.n_tiles)), dim3(1024), 0,
                           ctx->stream, ua.finish_job(), ur.finish_job());
    } else {
        for (UnionLaunch* u : {&ua, &ur})
            if (u->n_tiles)
                hipLaunchKernelGGL(jgk::k_finish, dim3(jgk::finish_blocks((uint32_t)u->n_tiles)), dim3(1024), 0, ctx->stream,
                                   u->out->cnt.as<uint32_t>(), (uint32_t)u->n_tiles, u->out->off.as<uint64_t>(), u->out->lut.as<uint32_t>(),
                                   (u->total >> jgk::kQShift) + 2, u->d_count);
    }
    JG_HIP(hipGetLastError());
    counted->counts_pending = true;
}

void flag_failed(jg_ctx* ctx, unsigned h, const char* fn) {
    if (h) {
        JG_HIP(hipMemsetAsync(ctx->flags.p, 0, sizeof h, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        if (h & 2u) jg::fail(JG_EINVAL, "%s: a record's ord is not below 2^32", fn);
        jg::fail(JG_ESTATE, "%s: device reported a broken precondition (flag %u)", fn, h);
    }
}

void check_err_flag(jg_ctx* ctx, const char* fn) {
    jg::pin_get(ctx, 0, ctx->flags.p, sizeof(unsigned));
    jg::pin_sync(ctx);
    unsigned h;
    std::memcpy(&h, jg::pin_at(ctx, 0), sizeof h);
    flag_failed(ctx, h, fn);
}

void upload_stream(jg_ctx* ctx, jg_stream_soa& s, const jg_tagrec* recs, uint64_t n, const char* fn) {
    s.reserve_records(n);
    jg::set_dense(ctx, s, n);
    s.next = 0;
    if (n == 0) return;
    auto* st = static_cast<jg_tagrec*>(jg::scratch(ctx, ctx->scratch2, n * sizeof(jg_tagrec)));
    auto* span = reinterpret_cast<unsigned long long*>(ctx->flags.as<char>() + 64);
    JG_HIP(hipMemcpyAsync(st, recs, n * sizeof(jg_tagrec), hipMemcpyHostToDevice, ctx->stream));
    JG_HIP(hipMemsetAsync(span, 0, 8, ctx->stream));
    hipLaunchKernelGGL(k_unpack, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, st, n, s.key.as<unsigned long long>(), s.tag.as<uint4>(),
                       s.ord.as<uint32_t>(), ctx->flags.as<unsigned>(), span);
    JG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, s.key.as<unsigned long long>(),
                       s.tag.as<uint4>(), n, ctx->flags.as<unsigned>());
    JG_HIP(hipGetLastError());
    unsigned long long h = 0;
    JG_HIP(hipMemcpyAsync(&h, span, 8, hipMemcpyDeviceToHost, ctx->stream));
    check_err_flag(ctx, fn);  // synchronises: h is valid after it
    s.next = h;
}

void download_stream(jg_ctx* ctx, const jg_stream_soa& s, jg_tagrec* out) {
    if (s.n == 0) return;
    auto* st = static_cast<jg_tagrec*>(jg::scratch(ctx, ctx->scratch2, s.n * sizeof(jg_tagrec)));
    hipLaunchKernelGGL(k_pack, dim3(grid_for(ctx, (uint64_t)s.nch * kChunk, 16)), dim3(kOB), 0, ctx->stream, view(s), s.cnt.as<uint32_t>(), st);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemcpyAsync(out, st, s.n * sizeof(jg_tagrec), hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
}

// In-place merge: s = (s minus the records of sets flagged in `drop`) ∪ src.
void merge_into(jg_orset* s, jg_orset* src, bool async, jgk::Drop drop = {nullptr, 0}) {
    jg_ctx* ctx = s->ctx;
    const bool tr = std::getenv("JANUS_TRACE_MERGE") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e6; };
    const double t0 = tr ? now() : 0;
    jg::sync_counts(s);
    const double t1 = tr ? now() : 0;
    ensure_ord_room(ctx, s->add, src->add);
    ensure_ord_room(ctx, s->rem, src->rem);
    const double t2 = tr ? now() : 0;
    s->spare_add.reserve_records(s->add.n + src->add.n);
    s->spare_rem.reserve_records(s->rem.n + src->rem.n);
    const double t3 = tr ? now() : 0;
    union_store(ctx, s, src, s->spare_add, s->spare_rem, s, drop);
    if (tr) std::fprintf(stderr, "merge_into: sync_counts %.0f us, ord room %.0f us, reserve %.0f us, launches %.0f us (a %llu + b %llu)\n", t1 - t0,
                         t2 - t1, t3 - t2, now() - t3, (unsigned long long)s->add.n, (unsigned long long)src->add.n);
    s->add.swap(s->spare_add);
    s->rem.swap(s->spare_rem);
    if (!async) {  // the error flag and the union's counts in one page-locked round trip
        jg::pin_get(ctx, 0, ctx->flags.p, sizeof(unsigned));
        jg::pin_get(ctx, 64, s->counts.p, 16);
        jg::pin_sync(ctx);
        unsigned h;
        std::memcpy(&h, jg::pin_at(ctx, 0), sizeof h);
        flag_failed(ctx, h, "jg_orset_merge");
        unsigned long long c[2];
        std::memcpy(c, jg::pin_at(ctx, 64), sizeof c);
        s->add.n = c[0];
        s->rem.n = c[1];
        s->counts_pending = false;
        jg::orset_free_retired(s);  // the stream has drained: blocks this union's reservations retired go now
    }
}

// Records of the queried keys (sorted, unique) currently in the store, per key.
struct Runs {
    std::vector<jg_tagrec> add, rem;
    std::vector<uint64_t> add_off, rem_off;  // n + 1 offsets into add / rem
};

void gather_stream(jg_ctx* ctx, const jg_stream_soa& st, const std::vector<uint64_t>& bounds, int which, uint64_t n,
                   std::vector<jg_tagrec>& out, std::vector<uint64_t>& off) {
    std::vector<uint64_t> src(n), len(n);
    off.assign(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        src[i] = bounds[4 * i + 2 * which];
        len[i] = bounds[4 * i + 2 * which + 1] - src[i];
        off[i + 1] = off[i] + len[i];
    }
    out.resize(off[n]);
    if (off[n] == 0) return;
    jg::DevBuf meta, data;
    meta.alloc(3 * n * 8);
    data.alloc(off[n] * sizeof(jg_tagrec));
    uint64_t* m = meta.as<uint64_t>();
    JG_HIP(hipMemcpyAsync(m, src.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
    JG_HIP(hipMemcpyAsync(m + n, len.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
    JG_HIP(hipMemcpyAsync(m + 2 * n, off.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_gather_ranges, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, view(st), m, m + n, m + 2 * n, n,
                       data.as<jg_tagrec>());
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemcpyAsync(out.data(), data.p, off[n] * sizeof(jg_tagrec), hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
}

Runs fetch_runs(jg_orset* s, const std::vector<unsigned long long>& keys) {
    Runs r;
    const uint64_t n = keys.size();
    r.add_off.assign(n + 1, 0);
    r.rem_off.assign(n + 1, 0);
    if (n == 0) return r;
    jg_ctx* ctx = s->ctx;
    jg::DevBuf q;
    q.alloc(n * 8 * 5);
    auto* dq = q.as<unsigned long long>();
    auto* db = reinterpret_cast<uint64_t*>(dq + n);
    JG_HIP(hipMemcpyAsync(dq, keys.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_runs, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), dq, n, db);
    JG_HIP(hipGetLastError());
    std::vector<uint64_t> bounds(4 * n);
    JG_HIP(hipMemcpyAsync(bounds.data(), db, 4 * n * 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    gather_stream(ctx, s->add, bounds, 0, n, r.add, r.add_off);
    gather_stream(ctx, s->rem, bounds, 1, n, r.rem, r.rem_off);
    return r;
}

using TagKey = std::pair<uint64_t, uint64_t>;

// One element's tag sets while a batch of ops runs: the enumeration order (existing records by
// (ord, tag), then the batch's own in the order it appended them) and membership.
struct ElemState {
    std::vector<TagKey> add, rem;
    std::set<TagKey> add_has, rem_has;
};

void load_group(const jg_tagrec* b, const jg_tagrec* e, std::vector<TagKey>& order, std::set<TagKey>& has) {
    std::vector<jg_tagrec> g(b, e);
    std::sort(g.begin(), g.end(), [](const jg_tagrec& x, const jg_tagrec& y) {
        return x.ord != y.ord ? x.ord < y.ord : x.tag_lo != y.tag_lo ? x.tag_lo < y.tag_lo : x.tag_hi < y.tag_hi;
    });
    for (const auto& r : g) {
        order.emplace_back(r.tag_lo, r.tag_hi);
        has.emplace(r.tag_lo, r.tag_hi);
    }
}

// ORSet.Add / Remove / Clear (ORSet.cs:134-198) in op order per set.  Host-side sequential
// semantics over the store's runs of every element a Remove touches (gathered from the device),
// then ONE device union: (store minus the sets Cleared in the batch) ∪ (records added after each
// set's last Clear).  Ords of the batch's records count from 0 in op order (the union puts them after
// the store's): an Add's tag is appended to its element's HashSet (:145-149); a Remove appends the
// element's add tags it lacks to the tombstone set, in the add set's enumeration order (UnionWith /
// the copy constructor of addSet[item], :175-183).
void apply_ops(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
               const uint64_t* tag_hi, uint8_t* result, uint64_t* add_lim = nullptr, uint64_t* rem_lim = nullptr) {
    static const bool tr = std::getenv("JANUS_TRACE_APPLY") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    double tp[6] = {tr ? now() : 0};
    // the ops grouped by set, op order kept within a set: a counting sort when the set ids are dense enough (the
    // comparison sort cost 2-5 ms of host time per 50-100k ORSetWorkload ops, JANUS_TRACE_APPLY), else a stable sort
    std::vector<uint64_t> order(n_ops);
    const uint32_t max_set = *std::max_element(set, set + n_ops);
    if ((uint64_t)max_set < 4 * n_ops + 65536) {
        std::vector<uint64_t> at((size_t)max_set + 2, 0);
        for (uint64_t i = 0; i < n_ops; ++i) ++at[(size_t)set[i] + 1];
        for (size_t k = 1; k < at.size(); ++k) at[k] += at[k - 1];
        for (uint64_t i = 0; i < n_ops; ++i) order[at[set[i]]++] = i;
    } else {
        for (uint64_t i = 0; i < n_ops; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return set[a] < set[b]; });
    }
    std::vector<unsigned long long> need;
    for (uint64_t i = 0; i < n_ops; ++i)
        if (op[i] == 2) need.push_back(((unsigned long long)set[i] << 32) | elem[i]);
    std::sort(need.begin(), need.end());
    need.erase(std::unique(need.begin(), need.end()), need.end());
    if (tr) tp[1] = now();
    const Runs runs = fetch_runs(s, need);
    if (tr) tp[2] = now();

    // the sets' groups of ops (order is sorted by set): each group processed on its own — sets are independent —
    // by the workers for a large batch, its records numbered from 0 in op order and sorted by (key, tag); then
    // every group's records and snapshot limits shifted by the records of the groups before it, so the batch ords
    // run in (set, op) order and the concatenation in set order is sorted (keys are set << 32 | elem)
    std::vector<uint64_t> gbeg;
    for (uint64_t g = 0; g < n_ops;) {
        gbeg.push_back(g);
        const uint32_t sid = set[order[g]];
        while (g < n_ops && set[order[g]] == sid) ++g;
    }
    const size_t G = gbeg.size();
    gbeg.push_back(n_ops);
    std::vector<std::vector<jg_tagrec>> ga(G), gr(G);
    std::vector<uint8_t> gclr(G, 0);
    std::vector<uint64_t> issued_a(G, 0), issued_r(G, 0);  // ords a group issued, those of records a Clear dropped included
    auto lt = [](const jg_tagrec& a, const jg_tagrec& b) {
        return a.key != b.key ? a.key < b.key : a.tag_lo != b.tag_lo ? a.tag_lo < b.tag_lo : a.tag_hi < b.tag_hi;
    };
    auto one_group = [&](size_t q) {
        const uint64_t g = gbeg[q], h = gbeg[q + 1];
        const uint32_t sid = set[order[g]];
        std::unordered_map<uint32_t, ElemState> st;
        bool was_cleared = false;
        std::vector<jg_tagrec>& sa = ga[q];
        std::vector<jg_tagrec>& sr = gr[q];
        uint64_t next_a = 0, next_r = 0;  // the group's ords (op order within the set)
        auto state = [&](uint32_t e) -> ElemState& {
            auto it = st.find(e);
            if (it != st.end()) return it->second;
            ElemState es;
            const unsigned long long key = ((unsigned long long)sid << 32) | e;
            auto nk = std::lower_bound(need.begin(), need.end(), key);
            if (!was_cleared && nk != need.end() && *nk == key) {
                const size_t k = nk - need.begin();
                load_group(runs.add.data() + runs.add_off[k], runs.add.data() + runs.add_off[k + 1], es.add, es.add_has);
                load_group(runs.rem.data() + runs.rem_off[k], runs.rem.data() + runs.rem_off[k + 1], es.rem, es.rem_has);
            }
            return st.emplace(e, std::move(es)).first->second;
        };
        for (uint64_t x = g; x < h; ++x) {
            const uint64_t i = order[x];
            const unsigned long long key = ((unsigned long long)sid << 32) | elem[i];
            if (op[i] == 1) {  // Add: a fresh tag (ORSet.cs:134-153); HashSet.Add keeps a present tag where it is
                ElemState& es = state(elem[i]);
                const TagKey t{tag_lo[i], tag_hi[i]};
                if (es.add_has.insert(t).second) {
                    es.add.push_back(t);
                    sa.push_back(jg_tagrec{key, t.first, t.second, next_a++});
                }
                result[i] = 1;
            } else if (op[i] == 2) {  // Remove: if Contains, tombstone every observed tag (ORSet.cs:161-186)
                ElemState& es = state(elem[i]);
                const bool present =
                    elem[i] == JG_NULL_ELEM ? es.add_has != es.rem_has : !es.add.empty() && (es.rem.empty() || es.add_has != es.rem_has);
                if (present)
                    for (const TagKey& t : es.add)
                        if (es.rem_has.insert(t).second) {
                            es.rem.push_back(t);
                            sr.push_back(jg_tagrec{key, t.first, t.second, next_r++});
                        }
                result[i] = present ? 1 : 0;
            } else {  // Clear (ORSet.cs:192-198)
                st.clear();
                sa.clear();
                sr.clear();
                was_cleared = true;
                result[i] = 1;
            }
            if (add_lim) add_lim[i] = next_a, rem_lim[i] = next_r;  // the group's ords so far: shifted below
        }
        gclr[q] = was_cleared ? 1 : 0;
        issued_a[q] = next_a, issued_r[q] = next_r;
        // the batch's records carry no duplicate (key, tag): the ElemStates filtered them
        std::sort(sa.begin(), sa.end(), lt);
        std::sort(sr.begin(), sr.end(), lt);
    };
    static thread_local std::unique_ptr<jg::WorkerPool> pool;
    const bool par = n_ops >= 8192 && G > 1;
    if (par && !pool) pool = std::make_unique<jg::WorkerPool>(jg::host_threads());
    if (par) jg::deal(*pool, true, G, [&](size_t q, int) { one_group(q); });
    else
        for (size_t q = 0; q < G; ++q) one_group(q);
    // base_*: the ords the groups before issued (the serial walk's running counters); at_*: where a group's kept
    // records go in the batch streams
    std::vector<uint64_t> base_a(G + 1, 0), base_r(G + 1, 0), at_a(G + 1, 0), at_r(G + 1, 0);
    std::vector<uint32_t> cleared;
    for (size_t q = 0; q < G; ++q) {
        base_a[q + 1] = base_a[q] + issued_a[q];
        base_r[q + 1] = base_r[q] + issued_r[q];
        at_a[q + 1] = at_a[q] + ga[q].size();
        at_r[q + 1] = at_r[q] + gr[q].size();
        if (gclr[q]) cleared.push_back(set[order[gbeg[q]]]);
    }
    const uint64_t next_a = base_a[G], next_r = base_r[G];
    std::vector<jg_tagrec> dadd(at_a[G]), drem(at_r[G]);
    auto place = [&](size_t q) {
        for (size_t k = 0; k < ga[q].size(); ++k) dadd[at_a[q] + k] = ga[q][k], dadd[at_a[q] + k].ord += base_a[q];
        for (size_t k = 0; k < gr[q].size(); ++k) drem[at_r[q] + k] = gr[q][k], drem[at_r[q] + k].ord += base_r[q];
        if (add_lim)
            for (uint64_t x = gbeg[q]; x < gbeg[q + 1]; ++x) add_lim[order[x]] += base_a[q], rem_lim[order[x]] += base_r[q];
    };
    if (tr) tp[3] = now();
    if (par) jg::deal(*pool, true, G, [&](size_t q, int) { place(q); });
    else
        for (size_t q = 0; q < G; ++q) place(q);
    if (tr) tp[4] = now();

    jg_ctx* ctx = s->ctx;
    jg::DevBuf drop;
    jgk::Drop d{nullptr, 0};
    if (!cleared.empty()) {
        const uint32_t max_set = *std::max_element(cleared.begin(), cleared.end());
        std::vector<unsigned> bits((max_set >> 5) + 1, 0u);
        for (uint32_t c : cleared) bits[c >> 5] |= 1u << (c & 31);
        drop.alloc(bits.size() * 4);
        JG_HIP(hipMemcpyAsync(drop.p, bits.data(), bits.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        d = jgk::Drop{drop.as<unsigned>(), (uint32_t)bits.size()};
    }
    // a snapshot right after op i keeps its set's records with ord below base + the batch ords issued so far: the
    // union appends the batch's records at base = the store's next (after any renumbering, ensure_ord_room)
    auto rebase = [&](uint64_t base_a, uint64_t base_r) {
        if (add_lim)
            for (uint64_t i = 0; i < n_ops; ++i) add_lim[i] += base_a, rem_lim[i] += base_r;
    };
    if (dadd.empty() && drem.empty() && cleared.empty()) {
        rebase(s->add.next, s->rem.next);
        return;
    }
    JG_REQUIRE(next_a < 0xFFFFFFFFull && next_r < 0xFFFFFFFFull, JG_EINVAL, "jg_orset_apply_ops: too many records in one batch");
    jg_orset tmp;
    tmp.ctx = ctx;
    upload_stream(ctx, tmp.add, dadd.data(), dadd.size(), "jg_orset_apply_ops(add)");
    upload_stream(ctx, tmp.rem, drem.data(), drem.size(), "jg_orset_apply_ops(rem)");
    ensure_ord_room(ctx, s->add, tmp.add);
    ensure_ord_room(ctx, s->rem, tmp.rem);
    rebase(s->add.next, s->rem.next);
    merge_into(s, &tmp, false, d);
    if (tr)
        std::fprintf(stderr, "orset apply_ops(%llu ops, %zu sets, %zu+%zu records): order %.1f ms, fetch runs (%zu keys) %.1f ms, groups %.1f ms, "
                     "place %.1f ms, upload + merge %.1f ms\n", (unsigned long long)n_ops, G, dadd.size(), drem.size(), tp[1] - tp[0], need.size(),
                     tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], now() - tp[4]);
}

}  // namespace

void jg_stream_soa::swap(jg_stream_soa& o) {
    auto swap_buf = [](jg::DevBuf& x, jg::DevBuf& y) {
        std::swap(x.p, y.p);
        std::swap(x.bytes, y.bytes);
        std::swap(x.own, y.own);
    };
    swap_buf(block, o.block);
    swap_buf(key, o.key);
    swap_buf(tag, o.tag);
    swap_buf(ord, o.ord);
    std::swap(next, o.next);
    swap_buf(cnt, o.cnt);
    swap_buf(off, o.off);
    swap_buf(lut, o.lut);
    std::swap(cap_chunks, o.cap_chunks);
    std::swap(n, o.n);
    std::swap(nch, o.nch);
    std::swap(dense, o.dense);
}

void jg_stream_soa::reserve_records(uint64_t records) {
    uint64_t c = (records + kChunk - 1) / kChunk;
    if (c <= cap_chunks && off.p) return;
    // a stable store only grows (merges never shrink it), wave after wave, and it swaps with its spare after
    // each in-place union: a growing stream takes twice what it needs, so it reallocates every few waves,
    // not every wave (hipFree + hipMalloc of the three arrays cost 0.24-0.88 ms of a 200k-state OR-Set wave,
    // JANUS_TRACE_MERGE)
    // (and on this device's HBM a small growing stream takes 4x what it needs: below 64M records the spare
    // headroom costs < 8 GB, and each reallocation of the ORSetWorkload store cost ~2.3 ms of host time
    // (hipMalloc + hipFree of the six arrays) — every second wave at 2x early on)
    if (cap_chunks) c = std::max<uint64_t>((c * kChunk < (64ull << 20) ? 4 : 2) * c, cap_chunks + cap_chunks / 2);
    const uint64_t slots = c * kChunk;
    // ONE block for the six arrays (hipFree costs ~0.2 ms of host time per call on the box: six per stream made
    // a growing store's reservation ~2.3 ms), the new block first, then the old one freed: hipMalloc does not
    // wait for the device, hipFree does, so a reservation made while the device is still busy
    // (orset_reserve_union, during a wave's uploads) costs the host that wait, not the device an idle gap
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t sz[6] = {al(slots * 8), al(slots * 16), al(slots * 4), al((c ? c : 1) * 4), al((c + 1) * 8), al(((slots >> jgk::kQShift) + 2) * 4)};
    static const bool tr = std::getenv("JANUS_TRACE_MERGE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    jg::DevBuf nb;
    nb.alloc(sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5]);
    const auto t1 = std::chrono::steady_clock::now();
    std::swap(block.p, nb.p);
    std::swap(block.bytes, nb.bytes);
    jg::DevBuf* cur[6] = {&key, &tag, &ord, &cnt, &off, &lut};
    char* q = block.as<char>();
    for (int i = 0; i < 6; ++i) {
        cur[i]->view(q, sz[i]);
        q += sz[i];
    }
    cap_chunks = c;
    // the old block is retired, not freed: hipFree waits for the whole device and then costs ms of host time on
    // the box (measured inside a node wave: 2.9-5.7 ms, uploads in flight).  Retired blocks are freed at the
    // next point where the store's streams are known idle (jg::orset_free_retired: the end of a node wave, of a
    // synchronous merge), so they never add up beyond one wave's growth
    if (nb.p) {
        retired.push_back(nb.p);
        nb.p = nullptr;
        nb.bytes = 0;
    }
    if (tr)
        std::fprintf(stderr, "reserve_records: %llu records: hipMalloc %.0f us\n", (unsigned long long)(c * kChunk),
                     std::chrono::duration<double>(t1 - t0).count() * 1e6);
}

jg_stream_soa::~jg_stream_soa() { free_retired(); }

void jg_stream_soa::free_retired() {
    for (void* p : retired) (void)hipFree(p);
    retired.clear();
}

namespace jg {
void set_dense(jg_ctx* ctx, jg_stream_soa& s, uint64_t n) {
    s.reserve_records(n);
    const uint64_t nch = (n + kChunk - 1) / kChunk;
    const uint64_t nlut = (n >> jgk::kQShift) + 2;
    hipLaunchKernelGGL(jgk::k_dense_meta, dim3(grid_for(ctx, std::max(nch + 1, nlut), 4)), dim3(256), 0, ctx->stream, n, kChunk, (uint32_t)nch,
                       s.cnt.as<uint32_t>(), s.off.as<uint64_t>(), s.lut.as<uint32_t>(), nlut);
    JG_HIP(hipGetLastError());
    s.n = n;
    s.nch = (uint32_t)nch;
    s.dense = true;
}

void orset_free_retired(jg_orset* s) {
    for (jg_stream_soa* st : {&s->add, &s->rem, &s->spare_add, &s->spare_rem})
        if (!st->retired.empty()) st->free_retired();
    if (s->wire) orset_wire_free_retired(s->wire);
}

OrsetGathered orset_gather_sets(jg_orset* s, uint64_t n, const uint32_t* d_sets, const unsigned long long* d_lim, jg::DevBuf& buf) {
    jg_ctx* ctx = s->ctx;
    sync_counts(s);
    OrsetGathered o{};
    if (buf.bytes < n * 32 + (2 * n + 1) * 16 + 512) buf.alloc((n * 32 + (2 * n + 1) * 16 + 512) * 5 / 4);
    auto* bounds = buf.as<uint64_t>();
    auto* cnt = reinterpret_cast<unsigned long long*>(bounds + 4 * n);
    auto* roff = cnt + 2 * n + 1;
    hipLaunchKernelGGL(k_set_runs, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), d_sets, n, bounds);
    hipLaunchKernelGGL(k_raw_counts, dim3((unsigned)((2 * n + 1 + 255) / 256)), dim3(256), 0, ctx->stream, bounds, n, cnt);
    JG_HIP(hipGetLastError());
    size_t temp = 0;
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, cnt, roff, (int)(2 * n + 1), ctx->stream));
    void* tmp = jg::scratch(ctx, ctx->scratch3, temp + 256);
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, temp, cnt, roff, (int)(2 * n + 1), ctx->stream));
    jg::pin_get(ctx, 0, roff + 2 * n, 8);
    jg::pin_sync(ctx);
    std::memcpy(&o.R, jg::pin_at(ctx, 0), 8);
    JG_REQUIRE(o.R < 0x7FFFFFF0ull, JG_EINVAL, "jg_orset_encode_json: %llu records exceed one call", (unsigned long long)o.R);
    o.roff = roff;
    if (o.R == 0) return o;
    auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
    const uint64_t head = al(n * 32 + (2 * n + 1) * 16);
    const uint64_t need = head + 3 * al(o.R * 8) + 2 * al(o.R * 4) + al(o.R);
    if (buf.bytes < need) {  // grown keeping the bounds and offsets
        jg::DevBuf nb;
        nb.alloc(need + need / 4);
        JG_HIP(hipMemcpyAsync(nb.p, buf.p, head, hipMemcpyDeviceToDevice, ctx->stream));
        std::swap(nb.p, buf.p);
        std::swap(nb.bytes, buf.bytes);
        JG_HIP(hipStreamSynchronize(ctx->stream));  // the old block's copy done before it is freed
        bounds = buf.as<uint64_t>();
        roff = reinterpret_cast<unsigned long long*>(bounds + 4 * n) + 2 * n + 1;
        o.roff = roff;
    }
    char* p = buf.as<char>() + head;
    o.key = reinterpret_cast<unsigned long long*>(p);
    o.tlo = reinterpret_cast<unsigned long long*>(p + al(o.R * 8));
    o.thi = reinterpret_cast<unsigned long long*>(p + 2 * al(o.R * 8));
    o.ord = reinterpret_cast<uint32_t*>(p + 3 * al(o.R * 8));
    o.qs = reinterpret_cast<uint32_t*>(p + 3 * al(o.R * 8) + al(o.R * 4));
    o.keep = reinterpret_cast<uint8_t*>(p + 3 * al(o.R * 8) + 2 * al(o.R * 4));
    hipLaunchKernelGGL(k_gather_raw, dim3(grid_for(ctx, o.R, 16)), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), bounds, roff, n, o.R, d_lim,
                       o.key, o.tlo, o.thi, o.ord, o.qs, o.keep);
    JG_HIP(hipGetLastError());
    return o;
}

void sync_counts(jg_orset* s) {
    if (!s->counts_pending) return;
    unsigned long long h[2];
    jg::pin_get(s->ctx, 0, s->counts.p, sizeof h);
    jg::pin_sync(s->ctx);
    std::memcpy(h, jg::pin_at(s->ctx, 0), sizeof h);
    s->add.n = h[0];
    s->rem.n = h[1];
    s->counts_pending = false;
}

// Runs received from the other shards (csrc/route.hip): each run is one source's records for this
// owner, sorted and duplicate-free (a stable partition of a sorted stream; the set-id rewrite is
// monotone within one owner).  Each run is copied into a dense stream and checked, the runs are
// unioned pairwise (log2(n_runs) levels), and the result is merged into the store: the same
// ORSet.Merge per set as jg_orset_merge, from device memory.  Run r's ords order its records among
// themselves; run r is merged after runs 0..r-1 (the tree keeps the left operand first), so a tag
// new to the store enumerates by (first run holding it, its ord there).
uint64_t ord_span(jg_ctx* ctx, const uint32_t* ord, uint64_t n) {
    if (n == 0) return 0;
    auto* span = reinterpret_cast<unsigned long long*>(ctx->flags.as<char>() + 64);
    JG_HIP(hipMemsetAsync(span, 0, 8, ctx->stream));
    hipLaunchKernelGGL(k_ord_span, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, ord, n, span);
    JG_HIP(hipGetLastError());
    unsigned long long h = 0;
    JG_HIP(hipMemcpyAsync(&h, span, 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    return h;
}

void orset_merge_runs(jg_orset* s, uint32_t n_runs, const uint64_t* add_counts, const uint64_t* rem_counts, const unsigned long long* add_key,
                      const uint4* add_tag, const uint32_t* add_ord, const unsigned long long* rem_key, const uint4* rem_tag,
                      const uint32_t* rem_ord) {
    jg_ctx* ctx = s->ctx;
    sync_counts(s);
    auto fresh = [ctx] {
        auto t = std::make_unique<jg_orset>();
        t->ctx = ctx;
        t->counts.alloc(16);
        return t;
    };
    auto fill = [ctx](jg_stream_soa& st, const unsigned long long* k, const uint4* t, const uint32_t* o, uint64_t n) {
        set_dense(ctx, st, n);
        st.next = 0;
        if (n == 0) return;
        JG_HIP(hipMemcpyAsync(st.key.p, k, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(st.tag.p, t, n * 16, hipMemcpyDeviceToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(st.ord.p, o, n * 4, hipMemcpyDeviceToDevice, ctx->stream));
        st.next = ord_span(ctx, st.ord.as<uint32_t>(), n);
        hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, st.key.as<unsigned long long>(),
                           st.tag.as<uint4>(), n, ctx->flags.as<unsigned>());
        JG_HIP(hipGetLastError());
    };
    std::vector<std::unique_ptr<jg_orset>> level;
    uint64_t ao = 0, ro = 0;
    for (uint32_t r = 0; r < n_runs; ++r) {
        if (add_counts[r] + rem_counts[r] > 0) {
            auto t = fresh();
            fill(t->add, add_key + ao, add_tag + ao, add_ord + ao, add_counts[r]);
            fill(t->rem, rem_key + ro, rem_tag + ro, rem_ord + ro, rem_counts[r]);
            level.push_back(std::move(t));
        }
        ao += add_counts[r];
        ro += rem_counts[r];
    }
    check_err_flag(ctx, "jg_orset_merge_device (a received run is not strictly increasing)");
    while (level.size() > 1) {
        std::vector<std::unique_ptr<jg_orset>> next;
        for (size_t i = 0; i + 1 < level.size(); i += 2) {
            auto o = fresh();
            union_store(ctx, level[i].get(), level[i + 1].get(), o->add, o->rem, o.get());
            next.push_back(std::move(o));
        }
        if (level.size() % 2) next.push_back(std::move(level.back()));
        for (auto& o : next) sync_counts(o.get());
        level = std::move(next);
    }
    if (!level.empty()) merge_into(s, level[0].get(), false);
}

void orset_merge_store(jg_orset* s, jg_orset* src, bool defer) { merge_into(s, src, defer); }

bool orset_pin_pending(jg_orset* s, size_t at) {
    if (!s->counts_pending) return false;
    jg::pin_get(s->ctx, at, s->ctx->flags.p, sizeof(unsigned));
    jg::pin_get(s->ctx, at + 8, s->counts.p, 16);
    return true;
}
void orset_settle_pending(jg_orset* s, size_t at) {
    unsigned h;
    std::memcpy(&h, jg::pin_at(s->ctx, at), sizeof h);
    flag_failed(s->ctx, h, "jg_orset_merge");
    unsigned long long c[2];
    std::memcpy(c, jg::pin_at(s->ctx, at + 8), sizeof c);
    s->add.n = c[0];
    s->rem.n = c[1];
    s->counts_pending = false;
}

// Room in the store's union targets for `add_in` / `rem_in` more records (merge_into reserves again if a
// union turns out larger).  Called by a node wave while its uploads are in flight, so a growing store's
// reallocation is not part of the commit behind the last upload.
void orset_reserve_union(jg_orset* s, uint64_t add_in, uint64_t rem_in) {
    if (s->counts_pending) return;  // the sizes are not known without a sync: the commit reserves
    s->spare_add.reserve_records(s->add.n + add_in);
    s->spare_rem.reserve_records(s->rem.n + rem_in);
    // and the union's partition workspace: grown inside the commit, the scratch's wait for the stream let the
    // device idle while the host queued the union (merge launches 237 us instead of 22 in a growing wave)
    (void)jg::scratch(s->ctx, s->ctx->scratch3, union_ws_bytes(s->add.n + add_in) + union_ws_bytes(s->rem.n + rem_in));
}
}  // namespace jg

extern "C" {

int jg_orset_create(jg_ctx* ctx, uint64_t cap_add, uint64_t cap_rem, jg_orset** out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_orset_create: NULL argument");
        jg::ensure_device(ctx);
        auto* s = new jg_orset();
        s->ctx = ctx;
        try {
            s->add.reserve_records(cap_add);
            s->rem.reserve_records(cap_rem);
            jg::set_dense(ctx, s->add, 0);
            jg::set_dense(ctx, s->rem, 0);
            s->counts.alloc(16);
            JG_HIP(hipMemset(s->counts.p, 0, 16));
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

int jg_orset_destroy(jg_orset* s) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_destroy");
        if (!s) return;
        jg::ensure_device(s->ctx);
        JG_HIP(hipStreamSynchronize(s->ctx->stream));
        delete s;
    });
}

int jg_orset_load(jg_orset* s, const jg_tagrec* add, uint64_t n_add, const jg_tagrec* rem, uint64_t n_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_load");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_load: store is NULL");
        JG_REQUIRE((add || n_add == 0) && (rem || n_rem == 0), JG_EINVAL, "jg_orset_load: NULL records");
        jg::ensure_device(s->ctx);
        JG_HIP(hipStreamSynchronize(s->ctx->stream));
        s->counts_pending = false;
        upload_stream(s->ctx, s->add, add, n_add, "jg_orset_load(add)");
        upload_stream(s->ctx, s->rem, rem, n_rem, "jg_orset_load(rem)");
    });
}

int jg_orset_size(jg_orset* s, uint64_t* n_add, uint64_t* n_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_size: store is NULL");
        jg::ensure_device(s->ctx);
        if (s->counts_pending) check_err_flag(s->ctx, "jg_orset_size");
        jg::sync_counts(s);
        if (n_add) *n_add = s->add.n;
        if (n_rem) *n_rem = s->rem.n;
    });
}

int jg_orset_read(jg_orset* s, jg_tagrec* add, uint64_t cap_add, jg_tagrec* rem, uint64_t cap_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_read: store is NULL");
        jg::ensure_device(s->ctx);
        jg::sync_counts(s);
        JG_REQUIRE(cap_add >= s->add.n && cap_rem >= s->rem.n, JG_EINVAL, "jg_orset_read: buffers (%llu, %llu) < state (%llu, %llu)",
                   (unsigned long long)cap_add, (unsigned long long)cap_rem, (unsigned long long)s->add.n, (unsigned long long)s->rem.n);
        JG_REQUIRE((add || s->add.n == 0) && (rem || s->rem.n == 0), JG_EINVAL, "jg_orset_read: NULL buffer");
        download_stream(s->ctx, s->add, add);
        download_stream(s->ctx, s->rem, rem);
    });
}

int jg_orset_merge(jg_orset* s, const jg_tagrec* add, uint64_t n_add, const jg_tagrec* rem, uint64_t n_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_merge");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_merge: store is NULL");
        JG_REQUIRE((add || n_add == 0) && (rem || n_rem == 0), JG_EINVAL, "jg_orset_merge: NULL records");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg_orset tmp;
        tmp.ctx = ctx;
        upload_stream(ctx, tmp.add, add, n_add, "jg_orset_merge(add)");
        upload_stream(ctx, tmp.rem, rem, n_rem, "jg_orset_merge(rem)");
        merge_into(s, &tmp, false);
    });
}

int jg_orset_merge_store(jg_orset* dst, const jg_orset* src, int async) {
    return jg::guard([&] {
        auto lk_ = jg::lock(dst);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(dst, "jg_orset_merge_store");
        JG_REQUIRE(dst && src && dst != src, JG_EINVAL, "jg_orset_merge_store: bad stores");
        JG_REQUIRE(dst->ctx == src->ctx, JG_EINVAL, "jg_orset_merge_store: stores belong to different contexts");
        jg::ensure_device(dst->ctx);
        jg::sync_counts(const_cast<jg_orset*>(src));
        merge_into(dst, const_cast<jg_orset*>(src), async == 0 ? false : true);  // renumbering may touch src's ords (order kept)
    });
}

int jg_orset_union(const jg_orset* a, const jg_orset* b, jg_orset* out, int async) {
    return jg::guard([&] {
        auto lk_ = jg::lock(a);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(out, "jg_orset_union");
        JG_REQUIRE(a && b && out, JG_EINVAL, "jg_orset_union: NULL store");
        JG_REQUIRE(out != a && out != b, JG_EINVAL, "jg_orset_union: out may not alias an input");
        JG_REQUIRE(a->ctx == b->ctx && a->ctx == out->ctx, JG_EINVAL, "jg_orset_union: stores belong to different contexts");
        jg_ctx* ctx = out->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(const_cast<jg_orset*>(a));
        jg::sync_counts(const_cast<jg_orset*>(b));
        union_store(ctx, const_cast<jg_orset*>(a), const_cast<jg_orset*>(b), out->add, out->rem, out);  // renumbering keeps order
        if (!async) {
            check_err_flag(ctx, "jg_orset_union");
            jg::sync_counts(out);
        }
    });
}

int jg_orset_apply_ops(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
                       const uint64_t* tag_hi, uint8_t* result) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_apply_ops");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_apply_ops: store is NULL");
        if (n_ops == 0) return;
        JG_REQUIRE(set && elem && op && tag_lo && tag_hi && result, JG_EINVAL, "jg_orset_apply_ops: NULL argument");
        for (uint64_t i = 0; i < n_ops; ++i)
            JG_REQUIRE(op[i] >= 1 && op[i] <= 3, JG_EINVAL, "jg_orset_apply_ops: op[%llu] = %u is not 1 (Add), 2 (Remove) or 3 (Clear)",
                       (unsigned long long)i, op[i]);
        jg::ensure_device(s->ctx);
        jg::sync_counts(s);
        apply_ops(s, n_ops, set, elem, op, tag_lo, tag_hi, result);
    });
}

int jg_orset_apply_ops_ords(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
                            const uint64_t* tag_hi, uint8_t* result, uint64_t* add_lim, uint64_t* rem_lim) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);
        jg::require_writable(s, "jg_orset_apply_ops_ords");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_apply_ops_ords: store is NULL");
        if (n_ops == 0) return;
        JG_REQUIRE(set && elem && op && tag_lo && tag_hi && result && add_lim && rem_lim, JG_EINVAL, "jg_orset_apply_ops_ords: NULL argument");
        for (uint64_t i = 0; i < n_ops; ++i)
            JG_REQUIRE(op[i] >= 1 && op[i] <= 3, JG_EINVAL, "jg_orset_apply_ops_ords: op[%llu] = %u is not 1 (Add), 2 (Remove) or 3 (Clear)",
                       (unsigned long long)i, op[i]);
        jg::ensure_device(s->ctx);
        jg::sync_counts(s);
        apply_ops(s, n_ops, set, elem, op, tag_lo, tag_hi, result, add_lim, rem_lim);
    });
}

int jg_orset_contains(jg_orset* s, const uint32_t* set, const uint32_t* elem, uint64_t n, uint8_t* out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_contains: store is NULL");
        if (n == 0) return;
        JG_REQUIRE(set && elem && out, JG_EINVAL, "jg_orset_contains: NULL argument");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(s);
        std::vector<unsigned long long> q(n);
        for (uint64_t i = 0; i < n; ++i) q[i] = ((unsigned long long)set[i] << 32) | elem[i];
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * 9 + 64));
        auto* dq = reinterpret_cast<unsigned long long*>(st);
        auto* dout = reinterpret_cast<uint8_t*>(st + n * 8);
        JG_HIP(hipMemcpyAsync(dq, q.data(), n * 8, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_contains, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), dq, n, dout);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_orset_read_sets(jg_orset* s, uint64_t n, const uint32_t* set, uint64_t* add_off, jg_tagrec* add, uint64_t cap_add, uint64_t* rem_off,
                       jg_tagrec* rem, uint64_t cap_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s && add_off && rem_off, JG_EINVAL, "jg_orset_read_sets: NULL argument");
        add_off[0] = rem_off[0] = 0;
        if (n == 0) return;
        JG_REQUIRE(set, JG_EINVAL, "jg_orset_read_sets: NULL set list");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(s);
        jg::DevBuf q;
        q.alloc(n * 4 + n * 32 + 64);
        auto* dset = q.as<uint32_t>();
        auto* db = reinterpret_cast<uint64_t*>(q.as<char>() + ((n * 4 + 15) & ~15ull));
        JG_HIP(hipMemcpyAsync(dset, set, n * 4, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_set_runs, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), dset, n, db);
        JG_HIP(hipGetLastError());
        std::vector<uint64_t> bounds(4 * n);
        JG_HIP(hipMemcpyAsync(bounds.data(), db, 4 * n * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        for (uint64_t i = 0; i < n; ++i) {
            add_off[i + 1] = add_off[i] + (bounds[4 * i + 1] - bounds[4 * i]);
            rem_off[i + 1] = rem_off[i] + (bounds[4 * i + 3] - bounds[4 * i + 2]);
        }
        if (!add && !rem) return;  // size query
        JG_REQUIRE(add && rem && add_off[n] <= cap_add && rem_off[n] <= cap_rem, JG_ESTATE,
                   "jg_orset_read_sets: (%llu, %llu) records exceed the buffers (%llu, %llu)", (unsigned long long)add_off[n],
                   (unsigned long long)rem_off[n], (unsigned long long)cap_add, (unsigned long long)cap_rem);
        std::vector<jg_tagrec> ra, rr;
        std::vector<uint64_t> oa, orr;
        gather_stream(ctx, s->add, bounds, 0, n, ra, oa);
        gather_stream(ctx, s->rem, bounds, 1, n, rr, orr);
        std::copy(ra.begin(), ra.end(), add);
        std::copy(rr.begin(), rr.end(), rem);
    });
}

int jg_orset_lookup_all(jg_orset* s, uint64_t n, const uint32_t* set, uint64_t* off, uint32_t* elems, uint64_t cap) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s && off, JG_EINVAL, "jg_orset_lookup_all: NULL argument");
        off[0] = 0;
        if (n == 0) return;
        JG_REQUIRE(set, JG_EINVAL, "jg_orset_lookup_all: NULL set list");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(s);
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * 12 + 64));
        auto* dset = reinterpret_cast<uint32_t*>(st);
        auto* dcnt = reinterpret_cast<uint64_t*>(st + ((n * 4 + 15) & ~15ull));
        JG_HIP(hipMemcpyAsync(dset, set, n * 4, hipMemcpyHostToDevice, ctx->stream));
        const unsigned g = grid_for(ctx, n, 16);
        hipLaunchKernelGGL(k_lookup_all<0>, dim3(g), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), dset, n, dcnt, nullptr);
        JG_HIP(hipGetLastError());
        std::vector<uint64_t> cnt(n);
        JG_HIP(hipMemcpyAsync(cnt.data(), dcnt, n * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        for (uint64_t i = 0; i < n; ++i) off[i + 1] = off[i] + cnt[i];
        if (!elems) return;  // size query
        JG_REQUIRE(off[n] <= cap, JG_ESTATE, "jg_orset_lookup_all: %llu members exceed cap %llu", (unsigned long long)off[n],
                   (unsigned long long)cap);
        if (off[n] == 0) return;
        auto* dout = static_cast<uint32_t*>(jg::scratch(ctx, ctx->scratch2, off[n] * 4 + 64));
        JG_HIP(hipMemcpyAsync(dcnt, off, n * 8, hipMemcpyHostToDevice, ctx->stream));  // exclusive offsets
        hipLaunchKernelGGL(k_lookup_all<1>, dim3(g), dim3(kOB), 0, ctx->stream, view(s->add), view(s->rem), dset, n, dcnt, dout);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(elems, dout, off[n] * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

}  // extern "C"
