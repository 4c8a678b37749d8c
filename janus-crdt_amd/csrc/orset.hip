// orset.hip — OR-Set store and kernels (gfx950, wave64; integer/byte work, no MFMA).
//
// Layout in HBM: two record streams per store (adds, tombstones), each structure-of-arrays
//   key[i] : uint64  = set << 32 | elem          (elem 0xFFFFFFFF = C# null)
//   tag[i] : 16 B    = the Guid, as {lo, hi} little-endian words
// sorted strictly increasing by (key, tag.lo, tag.hi).  A (set, elem)'s HashSet<Guid> is the run of
// its records; Dictionary membership of elem = the run being non-empty.
//
// ORSet.Merge (ORSet.cs:253-283) over a keyspace of sets = per-stream sorted set UNION:
//   k_partition : merge-path split of each TILE-record output diagonal (one binary search each).
//   k_union     : one tile per workgroup, tickets in launch order.  Stage the tile's slices of A
//                 and B in LDS, merge (A first on ties), drop a B record equal to the A record
//                 before it in merged order (the only way a duplicate can appear, since each input
//                 is duplicate-free), compact through a block scan, and place the tile with a
//                 decoupled look-back over 8-byte {flag, count} status words (agent-scope relaxed
//                 atomics: the word IS the data, no payload is handed off between workgroups).
//   Roofline: HBM.  Reads 24 B per input record, writes 24 B per output record.
// ORSet.Contains (ORSet.cs:204-237): k_contains, binary search of each queried key in both streams,
// then SetEquals of the two sorted runs.
#include <algorithm>
#include <set>
#include <unordered_map>
#include <vector>

#include "jg_internal.hpp"
#include "orset_union.hpp"

namespace {

// Tile shape chosen by measurement (tools/tune_orset.hip; profiles/r01/tune_orset_*.txt): 512 x 6 =
// 3072 records per tile, 74 KB LDS, 2 workgroups per CU.
constexpr int kOB = 512;   // threads per workgroup
constexpr int kItems = 6;  // records per thread per tile
constexpr int kTile = kOB * kItems;

using jgk::Tag;
using jgk::ld_tag;
using jgk::to_u4;
using jgk::rec_lt;

// Strictly increasing check: err |= 1 at the first non-increasing neighbour pair.
__global__ __launch_bounds__(kOB) void k_check_sorted(const unsigned long long* __restrict__ k, const uint4* __restrict__ t, uint64_t n,
                                                      unsigned* err) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i + 1 < n; i += (uint64_t)gridDim.x * kOB) {
        if (!rec_lt(k[i], ld_tag(t + i), k[i + 1], ld_tag(t + i + 1))) atomicOr(err, 1u);
    }
}

// AoS <-> SoA for host transfers.
__global__ __launch_bounds__(kOB) void k_unpack(const jg_tagrec* __restrict__ in, uint64_t n, unsigned long long* __restrict__ k,
                                                uint4* __restrict__ t) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        const jg_tagrec r = in[i];
        k[i] = r.key;
        t[i] = to_u4(Tag{r.tag_lo, r.tag_hi});
    }
}
__global__ __launch_bounds__(kOB) void k_pack(const unsigned long long* __restrict__ k, const uint4* __restrict__ t, uint64_t n,
                                              jg_tagrec* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        const Tag g = ld_tag(t + i);
        out[i] = jg_tagrec{k[i], g.lo, g.hi};
    }
}

__device__ __forceinline__ uint64_t lower_key(const unsigned long long* k, uint64_t n, unsigned long long q) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (k[m] < q) lo = m + 1; else hi = m; }
    return lo;
}
__device__ __forceinline__ uint64_t upper_key(const unsigned long long* k, uint64_t n, unsigned long long q) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (k[m] <= q) lo = m + 1; else hi = m; }
    return lo;
}

__global__ __launch_bounds__(kOB) void k_contains(const unsigned long long* __restrict__ akey, const uint4* __restrict__ atag, uint64_t na,
                                                  const unsigned long long* __restrict__ rkey, const uint4* __restrict__ rtag, uint64_t nr,
                                                  const unsigned long long* __restrict__ q, uint64_t nq, uint8_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long key = q[i];
        const uint64_t a0 = lower_key(akey, na, key), a1 = upper_key(akey, na, key);
        const uint64_t r0 = lower_key(rkey, nr, key), r1 = upper_key(rkey, nr, key);
        const uint64_t ca = a1 - a0, cr = r1 - r0;
        bool same = ca == cr;
        for (uint64_t j = 0; same && j < ca; ++j) {
            const Tag x = ld_tag(atag + a0 + j), y = ld_tag(rtag + r0 + j);
            same = x.lo == y.lo && x.hi == y.hi;
        }
        bool present;
        if ((unsigned)key == JG_NULL_ELEM) present = !same;  // !nullRemoveGuid.SetEquals(nullAddGuid)
        else present = ca > 0 && (cr == 0 || !same);        // add key, and not in removeSet or !SetEquals
        out[i] = present ? 1 : 0;
    }
}

// Run bounds of each queried key in both streams: out[4i..4i+3] = a0, a1, r0, r1.
__global__ __launch_bounds__(kOB) void k_runs(const unsigned long long* __restrict__ akey, uint64_t na, const unsigned long long* __restrict__ rkey,
                                              uint64_t nr, const unsigned long long* __restrict__ q, uint64_t nq, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * kOB) {
        const unsigned long long key = q[i];
        out[4 * i + 0] = lower_key(akey, na, key);
        out[4 * i + 1] = upper_key(akey, na, key);
        out[4 * i + 2] = lower_key(rkey, nr, key);
        out[4 * i + 3] = upper_key(rkey, nr, key);
    }
}

// Copy ranges [src_off[i], src_off[i] + len[i]) of a stream to dst[dst_off[i] ...] as AoS records.
__global__ __launch_bounds__(kOB) void k_gather_ranges(const unsigned long long* __restrict__ k, const uint4* __restrict__ t,
                                                       const uint64_t* __restrict__ src_off, const uint64_t* __restrict__ len,
                                                       const uint64_t* __restrict__ dst_off, uint64_t n, jg_tagrec* __restrict__ dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * kOB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kOB) {
        for (uint64_t j = 0; j < len[i]; ++j) {
            const Tag g = ld_tag(t + src_off[i] + j);
            dst[dst_off[i] + j] = jg_tagrec{k[src_off[i] + j], g.lo, g.hi};
        }
    }
}

unsigned grid_for(jg_ctx* ctx, uint64_t items, unsigned per_cu = 8) {
    uint64_t g = (items + kOB - 1) / kOB;
    const uint64_t cap = (uint64_t)ctx->num_cus * per_cu;
    if (g > cap) g = cap;
    return g == 0 ? 1u : (unsigned)g;
}

// Workspace of one union: [status n_tiles x 8 | ticket | pad to 256][part (n_tiles+1) x 8 | pad].
size_t union_ws_bytes(uint64_t total) {
    const uint64_t n_tiles = (total + kTile - 1) / kTile;
    return (((n_tiles * 8 + 16) + 255) & ~(size_t)255) + (((n_tiles + 1) * 8 + 255) & ~(size_t)255);
}

// Union of two streams into `out` (capacity checked by the caller).  Async on ctx->stream; the
// output count lands in *d_count (device).  `ws` holds union_ws_bytes(a.n + b.n) bytes.
void launch_union(jg_ctx* ctx, const jg_stream_soa& a, const jg_stream_soa& b, jg_stream_soa& out, unsigned long long* d_count, char* ws,
                  const unsigned* drop = nullptr) {
    const uint64_t total = a.n + b.n;
    if (total == 0) {
        JG_HIP(hipMemsetAsync(d_count, 0, sizeof(unsigned long long), ctx->stream));
        return;
    }
    const uint64_t n_tiles = (total + kTile - 1) / kTile;
    const size_t status_bytes = ((n_tiles * 8 + 16) + 255) & ~(size_t)255;
    auto* status = reinterpret_cast<unsigned long long*>(ws);
    auto* ticket = reinterpret_cast<unsigned*>(ws + n_tiles * 8);
    auto* part = reinterpret_cast<uint64_t*>(ws + status_bytes);
    JG_HIP(hipMemsetAsync(ws, 0, status_bytes, ctx->stream));  // every polled word zeroed per call
    hipLaunchKernelGGL((jgk::k_partition<kOB, kItems>), dim3((unsigned)((n_tiles + 1 + kOB - 1) / kOB)), dim3(kOB), 0, ctx->stream, a.key.as<unsigned long long>(),
                       a.tag.as<uint4>(), a.n, b.key.as<unsigned long long>(), b.tag.as<uint4>(), b.n, n_tiles + 1, part);
    JG_HIP(hipGetLastError());
    hipLaunchKernelGGL((jgk::k_union<kOB, kItems>), dim3((unsigned)n_tiles), dim3(kOB), 0, ctx->stream, a.key.as<unsigned long long>(), a.tag.as<uint4>(), a.n,
                       b.key.as<unsigned long long>(), b.tag.as<uint4>(), b.n, part, n_tiles, out.key.as<unsigned long long>(),
                       out.tag.as<uint4>(), status, ticket, d_count, ctx->flags.as<unsigned>(), drop);
    JG_HIP(hipGetLastError());
}

// Union of both streams of two stores into `oa`/`orr`; counts to counted->counts.
void union_store(jg_ctx* ctx, const jg_orset* a, const jg_orset* b, jg_stream_soa& oa, jg_stream_soa& orr, jg_orset* counted,
                 const unsigned* drop = nullptr) {
    JG_REQUIRE(oa.cap >= a->add.n + b->add.n && orr.cap >= a->rem.n + b->rem.n, JG_ESTATE,
               "union: output capacity (%llu, %llu) < inputs (%llu, %llu)", (unsigned long long)oa.cap, (unsigned long long)orr.cap,
               (unsigned long long)(a->add.n + b->add.n), (unsigned long long)(a->rem.n + b->rem.n));
    unsigned long long* d = counted->counts.as<unsigned long long>();
    const size_t ws_add = union_ws_bytes(a->add.n + b->add.n);
    char* ws = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, ws_add + union_ws_bytes(a->rem.n + b->rem.n)));
    launch_union(ctx, a->add, b->add, oa, d, ws, drop);
    launch_union(ctx, a->rem, b->rem, orr, d + 1, ws + ws_add, drop);
    counted->counts_pending = true;
}

void check_err_flag(jg_ctx* ctx, const char* fn) {
    unsigned h = 0;
    JG_HIP(hipMemcpyAsync(&h, ctx->flags.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    if (h) {
        JG_HIP(hipMemsetAsync(ctx->flags.p, 0, sizeof h, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        jg::fail(JG_ESTATE, "%s: device reported a broken precondition or look-back timeout (flag %u)", fn, h);
    }
}

void upload_stream(jg_ctx* ctx, jg_stream_soa& s, const jg_tagrec* recs, uint64_t n, const char* fn) {
    s.reserve(n);
    s.n = n;
    if (n == 0) return;
    auto* st = static_cast<jg_tagrec*>(jg::scratch(ctx, ctx->scratch2, n * sizeof(jg_tagrec)));
    JG_HIP(hipMemcpyAsync(st, recs, n * sizeof(jg_tagrec), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_unpack, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, st, n, s.key.as<unsigned long long>(), s.tag.as<uint4>());
    JG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, s.key.as<unsigned long long>(),
                       s.tag.as<uint4>(), n, ctx->flags.as<unsigned>());
    JG_HIP(hipGetLastError());
    check_err_flag(ctx, fn);
}

void download_stream(jg_ctx* ctx, const jg_stream_soa& s, jg_tagrec* out) {
    if (s.n == 0) return;
    auto* st = static_cast<jg_tagrec*>(jg::scratch(ctx, ctx->scratch2, s.n * sizeof(jg_tagrec)));
    hipLaunchKernelGGL(k_pack, dim3(grid_for(ctx, s.n, 16)), dim3(kOB), 0, ctx->stream, s.key.as<unsigned long long>(), s.tag.as<uint4>(), s.n,
                       st);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemcpyAsync(out, st, s.n * sizeof(jg_tagrec), hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
}

// In-place merge: s = (s minus the records of sets flagged in `drop`) ∪ src.
void merge_into(jg_orset* s, const jg_orset* src, bool async, const unsigned* drop = nullptr) {
    jg_ctx* ctx = s->ctx;
    jg::sync_counts(s);
    s->spare_add.reserve(s->add.n + src->add.n);
    s->spare_rem.reserve(s->rem.n + src->rem.n);
    union_store(ctx, s, src, s->spare_add, s->spare_rem, s, drop);
    s->add.swap(s->spare_add);
    s->rem.swap(s->spare_rem);
    if (!async) {
        check_err_flag(ctx, "jg_orset_merge");
        jg::sync_counts(s);
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
    hipLaunchKernelGGL(k_gather_ranges, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, st.key.as<unsigned long long>(),
                       st.tag.as<uint4>(), m, m + n, m + 2 * n, n, data.as<jg_tagrec>());
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
    hipLaunchKernelGGL(k_runs, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, s->add.key.as<unsigned long long>(), s->add.n,
                       s->rem.key.as<unsigned long long>(), s->rem.n, dq, n, db);
    JG_HIP(hipGetLastError());
    std::vector<uint64_t> bounds(4 * n);
    JG_HIP(hipMemcpyAsync(bounds.data(), db, 4 * n * 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    gather_stream(ctx, s->add, bounds, 0, n, r.add, r.add_off);
    gather_stream(ctx, s->rem, bounds, 1, n, r.rem, r.rem_off);
    return r;
}

using TagSet = std::set<std::pair<uint64_t, uint64_t>>;

// ORSet.Add / Remove / Clear (ORSet.cs:134-198) in op order per set.  Host-side sequential
// semantics over the store's runs of every element a Remove touches (gathered from the device),
// then ONE device union: (store minus the sets Cleared in the batch) ∪ (records added after each
// set's last Clear).
void apply_ops(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
               const uint64_t* tag_hi, uint8_t* result) {
    std::vector<uint64_t> order(n_ops);
    for (uint64_t i = 0; i < n_ops; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return set[a] < set[b]; });
    std::vector<unsigned long long> need;
    for (uint64_t i = 0; i < n_ops; ++i)
        if (op[i] == 2) need.push_back(((unsigned long long)set[i] << 32) | elem[i]);
    std::sort(need.begin(), need.end());
    need.erase(std::unique(need.begin(), need.end()), need.end());
    const Runs runs = fetch_runs(s, need);

    std::vector<jg_tagrec> dadd, drem;
    std::vector<uint32_t> cleared;
    struct ElemState { TagSet add, rem; };
    for (uint64_t g = 0; g < n_ops;) {
        const uint32_t sid = set[order[g]];
        uint64_t h = g;
        while (h < n_ops && set[order[h]] == sid) ++h;
        std::unordered_map<uint32_t, ElemState> st;
        bool was_cleared = false;
        std::vector<jg_tagrec> sa, sr;
        auto state = [&](uint32_t e) -> ElemState& {
            auto it = st.find(e);
            if (it != st.end()) return it->second;
            ElemState es;
            const unsigned long long key = ((unsigned long long)sid << 32) | e;
            auto nk = std::lower_bound(need.begin(), need.end(), key);
            if (!was_cleared && nk != need.end() && *nk == key) {
                const size_t q = nk - need.begin();
                for (uint64_t j = runs.add_off[q]; j < runs.add_off[q + 1]; ++j) es.add.emplace(runs.add[j].tag_lo, runs.add[j].tag_hi);
                for (uint64_t j = runs.rem_off[q]; j < runs.rem_off[q + 1]; ++j) es.rem.emplace(runs.rem[j].tag_lo, runs.rem[j].tag_hi);
            }
            return st.emplace(e, std::move(es)).first->second;
        };
        for (uint64_t x = g; x < h; ++x) {
            const uint64_t i = order[x];
            const unsigned long long key = ((unsigned long long)sid << 32) | elem[i];
            if (op[i] == 1) {  // Add: a fresh tag (ORSet.cs:134-153)
                state(elem[i]).add.emplace(tag_lo[i], tag_hi[i]);
                sa.push_back(jg_tagrec{key, tag_lo[i], tag_hi[i]});
                result[i] = 1;
            } else if (op[i] == 2) {  // Remove: if Contains, tombstone every observed tag (ORSet.cs:161-186)
                ElemState& es = state(elem[i]);
                const bool present = elem[i] == JG_NULL_ELEM ? es.add != es.rem : !es.add.empty() && (es.rem.empty() || es.add != es.rem);
                if (present)
                    for (const auto& t : es.add) {
                        es.rem.insert(t);
                        sr.push_back(jg_tagrec{key, t.first, t.second});
                    }
                result[i] = present ? 1 : 0;
            } else {  // Clear (ORSet.cs:192-198)
                st.clear();
                sa.clear();
                sr.clear();
                was_cleared = true;
                result[i] = 1;
            }
        }
        if (was_cleared) cleared.push_back(sid);
        dadd.insert(dadd.end(), sa.begin(), sa.end());
        drem.insert(drem.end(), sr.begin(), sr.end());
        g = h;
    }
    auto lt = [](const jg_tagrec& a, const jg_tagrec& b) {
        return a.key != b.key ? a.key < b.key : a.tag_lo != b.tag_lo ? a.tag_lo < b.tag_lo : a.tag_hi < b.tag_hi;
    };
    auto eq = [](const jg_tagrec& a, const jg_tagrec& b) { return a.key == b.key && a.tag_lo == b.tag_lo && a.tag_hi == b.tag_hi; };
    std::sort(dadd.begin(), dadd.end(), lt);
    dadd.erase(std::unique(dadd.begin(), dadd.end(), eq), dadd.end());
    std::sort(drem.begin(), drem.end(), lt);
    drem.erase(std::unique(drem.begin(), drem.end(), eq), drem.end());

    jg_ctx* ctx = s->ctx;
    jg::DevBuf drop;
    if (!cleared.empty()) {
        // The union reads drop[set >> 5] for every store record, so the bitmap covers the largest set
        // id in the store (the last key of each sorted stream), not just the cleared ones.
        uint64_t max_set = *std::max_element(cleared.begin(), cleared.end());
        unsigned long long last[2] = {0, 0};
        if (s->add.n) JG_HIP(hipMemcpy(&last[0], s->add.key.as<unsigned long long>() + s->add.n - 1, 8, hipMemcpyDeviceToHost));
        if (s->rem.n) JG_HIP(hipMemcpy(&last[1], s->rem.key.as<unsigned long long>() + s->rem.n - 1, 8, hipMemcpyDeviceToHost));
        max_set = std::max<uint64_t>(max_set, std::max(last[0] >> 32, last[1] >> 32));
        std::vector<unsigned> bits((max_set >> 5) + 1, 0u);
        for (uint32_t c : cleared) bits[c >> 5] |= 1u << (c & 31);
        drop.alloc(bits.size() * 4);
        JG_HIP(hipMemcpyAsync(drop.p, bits.data(), bits.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    if (dadd.empty() && drem.empty() && cleared.empty()) return;
    jg_orset tmp;
    tmp.ctx = ctx;
    upload_stream(ctx, tmp.add, dadd.data(), dadd.size(), "jg_orset_apply_ops(add)");
    upload_stream(ctx, tmp.rem, drem.data(), drem.size(), "jg_orset_apply_ops(rem)");
    merge_into(s, &tmp, false, drop.as<unsigned>());
}

}  // namespace

void jg_stream_soa::swap(jg_stream_soa& o) {
    std::swap(key.p, o.key.p); std::swap(key.bytes, o.key.bytes);
    std::swap(tag.p, o.tag.p); std::swap(tag.bytes, o.tag.bytes);
    std::swap(cap, o.cap); std::swap(n, o.n);
}

void jg_stream_soa::reserve(uint64_t c) {
    if (c <= cap) return;
    key.alloc(c * 8);
    tag.alloc(c * 16);
    cap = c;
}

namespace jg {
void sync_counts(jg_orset* s) {
    if (!s->counts_pending) return;
    unsigned long long h[2];
    JG_HIP(hipMemcpyAsync(h, s->counts.p, sizeof h, hipMemcpyDeviceToHost, s->ctx->stream));
    JG_HIP(hipStreamSynchronize(s->ctx->stream));
    s->add.n = h[0];
    s->rem.n = h[1];
    s->counts_pending = false;
}
}  // namespace jg

extern "C" {

int jg_orset_create(jg_ctx* ctx, uint64_t cap_add, uint64_t cap_rem, jg_orset** out) {
    return jg::guard([&] {
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_orset_create: NULL argument");
        jg::ensure_device(ctx);
        auto* s = new jg_orset();
        s->ctx = ctx;
        try {
            s->add.reserve(cap_add);
            s->rem.reserve(cap_rem);
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
        if (!s) return;
        jg::ensure_device(s->ctx);
        JG_HIP(hipStreamSynchronize(s->ctx->stream));
        delete s;
    });
}

int jg_orset_load(jg_orset* s, const jg_tagrec* add, uint64_t n_add, const jg_tagrec* rem, uint64_t n_rem) {
    return jg::guard([&] {
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
        JG_REQUIRE(dst && src && dst != src, JG_EINVAL, "jg_orset_merge_store: bad stores");
        JG_REQUIRE(dst->ctx == src->ctx, JG_EINVAL, "jg_orset_merge_store: stores belong to different contexts");
        jg::ensure_device(dst->ctx);
        jg::sync_counts(const_cast<jg_orset*>(src));
        merge_into(dst, src, async == 0 ? false : true);
    });
}

int jg_orset_union(const jg_orset* a, const jg_orset* b, jg_orset* out, int async) {
    return jg::guard([&] {
        JG_REQUIRE(a && b && out, JG_EINVAL, "jg_orset_union: NULL store");
        JG_REQUIRE(out != a && out != b, JG_EINVAL, "jg_orset_union: out may not alias an input");
        JG_REQUIRE(a->ctx == b->ctx && a->ctx == out->ctx, JG_EINVAL, "jg_orset_union: stores belong to different contexts");
        jg_ctx* ctx = out->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(const_cast<jg_orset*>(a));
        jg::sync_counts(const_cast<jg_orset*>(b));
        union_store(ctx, a, b, out->add, out->rem, out);
        if (!async) {
            check_err_flag(ctx, "jg_orset_union");
            jg::sync_counts(out);
        }
    });
}

int jg_orset_apply_ops(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
                       const uint64_t* tag_hi, uint8_t* result) {
    return jg::guard([&] {
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

int jg_orset_contains(jg_orset* s, const uint32_t* set, const uint32_t* elem, uint64_t n, uint8_t* out) {
    return jg::guard([&] {
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
        hipLaunchKernelGGL(k_contains, dim3(grid_for(ctx, n, 16)), dim3(kOB), 0, ctx->stream, s->add.key.as<unsigned long long>(),
                           s->add.tag.as<uint4>(), s->add.n, s->rem.key.as<unsigned long long>(), s->rem.tag.as<uint4>(), s->rem.n, dq, n,
                           dout);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

}  // extern "C"
