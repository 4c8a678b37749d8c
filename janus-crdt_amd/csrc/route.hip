// route.hip — cross-shard exchange of received state, gfx950, wave64.
//
// The keyspace is sharded over the GPUs of a node: global key k (PN-Counter row, OR-Set set id) is
// owned by rank k % world and lives there as local key k / world.  Global key ids are positions in
// the node's key space, which every rank knows (KeySpaceManager replicates the key set to every
// node, BFT-CRDT/CRDTManagers/KeySpaceManager.cs:121-178), so any rank can route any state.
//
// When a received batch lands on a rank that does not own all of its keys, the batch is routed:
//   k_route_hist    per tile, how many items go to each destination rank;
//   k_route_scan    one exclusive scan over the destination-major histogram = every tile's write
//                   position in every destination's run (a stable partition);
//   k_route_scatter per tile, stable ranks through wave ballots, then the items move: a PN-Counter
//                   row (key + P + N) by one wave with 16-B vectors, an OR-Set record (key + tag) by
//                   one lane; keys are rewritten to the owner's local key on the way.
// The partitioned buffers are caller-owned DEVICE memory: the host hands them to the collective
// (RCCL all-to-all over xGMI, janus_gpu/shard.py) and the owner merges what it receives with
// jg_pnc_merge_device / jg_orset_merge_device.  Roofline: HBM, one read + one write of every byte
// of the batch (the histogram pass reads only the keys); the exchange itself is xGMI-bound.
#include <algorithm>
#include <type_traits>
#include <vector>

#include "jg_internal.hpp"

namespace {

constexpr int kRB = 256;              // threads per route workgroup (4 waves)
constexpr int kRW = kRB / 64;
constexpr uint32_t kMaxWorld = 64;
constexpr uint32_t kRowTile = 256;    // PN-Counter rows per tile (one round of the workgroup)

// Tile t covers slots [t*T, t*T + len(t)): dense rows (len from n) or a chunked OR-Set stream
// (len = the chunk's record count).
struct Tiles {
    uint64_t n;
    const uint32_t* cnt;
    uint32_t T;
    __device__ __forceinline__ uint32_t len(uint32_t t) const {
        if (cnt) return cnt[t];
        const uint64_t b = (uint64_t)t * T;
        return (uint32_t)(n - b < T ? n - b : T);
    }
};

struct RowOwner {  // PN-Counter rows: key_idx (NULL = identity rows)
    const uint32_t* keys;
    uint32_t world;
    __device__ __forceinline__ uint32_t owner(uint64_t s) const { return jg::owner_of_key(keys ? keys[s] : (uint32_t)s, world); }
};

struct RecOwner {  // OR-Set records: key = set << 32 | elem
    const unsigned long long* key;
    uint32_t world;
    __device__ __forceinline__ uint32_t owner(uint64_t s) const { return jg::owner_of_key(key[s] >> 32, world); }
};

template <class Own>
__global__ __launch_bounds__(kRB) void k_route_hist(Own own, Tiles tl, uint32_t n_tiles, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kMaxWorld];
    for (uint32_t d = threadIdx.x; d < own.world; d += kRB) h[d] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x, len = tl.len(t);
    const uint64_t s0 = (uint64_t)t * tl.T;
    for (uint32_t j = threadIdx.x; j < len; j += kRB) atomicAdd(&h[own.owner(s0 + j)], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < own.world; d += kRB) hist[(uint64_t)d * n_tiles + t] = h[d];
}

// Exclusive scan of hist[m] (destination-major) into pos[m + 1] by one workgroup; bounds[d] =
// pos[d * n_tiles] for d <= world (destination d's run is [bounds[d], bounds[d+1])).
__global__ __launch_bounds__(1024) void k_route_scan(const uint32_t* __restrict__ hist, uint64_t m, uint32_t n_tiles, uint32_t world,
                                                     uint64_t* __restrict__ pos, uint64_t* __restrict__ bounds) {
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x;
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t b = tid * per < m ? tid * per : m, e = b + per < m ? b + per : m;
    uint64_t s = 0;
    for (uint64_t i = b; i < e; ++i) s += hist[i];
    part[tid] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint64_t run = tid ? part[tid - 1] : 0;
    for (uint64_t i = b; i < e; ++i) {
        pos[i] = run;
        run += hist[i];
    }
    if (tid == 1023) pos[m] = part[1023];
    __syncthreads();
    for (uint32_t d = tid; d <= world; d += 1024) bounds[d] = pos[(uint64_t)d * n_tiles];
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load(const uint4* p) {
    return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)));
}
__device__ __forceinline__ void nt_store(uint4* p, uint4 v) {
    __builtin_nontemporal_store(__builtin_bit_cast(v4u, v), reinterpret_cast<v4u*>(p));
}

// PN-Counter row mover: one wave per row; VEC = the row (R x EB bytes) is a whole number of 16-B vectors.
template <int EB, bool VEC>
struct RowMover {
    const uint32_t* keys;
    const char* P;
    const char* N;
    uint32_t* okeys;
    char* oP;
    char* oN;
    uint32_t R, world;
    static constexpr int U = 4;  // rows in flight per wave (all loads issued before the stores)
    __device__ __forceinline__ void move(uint64_t s0, uint32_t cnt, const uint64_t* dst, int lane, int wv) const {
        const uint64_t row_bytes = (uint64_t)R * EB;
        if constexpr (VEC) {
            const uint32_t nv = (uint32_t)(row_bytes / 16);
            for (uint32_t i0 = wv; i0 < cnt; i0 += kRW * U) {
                if (lane < U && i0 + lane * kRW < cnt) {
                    const uint64_t s = s0 + i0 + lane * kRW;
                    okeys[dst[i0 + lane * kRW]] = (uint32_t)jg::local_of_key(keys ? keys[s] : (uint32_t)s, world);
                }
                for (uint32_t v = lane; v < 2 * nv; v += 64) {
                    const bool isP = v < nv;
                    const uint32_t w = isP ? v : v - nv;
                    const char* src = isP ? P : N;
                    char* out = isP ? oP : oN;
                    uint4 x[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = i0 + u * kRW;
                        if (i < cnt) x[u] = nt_load(reinterpret_cast<const uint4*>(src + (s0 + i) * row_bytes) + w);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = i0 + u * kRW;
                        if (i < cnt) nt_store(reinterpret_cast<uint4*>(out + dst[i] * row_bytes) + w, x[u]);
                    }
                }
            }
            return;
        }
        for (uint32_t i = wv; i < cnt; i += kRW) {
            const uint64_t s = s0 + i, d = dst[i];
            if (lane == 0) okeys[d] = (uint32_t)jg::local_of_key(keys ? keys[s] : (uint32_t)s, world);
            {
                using T = std::conditional_t<EB == 4, int, long long>;
                const T* sp = reinterpret_cast<const T*>(P) + s * R;
                const T* sn = reinterpret_cast<const T*>(N) + s * R;
                T* dp = reinterpret_cast<T*>(oP) + d * R;
                T* dn = reinterpret_cast<T*>(oN) + d * R;
                for (uint32_t c = lane; c < 2 * R; c += 64) {
                    if (c < R) dp[c] = sp[c];
                    else dn[c - R] = sn[c - R];
                }
            }
        }
    }
};

// OR-Set record mover: one lane per record; key rewritten to the owner's local set id.
struct RecMover {
    const unsigned long long* key;
    const uint4* tag;
    const uint32_t* ord;
    unsigned long long* okey;
    uint4* otag;
    uint32_t* oord;
    uint32_t world;
    __device__ __forceinline__ void move(uint64_t s0, uint32_t cnt, const uint64_t* dst, int, int) const {
        const uint32_t i = threadIdx.x;
        if (i < cnt) {
            const unsigned long long k = key[s0 + i];
            const unsigned long long set = k >> 32;
            okey[dst[i]] = (jg::local_of_key(set, world) << 32) | (k & 0xFFFFFFFFull);
            otag[dst[i]] = tag[s0 + i];
            oord[dst[i]] = ord[s0 + i];
        }
    }
};

template <class Own, class Mover>
__global__ __launch_bounds__(kRB) void k_route_scatter(Own own, Tiles tl, uint32_t n_tiles, const uint64_t* __restrict__ pos, Mover mv) {
    __shared__ uint32_t wcnt[kRW][kMaxWorld];
    __shared__ uint64_t base[kMaxWorld];
    __shared__ uint64_t dst[kRB];
    const uint32_t t = blockIdx.x, len = tl.len(t);
    const uint64_t s0 = (uint64_t)t * tl.T;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1;
    for (uint32_t d = threadIdx.x; d < own.world; d += kRB) base[d] = pos[(uint64_t)d * n_tiles + t];
    __syncthreads();
    for (uint32_t r0 = 0; r0 < len; r0 += kRB) {
        const uint32_t j = r0 + threadIdx.x;
        const uint32_t me = j < len ? own.owner(s0 + j) : 0xFFFFFFFFu;
        uint32_t rank = 0;
        for (uint32_t d = 0; d < own.world; ++d) {  // stable rank among this wave's items bound for d
            const unsigned long long m = __ballot(me == d);
            if (me == d) rank = (uint32_t)__popcll(m & lt);
            if (lane == 0) wcnt[wv][d] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (me != 0xFFFFFFFFu) {
            uint64_t p = base[me] + rank;
            for (int w = 0; w < wv; ++w) p += wcnt[w][me];
            dst[threadIdx.x] = p;
        }
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < own.world; d += kRB) {
            uint32_t s = 0;
            for (int w = 0; w < kRW; ++w) s += wcnt[w][d];
            base[d] += s;
        }
        mv.move(s0 + r0, len - r0 < (uint32_t)kRB ? len - r0 : (uint32_t)kRB, dst, lane, wv);
        __syncthreads();
    }
}

__global__ __launch_bounds__(kRB) void k_check_keys(const uint32_t* __restrict__ k, uint64_t n, uint64_t n_keys, unsigned* err) {
    for (uint64_t i = (uint64_t)blockIdx.x * kRB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kRB)
        if (k[i] >= n_keys) atomicOr(err, 2u);
}

// A caller device buffer: device memory of ctx's device holding at least `bytes` from p.
void check_dev(jg_ctx* ctx, const void* p, uint64_t bytes, const char* fn, const char* what) {
    if (bytes == 0) return;
    JG_REQUIRE(p, JG_EINVAL, "%s: %s is NULL", fn, what);
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        jg::fail(JG_EINVAL, "%s: %s (%p) is not HIP memory", fn, what, p);
    }
    JG_REQUIRE(a.type == hipMemoryTypeDevice && a.device == ctx->device, JG_EINVAL, "%s: %s is not device memory of device %d", fn,
               what, ctx->device);
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) == hipSuccess && base) {
        const char* end = static_cast<const char*>(base) + size;
        JG_REQUIRE(static_cast<const char*>(p) + bytes <= end, JG_EINVAL, "%s: %s holds %llu bytes, %llu needed", fn, what,
                   (unsigned long long)(end - static_cast<const char*>(p)), (unsigned long long)bytes);
    } else {
        (void)hipGetLastError();
    }
}

unsigned grid_for(jg_ctx* ctx, uint64_t items) {
    uint64_t g = (items + kRB - 1) / kRB, cap = (uint64_t)ctx->num_cus * 16;
    return (unsigned)(g > cap ? cap : (g ? g : 1));
}

// Histogram + scan of one source: per-destination counts to the host, write positions in ctx scratch.
template <class Own>
const uint64_t* route_plan(jg_ctx* ctx, Own own, Tiles tl, uint32_t n_tiles, uint32_t world, uint64_t* counts) {
    const uint64_t m = (uint64_t)world * n_tiles;
    char* ws = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, m * 4 + (m + world + 2) * 8 + 64));
    auto* hist = reinterpret_cast<uint32_t*>(ws);
    auto* pos = reinterpret_cast<uint64_t*>(ws + ((m * 4 + 15) & ~15ull));
    auto* bounds = pos + m + 1;
    hipLaunchKernelGGL(k_route_hist<Own>, dim3(n_tiles), dim3(kRB), 0, ctx->stream, own, tl, n_tiles, hist);
    JG_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, ctx->stream, hist, m, n_tiles, world, pos, bounds);
    JG_HIP(hipGetLastError());
    std::vector<uint64_t> b(world + 1);
    JG_HIP(hipMemcpyAsync(b.data(), bounds, (world + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    for (uint32_t d = 0; d < world; ++d) counts[d] = b[d + 1] - b[d];
    return pos;
}

template <int EB>
void route_rows(jg_ctx* ctx, const jg_rows* r, uint32_t world, uint64_t* counts, void* dk, void* dP, void* dN) {
    const uint32_t n_tiles = (uint32_t)((r->n_rows + kRowTile - 1) / kRowTile);
    const uint32_t* keys = r->has_keys ? r->keys.as<uint32_t>() : nullptr;
    const RowOwner own{keys, world};
    const Tiles tl{r->n_rows, nullptr, kRowTile};
    const uint64_t* pos = route_plan(ctx, own, tl, n_tiles, world, counts);
    if (((uint64_t)r->R * EB) % 16 == 0) {
        const RowMover<EB, true> mv{keys, r->P.as<char>(), r->N.as<char>(), (uint32_t*)dk, (char*)dP, (char*)dN, r->R, world};
        hipLaunchKernelGGL((k_route_scatter<RowOwner, RowMover<EB, true>>), dim3(n_tiles), dim3(kRB), 0, ctx->stream, own, tl, n_tiles, pos, mv);
    } else {
        const RowMover<EB, false> mv{keys, r->P.as<char>(), r->N.as<char>(), (uint32_t*)dk, (char*)dP, (char*)dN, r->R, world};
        hipLaunchKernelGGL((k_route_scatter<RowOwner, RowMover<EB, false>>), dim3(n_tiles), dim3(kRB), 0, ctx->stream, own, tl, n_tiles, pos,
                           mv);
    }
    JG_HIP(hipGetLastError());
}

void route_stream(jg_ctx* ctx, const jg_stream_soa& s, uint32_t world, uint64_t* counts, void* dk, void* dt, void* dord) {
    if (s.n == 0 || s.nch == 0) {
        std::fill(counts, counts + world, 0ull);
        return;
    }
    const RecOwner own{s.key.as<unsigned long long>(), world};
    const Tiles tl{s.n, s.cnt.as<uint32_t>(), kChunk};
    const uint64_t* pos = route_plan(ctx, own, tl, s.nch, world, counts);
    const RecMover mv{s.key.as<unsigned long long>(), s.tag.as<uint4>(), s.ord.as<uint32_t>(), (unsigned long long*)dk, (uint4*)dt,
                      (uint32_t*)dord, world};
    hipLaunchKernelGGL((k_route_scatter<RecOwner, RecMover>), dim3(s.nch), dim3(kRB), 0, ctx->stream, own, tl, s.nch, pos, mv);
    JG_HIP(hipGetLastError());
}

}  // namespace

extern "C" {

int jg_rows_route(const jg_rows* r, uint32_t world, uint64_t* counts, void* d_keys, void* d_P, void* d_N, uint64_t cap_rows) {
    return jg::guard([&] {
        auto lk_ = jg::lock(r);  // calls on one context are serialised (shared scratch, stream)
        const char* fn = "jg_rows_route";
        JG_REQUIRE(r && counts, JG_EINVAL, "%s: NULL argument", fn);
        JG_REQUIRE(world >= 1 && world <= kMaxWorld, JG_EINVAL, "%s: world %u outside [1, %u]", fn, world, kMaxWorld);
        JG_REQUIRE(cap_rows >= r->n_rows, JG_EINVAL, "%s: buffers hold %llu rows, the batch has %llu", fn, (unsigned long long)cap_rows,
                   (unsigned long long)r->n_rows);
        JG_REQUIRE(r->n_rows < 0xFFFFFFFFull * kRowTile, JG_EINVAL, "%s: batch too large", fn);
        jg_ctx* ctx = r->ctx;
        jg::ensure_device(ctx);
        const uint64_t row_bytes = (uint64_t)r->R * r->eb;
        check_dev(ctx, d_keys, r->n_rows * 4, fn, "d_keys");
        check_dev(ctx, d_P, r->n_rows * row_bytes, fn, "d_P");
        check_dev(ctx, d_N, r->n_rows * row_bytes, fn, "d_N");
        if (r->eb == 8) route_rows<8>(ctx, r, world, counts, d_keys, d_P, d_N);
        else route_rows<4>(ctx, r, world, counts, d_keys, d_P, d_N);
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_merge_device(jg_pnc* p, uint64_t n_rows, const void* d_keys, const void* d_P, const void* d_N) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_merge_device");
        const char* fn = "jg_pnc_merge_device";
        JG_REQUIRE(p, JG_EINVAL, "%s: store is NULL", fn);
        if (n_rows == 0) return;
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const uint64_t row_bytes = (uint64_t)p->R * p->eb;
        check_dev(ctx, d_keys, n_rows * 4, fn, "d_keys");
        check_dev(ctx, d_P, n_rows * row_bytes, fn, "d_P");
        check_dev(ctx, d_N, n_rows * row_bytes, fn, "d_N");
        // every key must address the store before anything merges (all or nothing)
        hipLaunchKernelGGL(k_check_keys, dim3(grid_for(ctx, n_rows)), dim3(kRB), 0, ctx->stream, (const uint32_t*)d_keys, n_rows, p->n_keys,
                           ctx->flags.as<unsigned>());
        JG_HIP(hipGetLastError());
        unsigned h = 0;
        JG_HIP(hipMemcpyAsync(&h, ctx->flags.p, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        if (h) {
            JG_HIP(hipMemsetAsync(ctx->flags.p, 0, sizeof h, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            jg::fail(JG_EINVAL, "%s: a key_idx is >= n_keys %llu", fn, (unsigned long long)p->n_keys);
        }
        jg::pnc_merge_indexed(p, d_P, d_N, (const uint32_t*)d_keys, n_rows);
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_orset_route(jg_orset* s, uint32_t world, uint64_t* add_counts, uint64_t* rem_counts, void* d_add_key, void* d_add_tag,
                   void* d_add_ord, uint64_t cap_add, void* d_rem_key, void* d_rem_tag, void* d_rem_ord, uint64_t cap_rem) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        const char* fn = "jg_orset_route";
        JG_REQUIRE(s && add_counts && rem_counts, JG_EINVAL, "%s: NULL argument", fn);
        JG_REQUIRE(world >= 1 && world <= kMaxWorld, JG_EINVAL, "%s: world %u outside [1, %u]", fn, world, kMaxWorld);
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(s);
        JG_REQUIRE(cap_add >= s->add.n && cap_rem >= s->rem.n, JG_EINVAL, "%s: buffers (%llu, %llu) < state (%llu, %llu)", fn,
                   (unsigned long long)cap_add, (unsigned long long)cap_rem, (unsigned long long)s->add.n, (unsigned long long)s->rem.n);
        check_dev(ctx, d_add_key, s->add.n * 8, fn, "d_add_key");
        check_dev(ctx, d_add_tag, s->add.n * 16, fn, "d_add_tag");
        check_dev(ctx, d_add_ord, s->add.n * 4, fn, "d_add_ord");
        check_dev(ctx, d_rem_key, s->rem.n * 8, fn, "d_rem_key");
        check_dev(ctx, d_rem_tag, s->rem.n * 16, fn, "d_rem_tag");
        check_dev(ctx, d_rem_ord, s->rem.n * 4, fn, "d_rem_ord");
        route_stream(ctx, s->add, world, add_counts, d_add_key, d_add_tag, d_add_ord);
        route_stream(ctx, s->rem, world, rem_counts, d_rem_key, d_rem_tag, d_rem_ord);
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_orset_merge_device(jg_orset* s, uint32_t n_runs, const uint64_t* add_counts, const uint64_t* rem_counts, const void* d_add_key,
                          const void* d_add_tag, const void* d_add_ord, const void* d_rem_key, const void* d_rem_tag, const void* d_rem_ord) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_merge_device");
        const char* fn = "jg_orset_merge_device";
        JG_REQUIRE(s && (n_runs == 0 || (add_counts && rem_counts)), JG_EINVAL, "%s: NULL argument", fn);
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        uint64_t na = 0, nr = 0;
        for (uint32_t i = 0; i < n_runs; ++i) {
            na += add_counts[i];
            nr += rem_counts[i];
        }
        check_dev(ctx, d_add_key, na * 8, fn, "d_add_key");
        check_dev(ctx, d_add_tag, na * 16, fn, "d_add_tag");
        check_dev(ctx, d_add_ord, na * 4, fn, "d_add_ord");
        check_dev(ctx, d_rem_key, nr * 8, fn, "d_rem_key");
        check_dev(ctx, d_rem_tag, nr * 16, fn, "d_rem_tag");
        check_dev(ctx, d_rem_ord, nr * 4, fn, "d_rem_ord");
        jg::orset_merge_runs(s, n_runs, add_counts, rem_counts, (const unsigned long long*)d_add_key, (const uint4*)d_add_tag,
                             (const uint32_t*)d_add_ord, (const unsigned long long*)d_rem_key, (const uint4*)d_rem_tag, (const uint32_t*)d_rem_ord);
    });
}

}  // extern "C"
