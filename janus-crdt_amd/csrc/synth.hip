// synth.hip — device-side synthetic workloads (DESIGN.md §Synthetic inputs).  Counter-based, so
// any cell / record can be recomputed on the host (the test oracle holds the same formulas in
// oracle/capi.cpp) for size-independent parity checks at full BASELINE sizes.
#include "jg_internal.hpp"

namespace {

constexpr int kB = 256;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31; return x;
}

// cell (key, col) of array `which` (0 local P, 1 local N, 2 received P, 3 received N):
// 30 % unseen (0 locally, ABSENT when received), else uniform in [0, 2^31 - 1).
template <class T>
__global__ __launch_bounds__(kB) void k_synth_pnc(T* __restrict__ out, uint64_t key0, uint64_t n_keys, uint32_t R, uint32_t which,
                                                  unsigned long long seed) {
    const uint64_t n = n_keys * R;
    const T absent = sizeof(T) == 4 ? (T)INT32_MIN : (T)INT64_MIN;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) {
        const uint64_t k = key0 + i / R, c = i % R;
        const unsigned long long idx = ((k * R + c) << 2) | which;
        const unsigned long long h = mix64(seed + (idx + 1) * 0x9E3779B97F4A7C15ull);
        T v;
        if (h % 100 < 30) v = which < 2 ? (T)0 : absent;
        else v = (T)((h >> 33) % 2147483647ull);
        out[i] = v;
    }
}

// record i of a stream with `per` tags u in [u0, u0+per) per group, groups in order; arrival ord = i
// (the stream arrived in its canonical order).
__global__ __launch_bounds__(kB) void k_synth_orset(unsigned long long* __restrict__ key, uint4* __restrict__ tag, uint32_t* __restrict__ ord,
                                                    uint64_t n, uint32_t E, uint32_t per, uint32_t u0, unsigned long long seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kB) {
        const uint64_t g = i / per;
        const unsigned long long u = u0 + (i % per);
        const unsigned long long h1 = mix64(seed ^ mix64(g * 256 + u + 1));
        const unsigned long long h2 = mix64(h1 + 0x9E3779B97F4A7C15ull);
        key[i] = ((g / E) << 32) | (g % E);
        const unsigned long long t0 = (u << 56) | (h1 >> 8);
        tag[i] = make_uint4((unsigned)t0, (unsigned)(t0 >> 32), (unsigned)h2, (unsigned)(h2 >> 32));
        ord[i] = (uint32_t)i;
    }
}

unsigned grid_for(jg_ctx* ctx, uint64_t n) {
    uint64_t g = (n + kB - 1) / kB, cap = (uint64_t)ctx->num_cus * 16;
    return (unsigned)(g > cap ? cap : (g ? g : 1));
}

template <class T>
void fill_pnc(jg_ctx* ctx, void* P, void* N, uint64_t key0, uint64_t n_keys, uint32_t R, uint32_t w0, uint64_t seed) {
    const unsigned g = grid_for(ctx, n_keys * R);
    hipLaunchKernelGGL(k_synth_pnc<T>, dim3(g), dim3(kB), 0, ctx->stream, (T*)P, key0, n_keys, R, w0, (unsigned long long)seed);
    hipLaunchKernelGGL(k_synth_pnc<T>, dim3(g), dim3(kB), 0, ctx->stream, (T*)N, key0, n_keys, R, w0 + 1, (unsigned long long)seed);
    JG_HIP(hipGetLastError());
}

}  // namespace

extern "C" {

int jg_synth_pnc_store(jg_pnc* p, uint64_t seed) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_synth_pnc_store");
        JG_REQUIRE(p, JG_EINVAL, "jg_synth_pnc_store: store is NULL");
        jg::ensure_device(p->ctx);
        if (p->eb == 8) fill_pnc<long long>(p->ctx, p->P.p, p->N.p, 0, p->n_keys, p->R, 0, seed);
        else fill_pnc<int>(p->ctx, p->P.p, p->N.p, 0, p->n_keys, p->R, 0, seed);
        JG_HIP(hipStreamSynchronize(p->ctx->stream));
    });
}

int jg_synth_pnc_rows(jg_rows* r, uint64_t seed, uint64_t key0) {
    return jg::guard([&] {
        auto lk_ = jg::lock(r);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(r, JG_EINVAL, "jg_synth_pnc_rows: rows is NULL");
        jg::ensure_device(r->ctx);
        if (r->eb == 8) fill_pnc<long long>(r->ctx, r->P.p, r->N.p, key0, r->n_rows, r->R, 2, seed);
        else fill_pnc<int>(r->ctx, r->P.p, r->N.p, key0, r->n_rows, r->R, 2, seed);  // key indices (if uploaded) are kept
        JG_HIP(hipStreamSynchronize(r->ctx->stream));
    });
}

int jg_synth_orset(jg_orset* s, uint64_t seed, uint64_t n_groups, uint32_t elems_per_set, uint32_t add_per_group, uint32_t add_u0,
                   uint32_t rem_per_group, uint32_t rem_u0) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_synth_orset");
        JG_REQUIRE(s, JG_EINVAL, "jg_synth_orset: store is NULL");
        JG_REQUIRE(elems_per_set > 0 && add_u0 + add_per_group <= 256 && rem_u0 + rem_per_group <= 256, JG_EINVAL,
                   "jg_synth_orset: tag index u must stay below 256");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg::sync_counts(s);
        const uint64_t na = n_groups * add_per_group, nr = n_groups * rem_per_group;
        JG_REQUIRE(na < 0xFFFFFFFFull && nr < 0xFFFFFFFFull, JG_EINVAL, "jg_synth_orset: a stream of 2^32 records or more");
        jg::set_dense(ctx, s->add, na);
        jg::set_dense(ctx, s->rem, nr);
        s->add.next = na;
        s->rem.next = nr;
        if (na)
            hipLaunchKernelGGL(k_synth_orset, dim3(grid_for(ctx, na)), dim3(kB), 0, ctx->stream, s->add.key.as<unsigned long long>(),
                               s->add.tag.as<uint4>(), s->add.ord.as<uint32_t>(), na, elems_per_set, add_per_group, add_u0, (unsigned long long)seed);
        if (nr)
            hipLaunchKernelGGL(k_synth_orset, dim3(grid_for(ctx, nr)), dim3(kB), 0, ctx->stream, s->rem.key.as<unsigned long long>(),
                               s->rem.tag.as<uint4>(), s->rem.ord.as<uint32_t>(), nr, elems_per_set, rem_per_group, rem_u0, (unsigned long long)seed);
        JG_HIP(hipGetLastError());
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

}  // extern "C"
