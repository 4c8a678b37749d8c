// jg_internal.hpp — shared internals of libjanusgpu (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "janus_gpu.h"

namespace jg {

// Row / set id of a message of another kind in a node wave (csrc/node.hip): the PN-Counter and OR-Set
// passes run over the same uploaded wave and skip each other's messages.
constexpr uint32_t kSkipIdx = 0xFFFFFFFFu;

// ---- the one owner rule of a sharded node -------------------
// A key uid belongs to rank shard_of_uid(uid, world) (the apply loop's shard shortcut, jg_shard_of); its
// global key (PN-Counter row / OR-Set set id in the node's key space) is local x world + owner
// (jg_global_key), so the exchange's routing rule owner_of_key(global) = global % world (route.hip, comm.hip)
// names the same rank, and the owner stores it as local key global / world.
__host__ __device__ __forceinline__ uint64_t uid_hash(uint64_t lo, uint64_t hi) {
    uint64_t x = lo ^ (hi * 0x9E3779B97F4A7C15ull);
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x;
}
__host__ __device__ __forceinline__ uint32_t shard_of_uid(uint64_t lo, uint64_t hi, uint32_t world) {
    return world <= 1 ? 0u : (uint32_t)((uid_hash(lo, hi) >> 7) % world);
}
__host__ __device__ __forceinline__ uint32_t owner_of_key(uint64_t global_key, uint32_t world) { return (uint32_t)(global_key % world); }
__host__ __device__ __forceinline__ uint64_t local_of_key(uint64_t global_key, uint32_t world) { return global_key / world; }

// ---- errors ------------------------------------------------------------------------------------
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

struct Error {  // thrown inside the library only; converted to a code at the ABI edge
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define JG_HIP(call)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) ::jg::fail(JG_EHIP, "%s failed: %s (%s:%d)", #call,               \
                                        hipGetErrorString(e_), __FILE__, __LINE__);             \
    } while (0)

#define JG_REQUIRE(cond, code, ...) \
    do { if (!(cond)) ::jg::fail((code), __VA_ARGS__); } while (0)

// Run `body` and translate any library error / bad_alloc into an ABI return code.
template <class F> int guard(F&& body) {
    try {
        clear_error();
        body();
        return JG_OK;
    } catch (const Error& e) {
        set_error("%s", e.msg.c_str());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return JG_ENOMEM;
    } catch (...) {
        set_error("unexpected C++ exception");
        return JG_EINVAL;
    }
}

// ---- device buffers ------------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool own = true;       // false: a view into another DevBuf's block (never freed through this one)
    void alloc(size_t n);  // frees the old block; n == 0 leaves p null
    void view(void* q, size_t n) {  // a non-owning view (the owner frees the block)
        release();
        p = q;
        bytes = n;
        own = false;
    }
    void release();
    ~DevBuf() { release(); }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    template <class T> T* as() const { return static_cast<T*>(p); }
};

}  // namespace jg

// ---- handle types (opaque at the ABI) ------------------------------------------------------------
struct jg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int num_cus = 256;
    jg::DevBuf scratch;  // reusable per-call device scratch (key indices, query keys, staging)
    jg::DevBuf scratch2;
    jg::DevBuf scratch3;
    jg::DevBuf flags;    // small zero-initialised status words (error flags)
    // page-locked bytes for small status reads and writes (a pageable copy is staged by the runtime: a blit
    // kernel plus a host copy, ~30-40 us of host gap per round trip): reads at [0, kPinRead), writes from
    // kPinRead (jg::pin_get / pin_sync / pin_at)
    void* hstat = nullptr;
    hipStream_t copy = nullptr;    // wave uploads: chunk k+1's H2D overlaps chunk k's parse on `stream`
    hipEvent_t copied = nullptr;
    // pipelined digests (jg_waves_update_digests): wave k's second-level chains run on `side` while
    // `level1` runs wave k+1's first level, on disjoint CU sets (queue CU masks: a chain that shares its
    // SIMDs with k_sha_msgs waves slows by a quarter); chain_free[s] / level1_done[s] guard the two
    // scratch slots, `begun` orders both after the work already queued on `stream`
    hipStream_t side = nullptr, level1 = nullptr;
    bool cu_masked = false;  // side / level1 hold disjoint CU sets (false: plain streams sharing every CU)
    hipEvent_t level1_done[2] = {nullptr, nullptr}, chain_free[2] = {nullptr, nullptr}, begun = nullptr;
    // Every entry point that reaches this context holds `mu` for the call: the scratch buffers and the
    // streams are shared by all of the context's handles, so concurrent callers (the reference's
    // receiver threads merging prospective copies, readers querying) are serialised here.  Recursive:
    // one-shot entry points reuse the streamed ones on the same thread.
    std::recursive_mutex mu;
};

struct jg_pnc {
    jg_ctx* ctx;
    uint64_t n_keys;
    uint32_t R;
    uint32_t eb;  // elem bytes (4 | 8)
    jg::DevBuf P, N;
    // replica table (json.hip): [n_keys x R] 16-byte Guids + [n_keys] column counts, first use only
    jg::DevBuf cols, ncols;
    // grouped indexed merge (k_group_*): per-key list head of the batch being merged (gen << 32 | row,
    // generation-tagged: no reset between calls) and a next[] link per received row; first use
    jg::DevBuf head, next;
    unsigned long long head_gen = 0;  // generation of the last grouped batch (heads hold gen << 32 | row)
    // open streamed wave (jg_pnc_wave_*): payload, offsets, rows, status + deferred list; pass A's
    // resolved entries per message and its list of messages pass B must parse again (json.hip)
    jg::DevBuf wbytes, woff, wrows, wstat, wemit, wguid, wslow;
    uint64_t wn = 0, wnb = 0;
    uint64_t scan_hi = 0;  // messages pass A scanned since the wave began (its fused applies are undone below this)
    bool wopen = false;
    bool fuse = true;       // the wave's pass A applies what it proves (JANUS_JSON_FUSE, latched when the wave begins)
    bool status_clean = false;  // the wave status words hold their initial values (the last wave ended clean): no reset
    bool node_open = false;  // a node wave (node.hip) holds the store: see jg::require_writable
};

// Device-resident wave of encoded state messages (json.hip jg_wave_*; digest.hip reads it too).
struct jg_wave {
    jg_ctx* ctx;
    uint64_t cap_msgs, cap_bytes;
    uint64_t n = 0, n_bytes = 0;
    uint32_t max_key = 0;
    jg::DevBuf bytes, off, keys;
};

struct jg_rows {
    jg_ctx* ctx;
    uint64_t n_rows;
    uint32_t R;
    uint32_t eb;
    bool has_keys = false;
    uint32_t max_key = 0;  // largest key_idx uploaded (validated against the store at merge)
    jg::DevBuf P, N, keys;
};

// One sorted tag-record stream in the CHUNKED layout (orset_union.hpp): structure of arrays
// key[slot] (8 B), tag[slot] (16 B) and ord[slot] (4 B, the arrival ordinal: jg_tagrec.ord); chunk c
// holds ranks [off[c], off[c+1]) in slots [c*kChunk, c*kChunk + cnt[c]); lut[q] = the last chunk
// starting at or before rank q*512.
constexpr uint32_t kChunk = 3072;  // = one union tile (orset.hip kOB * kItems)
struct jg_stream_soa {
    jg::DevBuf block;          // one device block holding the six arrays below (views into it): one hipMalloc and
                               // one hipFree per reservation (hipFree costs ~0.2 ms of host time each on the box)
    jg::DevBuf key, tag, ord;  // cap_chunks * kChunk slots
    uint64_t next = 0;         // every record's ord < next (host copy; a union's B records land at next + ord)
    jg::DevBuf cnt;       // uint32 [cap_chunks]
    jg::DevBuf off;       // uint64 [cap_chunks + 1]
    jg::DevBuf lut;       // uint32 [(cap_chunks * kChunk >> 9) + 2]
    uint64_t cap_chunks = 0;
    uint64_t n = 0;       // records (host copy; see jg_orset::counts_pending)
    uint32_t nch = 0;     // chunks in use
    bool dense = true;    // chunks full except the last (slot = rank): uploads and generated streams
    void reserve_records(uint64_t records);  // room for a dense stream or a union output of `records`
    void swap(jg_stream_soa& o);
    std::vector<void*> retired;  // blocks of earlier reservations (reserve_records), freed at the next idle point
    void free_retired();         // hipFree them (the caller's streams have drained)
    jg_stream_soa() = default;
    jg_stream_soa(const jg_stream_soa&) = delete;
    jg_stream_soa& operator=(const jg_stream_soa&) = delete;
    ~jg_stream_soa();
};

struct jg_orset_wire;  // orset_wire.hip: element table + open payload wave (first use only)
namespace jg {
void orset_wire_free(jg_orset_wire* w);
void orset_wire_free_retired(jg_orset_wire* w);
}

struct jg_orset {
    jg_ctx* ctx;
    jg_stream_soa add, rem;
    jg_stream_soa spare_add, spare_rem;  // union target for in-place merges (swapped in)
    jg::DevBuf counts;     // device-side uint64 [2]: n_add, n_rem written by the union kernel
    bool counts_pending = false;  // an async union wrote `counts`; host n's are stale
    jg_orset_wire* wire = nullptr;
    bool node_open = false;  // a node wave (node.hip) holds the store: see jg::require_writable
    jg_orset() = default;
    jg_orset(const jg_orset&) = delete;
    jg_orset& operator=(const jg_orset&) = delete;
    ~jg_orset() { jg::orset_wire_free(wire); }
};

namespace jg {
using CtxLock = std::unique_lock<std::recursive_mutex>;
inline CtxLock lock(jg_ctx* c) { return c ? CtxLock(c->mu) : CtxLock(); }
constexpr size_t kPinRead = 32 << 10, kPinBytes = 64 << 10;
// Queue a small device -> host read into the context's page-locked bytes at `at` (< kPinRead); several reads
// share one pin_sync, then pin_at reads them.  Calls on a context are serialised (ctx->mu), and every reader
// syncs before it returns, so the bytes are free at the start of each call.
inline void pin_get(jg_ctx* ctx, size_t at, const void* d, size_t n) {
    if (at + n > kPinRead) fail(JG_EINVAL, "pin_get: %zu bytes at %zu exceed the page-locked read area", n, at);
    JG_HIP(hipMemcpyAsync(static_cast<char*>(ctx->hstat) + at, d, n, hipMemcpyDeviceToHost, ctx->stream));
}
inline void pin_sync(jg_ctx* ctx) { JG_HIP(hipStreamSynchronize(ctx->stream)); }  // (polling measured no gain)
inline const void* pin_at(jg_ctx* ctx, size_t at) { return static_cast<const char*>(ctx->hstat) + at; }
template <class H> inline CtxLock lock(const H* h) { return lock(h ? h->ctx : nullptr); }
// A node wave (node.hip) holds its stores from its begin to its end: the PN-Counter store's wave scratch and
// fused pass A's undo records, the OR-Set store's wave tables (whose element-table lookups assume the committed
// names do not change until the commit).  The one-call form runs under the context lock, but the streamed form
// (jg_apply_stream_begin / _append / _end) keeps the wave open across unlocked calls, so every call that writes
// a store, or reuses the scratch its open wave holds, is refused until the wave ends.
template <class S> inline void require_writable(const S* s, const char* fn) {
    JG_REQUIRE(!s || !s->node_open, JG_EINVAL, "%s: a node wave (jg_apply_stream_begin .. _end) holds this store", fn);
}
void ensure_device(jg_ctx* ctx);  // hipSetDevice(ctx->device) on the calling thread
void* scratch(jg_ctx* ctx, DevBuf& b, size_t bytes);
// After H2D copies queued on ctx->copy: make ctx->stream wait for them (stream order for the kernels
// that read the uploaded chunk).  Callers keep the copy stream off buffers the compute stream may still
// use: before a wave's first upload they record an event at the compute stream's tail (after every setup
// launch of the wave) and make ctx->copy wait on it on the device (node.hip `drained`; the one-shot
// jg_*_wave_append paths synchronise ctx->stream instead), and they synchronise ctx->copy before
// reallocating an upload target (grow_keep) — the same rule covers the D2H copies of issued OR-Set names
// that a commit queues on ctx->copy.
void upload_done(jg_ctx* ctx);
void sync_counts(jg_orset* s);   // fold a pending async count into the host copy
// Dense chunk metadata for a stream whose n records sit contiguously in slots [0, n) (async).
void set_dense(jg_ctx* ctx, jg_stream_soa& s, uint64_t n);
// pnc.hip: scatter-max of n_rows device rows into the store's keys (async on the store's stream).
void pnc_merge_indexed(jg_pnc* p, const void* BP, const void* BN, const uint32_t* d_keys, uint64_t n_rows);
// orset.hip: merge n_runs sorted, duplicate-free runs (device SoA, run after run) into the store.
void orset_merge_runs(jg_orset* s, uint32_t n_runs, const uint64_t* add_counts, const uint64_t* rem_counts, const unsigned long long* add_key,
                      const uint4* add_tag, const uint32_t* add_ord, const unsigned long long* rem_key, const uint4* rem_tag,
                      const uint32_t* rem_ord);
// orset.hip: largest ord + 1 of n device ords (0 if n == 0), synchronous.
uint64_t ord_span(jg_ctx* ctx, const uint32_t* ord, uint64_t n);
// orset.hip: s = s ∪ src (both streams), src's streams may be dense or chunked; synchronous (the union's error
// flag and counts read back) unless `defer`: then the counts stay pending for orset_pin_pending / _settle.
void orset_merge_store(jg_orset* s, jg_orset* src, bool defer = false);
// orset.hip: a deferred union's error flag and counts queued into the context's page-locked bytes at [at, at
// + 24) (no sync: the caller's own pin_sync brings them with its words; false if nothing is pending), and
// taken from there after that sync (the flag raised as the synchronous merge would).
bool orset_pin_pending(jg_orset* s, size_t at);
// hipFree the blocks the store's streams and element table retired while growing (the caller's streams drained)
void orset_free_retired(jg_orset* s);
// jg_orset_encode_json's first step: every record of the sets d_sets[0..n) (device), query by query, add side then
// tombstones, in store order (element id, tag), into `buf` (grown as needed): key, tag, ord, query << 1 | side, and
// keep = ord below d_lim[q << 1 | side] (d_lim NULL: every record).  roff: [2n + 1] segment offsets.  One round trip.
struct OrsetGathered {
    uint64_t R;
    unsigned long long *key, *tlo, *thi, *roff;
    uint32_t *ord, *qs;
    uint8_t* keep;
};
OrsetGathered orset_gather_sets(jg_orset* s, uint64_t n, const uint32_t* d_sets, const unsigned long long* d_lim, jg::DevBuf& buf);
void orset_settle_pending(jg_orset* s, size_t at);
// orset.hip: room in the store's union targets for that many more records (no sync; skipped while counts are pending).
void orset_reserve_union(jg_orset* s, uint64_t add_in, uint64_t rem_in);

// Node waves (node.hip): one upload of every kind's messages; rows / mset = the message's row / set id
// or kSkipIdx.  json.hip (PN-Counter):
void pnc_node_begin(jg_pnc* p, uint64_t n);
void pnc_node_scan(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t m0, uint64_t m1);
int pnc_node_finish(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, uint64_t* bad, std::string* why);
int pnc_node_prefix(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, uint64_t* bad, std::string* why);
void pnc_node_undo(jg_pnc* p, const uint32_t* rows);
// SHA-256 of n device-resident payloads into host out (n * 32 bytes), queued on ctx->stream (digest.hip)
void sha256_device(jg_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* out);  // a node wave abandoned after its chunks' (fused) pass A
// orset_wire.hip (OR-Set):
void orset_node_begin(jg_orset* s, uint8_t* bytes, uint64_t* off, uint32_t* mset, uint64_t n, uint64_t nbytes, uint32_t max_set);
void orset_node_parse(jg_orset* s, uint64_t m0, uint64_t m1);
int orset_node_check(jg_orset* s, uint64_t n, uint64_t nbytes, uint64_t* bad, std::string* why);
void orset_node_commit(jg_orset* s, uint64_t limit);
void orset_node_abort(jg_orset* s);
void orset_node_no_names(jg_orset* s);
}  // namespace jg
