// node.hip — the committed-wave apply loop behind the C ABI (SURVEY.md §8a A13, §8b B2 jg_apply_batch).
//
// SafeCRDTManager.HandleAfterConsensusUpdates (BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:109-160) walks a
// committed wave message by message: skip ManagerMsg_Create and Guid.Empty (:133-134), look the uid up in
// safeCRDTsIndexedByuid (:136), ApplyUpdateStable = Decode + Merge (SafeCRDT.cs:80-83), then
// safeUpdateTracker.TryRemove + notify (:141-142).  jg_apply_committed does the whole wave in one call:
//
//   host        the library's workers gather chunk c (payloads, uids, identities, types) into pinned
//               staging with non-temporal line stores while the device works on chunk c-1 — the only
//               per-message host work left (no table is touched on the host);
//   copy        the chunk's H2D on the context's copy stream;
//   k_classify  one lane per message: the skip rule, uid -> (type, row / set id) in the device uid table
//               (32-B slots, linear probing: one line per lookup), the tracker slot of the message's
//               identity and a first-occurrence claim on it (atomicMin of the commit index);
//   passes      the PN-Counter pass A (json_wave.hpp) and the OR-Set parse (orset_wire.hip) over the
//               chunk, each skipping the other kind's messages (row / set id kSkipIdx);
//   end         OR-Set check -> first rejected state (the cut); PN-Counter commit (all or nothing, the
//               prefix re-run when something cut the wave); OR-Set commit up to the cut; k_complete: a
//               message before the cut that claimed its identity first turns the tracker entry into a
//               tombstone and reports the origin; origins compacted in commit order (hipcub select).
//
// Uid table: open addressing over 32-B slots {uid lo, uid hi, type << 31 | idx}, (0, 0) = empty (Guid.Empty
// is never a key, :134); load <= 1/2.  The library keeps the authoritative copy on the host (registration
// is rare: key creation) and uploads the slots a registration touched before the next wave.
// Tracker: open addressing over 16-B slots {identity, origin}, 0 = empty, ~0 = removed (a tombstone:
// concurrent probes never see an entry move); rebuilt without tombstones when live + removed pass 1/2.
#include <cstring>
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <unordered_set>
#include <vector>

#include "host_pool.hpp"
#include "jg_internal.hpp"

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr unsigned long long kTomb = ~0ull;
constexpr uint32_t kOrSetBit = 0x80000000u;

unsigned blocks_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + kBlock - 1) / kBlock); }
uint64_t pow2_at_least(uint64_t x, uint64_t lo = 1024) {
    uint64_t p = lo;
    while (p < x) p <<= 1;
    return p;
}

struct UidSlot {
    unsigned long long lo, hi;
    uint32_t val, pad0;
    unsigned long long pad1;
};
static_assert(sizeof(UidSlot) == 32, "one uid slot = half a 64-B line");
struct TrackSlot { unsigned long long key, origin; };
struct Guid16 { unsigned long long lo, hi; };

using jg::uid_hash;
__host__ __device__ __forceinline__ uint32_t shard_of(uint64_t lo, uint64_t hi, uint32_t world) { return jg::shard_of_uid(lo, hi, world); }
__host__ __device__ __forceinline__ uint64_t seq_hash(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}

struct DevUids { const UidSlot* tab; uint64_t mask; };
struct DevTrack { TrackSlot* tab; uint32_t* claim; uint64_t mask; };

__global__ void k_uid_scatter(UidSlot* __restrict__ tab, const uint32_t* __restrict__ at, const UidSlot* __restrict__ v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) tab[at[i]] = v[i];
}

// TryAdd of pending (identity, origin) pairs, in add order: an identity already present keeps its entry,
// and an identity added twice in one batch keeps the origin of its FIRST add (ConcurrentDictionary.TryAdd,
// SafeCRDT.cs:55; ADVICE r03: whichever lane won the CAS used to keep its origin).  Pass 1 inserts the keys;
// every pair whose slot is new in this batch (origin still 0: origins are never 0, jg_tracker_add) claims it
// with atomicMin of its pair index in the slot's claim word (all 0xFFFFFFFF between waves); pass 2
// (k_track_origin) lets the smallest index write the origin and resets the claim.  *count += added.
__global__ __launch_bounds__(kBlock) void k_track_insert(DevTrack t, const unsigned long long* __restrict__ pairs, uint64_t n,
                                                         uint32_t* __restrict__ slot_of, unsigned long long* __restrict__ count) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool added = false;
    if (i < n) {
        const unsigned long long k = pairs[2 * i];
        uint32_t slot = kNoSlot;
        for (uint64_t s = seq_hash(k) & t.mask;; s = (s + 1) & t.mask) {
            unsigned long long w = t.tab[s].key;
            if (w == 0) {
                w = atomicCAS(&t.tab[s].key, 0ull, k);
                if (w == 0) {
                    added = true;
                    slot = (uint32_t)s;
                    break;
                }
            }
            if (w == k) {
                slot = (uint32_t)s;
                break;
            }
        }
        if (t.tab[slot].origin == 0) {  // new in this batch (an entry of an earlier batch has its origin)
            atomicMin(&t.claim[slot], (uint32_t)i);
        } else {
            slot = kNoSlot;
        }
        slot_of[i] = slot;
    }
    __shared__ uint32_t c;
    if (threadIdx.x == 0) c = 0;
    __syncthreads();
    if (added) atomicAdd(&c, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && c) atomicAdd(count, (unsigned long long)c);
}

__global__ void k_track_origin(DevTrack t, const unsigned long long* __restrict__ pairs, const uint32_t* __restrict__ slot_of, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = slot_of[i];
    if (s == kNoSlot || t.claim[s] != (uint32_t)i) return;
    t.tab[s].origin = pairs[2 * i + 1];
    t.claim[s] = 0xFFFFFFFFu;
}

// Live entries of the old table into the new one (tombstones dropped).
__global__ void k_track_rehash(const TrackSlot* __restrict__ old, uint64_t old_cap, DevTrack t) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= old_cap) return;
    const TrackSlot e = old[i];
    if (e.key == 0 || e.key == kTomb) return;
    for (uint64_t s = seq_hash(e.key) & t.mask;; s = (s + 1) & t.mask)
        if (atomicCAS(&t.tab[s].key, 0ull, e.key) == 0ull) {
            t.tab[s].origin = e.origin;
            return;
        }
}

__global__ void k_track_lookup(DevTrack t, const unsigned long long* __restrict__ seq, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const unsigned long long k = seq[i];
    uint8_t r = 0;
    if (k != 0 && k != kTomb && t.tab)
        for (uint64_t s = seq_hash(k) & t.mask;; s = (s + 1) & t.mask) {
            const unsigned long long w = t.tab[s].key;
            if (w == 0) break;
            if (w == k) { r = 1; break; }
        }
    out[i] = r;
}

// A chunk's per-message arrays arrive as ONE upload (the staging layout: end offsets [m + 1] from 0, uids
// [m], identities [m], types [m], back to back) and are scattered here into the wave's arrays, offsets
// rebased to the chunk's first payload byte: one copy per chunk instead of four (each copy on the queue
// cost ~8-17 us of gap on top of its bytes: ~60 us per 131k-message chunk, 6 % of its upload).
__global__ __launch_bounds__(kBlock) void k_unstage(const uint8_t* __restrict__ meta, uint64_t m, uint64_t m0, uint64_t b0,
                                                    uint64_t* __restrict__ off, Guid16* __restrict__ uid, uint64_t* __restrict__ seq,
                                                    uint8_t* __restrict__ type) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= m) return;
    const auto* soff = reinterpret_cast<const uint64_t*>(meta);
    const auto* suid = reinterpret_cast<const uint64_t*>(soff + m + 1);  // 8-B aligned: two words per uid
    const auto* sseq = suid + 2 * m;
    const auto* stype = reinterpret_cast<const uint8_t*>(sseq + m);
    off[m0 + 1 + j] = soff[j + 1] + b0;
    uid[m0 + j] = Guid16{suid[2 * j], suid[2 * j + 1]};
    seq[m0 + j] = sseq[j];
    type[m0 + j] = stype[j];
}

// Per message of [m0, m1): the loop's skip rule (:133-134), the uid lookup (:136), the tracker slot of its
// identity and a first-occurrence claim.  status[0] = first CRDT state of an unknown uid (block mode).
__global__ __launch_bounds__(kBlock) void k_classify(const Guid16* __restrict__ uid, const uint8_t* __restrict__ type,
                                                     const unsigned long long* __restrict__ seq, uint64_t m0, uint64_t m1, DevUids u,
                                                     DevTrack t, uint32_t* __restrict__ rows, uint32_t* __restrict__ mset,
                                                     uint32_t* __restrict__ tslot, unsigned long long* __restrict__ status) {
    const uint64_t i = m0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= m1) return;
    uint32_t r = jg::kSkipIdx, s = jg::kSkipIdx, ts = kNoSlot;
    const Guid16 g = uid[i];
    if (type[i] != 0 && (g.lo | g.hi) != 0) {  // CRDTMsg of a key (not ManagerMsg_Create, not the key space)
        uint32_t v = kNoSlot;
        for (uint64_t q = uid_hash(g.lo, g.hi) & u.mask;; q = (q + 1) & u.mask) {
            const UidSlot e = u.tab[q];
            if ((e.lo | e.hi) == 0) break;
            if (e.lo == g.lo && e.hi == g.hi) { v = e.val; break; }
        }
        if (v == kNoSlot) {
            atomicMin(status, (unsigned long long)i);  // TryGetValue false: skipped (:136); KeyNotFound in RM:329
        } else {
            if (v & kOrSetBit) s = v & ~kOrSetBit;
            else r = v;
            const unsigned long long k = seq[i];
            if (t.tab && k != 0 && k != kTomb)
                for (uint64_t q = seq_hash(k) & t.mask;; q = (q + 1) & t.mask) {
                    const unsigned long long w = t.tab[q].key;
                    if (w == 0) break;
                    if (w == k) {
                        ts = (uint32_t)q;
                        if (t.claim[q] > (uint32_t)i) atomicMin(&t.claim[q], (uint32_t)i);
                        break;
                    }
                }
        }
    }
    rows[i] = r;
    mset[i] = s;
    tslot[i] = ts;
}

// Messages before the cut: the first occurrence of a tracked identity removes the entry (TryRemove) and
// reports its origin (the notifier call); every other message reports 0.
__global__ void k_complete(const uint32_t* __restrict__ tslot, uint64_t cut, DevTrack t, unsigned long long* __restrict__ origin) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= cut) return;
    const uint32_t ts = tslot[i];
    unsigned long long o = 0;
    if (ts != kNoSlot && t.claim[ts] == (uint32_t)i) {
        o = t.tab[ts].origin;
        t.tab[ts].key = kTomb;
    }
    origin[i] = o;
}

__global__ void k_claim_reset(const uint32_t* __restrict__ tslot, uint64_t n, uint32_t* __restrict__ claim) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && tslot[i] != kNoSlot) claim[tslot[i]] = 0xFFFFFFFFu;
}

__global__ void k_count_sub(unsigned long long* __restrict__ count, const unsigned long long* __restrict__ sub) { *count -= *sub; }

// Messages before the cut that reached a registered key (the states the loop applied) into *out.
__global__ __launch_bounds__(kBlock) void k_count_applied(const uint32_t* __restrict__ rows, const uint32_t* __restrict__ mset, uint64_t cut,
                                                          unsigned long long* __restrict__ out) {
    uint32_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < cut; i += (uint64_t)gridDim.x * kBlock)
        c += (rows[i] != jg::kSkipIdx || mset[i] != jg::kSkipIdx) ? 1u : 0u;
    __shared__ uint32_t s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    atomicAdd(&s, c);
    __syncthreads();
    if (threadIdx.x == 0 && s) atomicAdd(out, (unsigned long long)s);
}

struct NonZero {
    __host__ __device__ bool operator()(const unsigned long long& x) const { return x != 0; }
};

void ensure(jg::DevBuf& b, size_t bytes) {
    if (b.bytes < bytes) b.alloc(bytes + bytes / 4 + 256);
}

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

struct jg_tracker {
    jg_ctx* ctx;
    // jg_tracker_add runs on the callers' threads (SafeCRDT.Update), not under the context lock: it appends
    // (identity, origin) pairs to page-locked buffer `cur` under pend_mu; a flush uploads that buffer
    // (async, stream-ordered before the wave's classify), records the buffer's event after the copy and
    // switches to the other one.  A buffer is written or reallocated only after its event completed (the
    // first append after a switch waits on it): no call has to end with a stream sync for the pair of
    // buffers to be safe (an empty wave returned after a flush without one).
    std::mutex pend_mu;
    // A buffer is a list of page-locked blocks filled in order and kept across flushes (round 6: one block grown by
    // doubling cost a hipHostMalloc + copy + hipHostFree — which waits for the device — each time the pending adds
    // outgrew it: 10-30 ms spikes in the producer bench, whose adds accumulate with no wave to flush them).
    struct Block {
        unsigned long long* p = nullptr;
        size_t cap = 0, n = 0;  // pairs
    };
    struct Pin {
        std::vector<Block> blocks;
        size_t at = 0;            // the block being filled
        size_t n = 0;             // pairs pending over all blocks
        hipEvent_t up = nullptr;  // recorded after the buffer's last upload
        bool wait = false;        // the upload may still be queued: wait on `up` before touching the blocks
        void reset() {
            for (Block& k : blocks) k.n = 0;
            at = 0;
            n = 0;
        }
    } pin[2];
    int cur = 0;
    jg::DevBuf tab, claim, count, dpairs;
    jg::DevBuf spare_tab, spare_claim;  // the other pair of a rebuild (tables are rebuilt into it, then swapped)
    uint64_t cap = 0;
    uint64_t used = 0;  // live + tombstones, an upper bound (TryAdd of a present identity counted too)
    int waves = 0;      // node waves using the tracker (a streamed one spans unlocked calls): destroy is refused

    ~jg_tracker() {
        for (Pin& b : pin) {
            if (b.up) (void)hipEventSynchronize(b.up);
            for (Block& k : b.blocks)
                if (k.p) (void)hipHostFree(k.p);
            if (b.up) (void)hipEventDestroy(b.up);
        }
    }
    DevTrack dev() const { return DevTrack{tab.as<TrackSlot>(), claim.as<uint32_t>(), cap ? cap - 1 : 0}; }

    void append(uint64_t n, const uint64_t* seq, const uint64_t* origin) {  // under pend_mu
        Pin& b = pin[cur];
        if (b.wait) {  // its last upload (queued by the flush before the one that switched to it) must be done
            JG_HIP(hipEventSynchronize(b.up));
            b.wait = false;
        }
        uint64_t i = 0;
        while (i < n) {
            if (b.at == b.blocks.size()) {  // a new block, twice the last (64k .. 4M pairs), at least what is left
                const size_t last = b.blocks.empty() ? 0 : b.blocks.back().cap;
                const size_t nc = std::max<size_t>(std::min<size_t>(std::max<size_t>(2 * last, 65536), size_t(1) << 22), std::min<uint64_t>(n - i, size_t(1) << 22));
                void* p = nullptr;
                JG_HIP(hipHostMalloc(&p, nc * 16, hipHostMallocDefault));
                b.blocks.push_back(Block{static_cast<unsigned long long*>(p), nc, 0});
            }
            Block& k = b.blocks[b.at];
            const uint64_t take = std::min<uint64_t>(n - i, k.cap - k.n);
            for (uint64_t j = 0; j < take; ++j) {
                k.p[2 * (k.n + j)] = seq[i + j];
                k.p[2 * (k.n + j) + 1] = origin[i + j];
            }
            k.n += take;
            b.n += take;
            i += take;
            if (k.n == k.cap) ++b.at;
        }
    }

    // The pending adds into the device table, queued on the context's stream (under the context lock).
    void flush() {
        Pin* b;
        {
            std::lock_guard<std::mutex> g(pend_mu);
            b = &pin[cur];
            cur ^= 1;
            pin[cur].reset();
            pin[cur].wait = pin[cur].up != nullptr;  // appends to it wait for its previous upload first
        }
        if (!count.p) {
            count.alloc(8);
            JG_HIP(hipMemsetAsync(count.p, 0, 8, ctx->stream));
        }
        const uint64_t np = b->n;
        if (np == 0) return;
        if (cap == 0 || 2 * (used + np) > cap) {  // rebuild without tombstones, into the spare table
            unsigned long long live = 0;
            if (cap) {
                JG_HIP(hipMemcpyAsync(&live, count.p, 8, hipMemcpyDeviceToHost, ctx->stream));
                JG_HIP(hipStreamSynchronize(ctx->stream));
            }
            const uint64_t ncap = pow2_at_least(4 * (live + np), 4096);
            // the spare is the table before the last rebuild: reused while it is large enough (a steady
            // wave stream rebuilds every wave or two at the same capacity; hipMalloc + hipFree of the
            // tables cost ~0.7 ms of a C5 wave's setup), freed-and-grown otherwise.  Stream order keeps
            // the rehash reading the old table before anything clears it.
            if (spare_tab.bytes < ncap * sizeof(TrackSlot)) spare_tab.alloc(ncap * sizeof(TrackSlot));
            if (spare_claim.bytes < ncap * 4) spare_claim.alloc(ncap * 4);
            JG_HIP(hipMemsetAsync(spare_tab.p, 0, ncap * sizeof(TrackSlot), ctx->stream));
            JG_HIP(hipMemsetAsync(spare_claim.p, 0xFF, ncap * 4, ctx->stream));
            const DevTrack nd{spare_tab.as<TrackSlot>(), spare_claim.as<uint32_t>(), ncap - 1};
            if (cap) hipLaunchKernelGGL(k_track_rehash, dim3(blocks_for(cap)), dim3(kBlock), 0, ctx->stream, tab.as<TrackSlot>(), cap, nd);
            JG_HIP(hipGetLastError());
            std::swap(tab.p, spare_tab.p);
            std::swap(tab.bytes, spare_tab.bytes);
            std::swap(claim.p, spare_claim.p);
            std::swap(claim.bytes, spare_claim.bytes);
            cap = ncap;
            used = live;
        }
        ensure(dpairs, np * 20);  // pairs, then each pair's slot
        uint64_t at = 0;
        for (const Block& k : b->blocks) {
            if (k.n == 0) break;  // blocks fill in order
            JG_HIP(hipMemcpyAsync(dpairs.as<char>() + at * 16, k.p, k.n * 16, hipMemcpyHostToDevice, ctx->stream));
            at += k.n;
        }
        if (!b->up) JG_HIP(hipEventCreateWithFlags(&b->up, hipEventDisableTiming));
        JG_HIP(hipEventRecord(b->up, ctx->stream));
        auto* slot_of = reinterpret_cast<uint32_t*>(dpairs.as<char>() + np * 16);
        hipLaunchKernelGGL(k_track_insert, dim3(blocks_for(np)), dim3(kBlock), 0, ctx->stream, dev(), dpairs.as<unsigned long long>(), np, slot_of,
                           count.as<unsigned long long>());
        hipLaunchKernelGGL(k_track_origin, dim3(blocks_for(np)), dim3(kBlock), 0, ctx->stream, dev(), dpairs.as<unsigned long long>(), slot_of, np);
        JG_HIP(hipGetLastError());
        used += np;
    }
};

// One wave in flight on a node.  jg_apply_committed / jg_apply_block run it from begin to end in one call; the
// streamed form (jg_apply_stream_begin / _append / _end) hands the wave over part by part, so a caller that copies
// its committed byte[]s into page-locked memory block by block overlaps that copy with the
// uploads and parses of the parts before.  Messages are numbered in hand-over order (= commit order).
struct WaveRun {
    bool active = false, block_mode = false, filter = false, trace = false, do_pnc = false, do_orset = false;
    bool held = false;  // wave_end is running: the stores are still held (hold) though no more parts are taken
    jg_tracker* tr = nullptr;
    uint64_t n = 0, total_bytes = 0;  // the wave's messages and payload bytes (stream: upper bounds from begin)
    uint64_t seen = 0;                // messages handed over (commit index of the next)
    uint64_t m0 = 0, b0 = 0, mo = 0;  // messages, payload bytes and meta bytes on the device
    uint64_t meta_cap = 0;
    size_t n_ev = 0, chunk_msgs = 0, tail = 0, min_par = 0;
    uint32_t rank = 0, world = 1;
    double t_begin = 0, t_loop = 0, t_gather = 0;
    hipEvent_t up_ev[2] = {nullptr, nullptr};
    DevUids du{};
    DevTrack dt{};
    std::vector<uint64_t> tcnt, tbytes;
};

struct jg_node {
    jg_ctx* ctx;
    jg_pnc* pnc;
    jg_orset* orset;
    // uid table: host copy (authoritative) + device copy
    std::vector<UidSlot> htab;
    uint64_t n_keys = 0, n_pnc = 0, n_orset = 0;
    uint32_t max_set = 0;
    jg::DevBuf dtab;
    bool upload_all = true;
    std::vector<uint32_t> dirty;
    // key-space shard (jg_node_set_shard)
    uint32_t shard_rank = 0, shard_world = 1;
    bool foreign = false;
    // the wave on the device
    jg::DevBuf bytes, off, uid, seq, type, rows, mset, tslot, origin, done, status, cub;
    jg::DevBuf meta;  // the wave's per-message arrays as uploaded, chunk after chunk (k_unstage)
    // pinned staging arenas, carved front to back each wave and kept
    std::vector<std::pair<char*, size_t>> arenas;
    size_t arena_i = 0, arena_off = 0;
    std::unique_ptr<jg::WorkerPool> pool;
    double avg_msg_bytes = 357.0;
    std::vector<uint64_t> dmap;  // device index -> commit index (when the shard shortcut dropped messages)
    jg_apply_stats stats{};
    std::vector<hipEvent_t> ev;  // pairs around each chunk's kernels and the final phase (device_busy_s)
    hipEvent_t drained = nullptr;  // the compute stream's tail when a wave starts (the copy queue waits on it)
    WaveRun run;                   // the wave in flight (one call, or a streamed wave between begin and end)

    ~jg_node() {
        for (auto& a : arenas) (void)hipHostFree(a.first);
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        if (drained) (void)hipEventDestroy(drained);
    }
    hipEvent_t event(size_t k) {
        while (ev.size() <= k) {
            hipEvent_t e;
            JG_HIP(hipEventCreate(&e));
            ev.push_back(e);
        }
        return ev[k];
    }
    jg::WorkerPool& workers() {
        const int want = jg::host_threads();
        if (!pool || pool->size() != want) pool = std::make_unique<jg::WorkerPool>(want);
        return *pool;
    }
    char* stage(size_t n) {
        n = (n + 255) & ~size_t(255);
        while (arena_i < arenas.size() && arena_off + n > arenas[arena_i].second) {
            ++arena_i;
            arena_off = 0;
        }
        if (arena_i == arenas.size()) {  // a bigger wave: one more arena as large as the pool so far
            size_t total = 0;
            for (const auto& a : arenas) total += a.second;
            const size_t cap = std::max({n, total, size_t(64) << 20});
            void* p = nullptr;
            JG_HIP(hipHostMalloc(&p, cap, hipHostMallocDefault));
            arenas.emplace_back(static_cast<char*>(p), cap);
            arena_off = 0;
        }
        char* r = arenas[arena_i].first + arena_off;
        arena_off += n;
        return r;
    }
    bool insert(const UidSlot& e) {  // host table; false if present
        const uint64_t mask = htab.size() - 1;
        for (uint64_t q = uid_hash(e.lo, e.hi) & mask;; q = (q + 1) & mask) {
            UidSlot& s = htab[q];
            if ((s.lo | s.hi) == 0) {
                s = e;
                if (!upload_all) dirty.push_back((uint32_t)q);
                return true;
            }
            if (s.lo == e.lo && s.hi == e.hi) return false;
        }
    }
    const UidSlot* find(uint64_t lo, uint64_t hi) const {
        if (htab.empty()) return nullptr;
        const uint64_t mask = htab.size() - 1;
        for (uint64_t q = uid_hash(lo, hi) & mask;; q = (q + 1) & mask) {
            const UidSlot& s = htab[q];
            if ((s.lo | s.hi) == 0) return nullptr;
            if (s.lo == lo && s.hi == hi) return &s;
        }
    }
    void grow(uint64_t total) {
        if (!htab.empty() && 2 * total <= htab.size()) return;
        std::vector<UidSlot> old;
        old.swap(htab);
        htab.assign(pow2_at_least(4 * total), UidSlot{0, 0, 0, 0, 0});
        upload_all = true;
        dirty.clear();
        for (const UidSlot& s : old)
            if ((s.lo | s.hi) != 0) insert(s);
    }
    void sync_table() {  // the registrations since the last wave, to the device
        if (upload_all) {
            if (htab.empty()) grow(1);
            dtab.alloc(htab.size() * sizeof(UidSlot));
            JG_HIP(hipMemcpyAsync(dtab.p, htab.data(), dtab.bytes, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            upload_all = false;
            dirty.clear();
            return;
        }
        if (dirty.empty()) return;
        const uint64_t n = dirty.size();
        std::vector<UidSlot> v(n);
        for (uint64_t i = 0; i < n; ++i) v[i] = htab[dirty[i]];
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * 36 + 512));
        auto* dat = reinterpret_cast<uint32_t*>(st);
        auto* dv = reinterpret_cast<UidSlot*>(st + ((n * 4 + 255) & ~255ull));
        JG_HIP(hipMemcpyAsync(dat, dirty.data(), n * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(dv, v.data(), n * sizeof(UidSlot), hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_uid_scatter, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, dtab.as<UidSlot>(), dat, dv, n);
        JG_HIP(hipGetLastError());
        JG_HIP(hipStreamSynchronize(ctx->stream));
        dirty.clear();
    }
    bool shortcut() const { return shard_world > 1 && !foreign; }
};

namespace {

bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// A fault injector for one test: JANUS_TEST_ORSET_COMMIT_FAIL=1 makes the wave's OR-Set commit raise its device
// error flag, so the deferred error path (completions reported first, then the error) runs without a real
// overflow.  Compiled into the test build only (lib/libjanusgpu_test.so, -DJANUS_TEST_HOOKS): the
// production library has no injector on its path.
#ifdef JANUS_TEST_HOOKS
bool test_commit_fail() {
    const char* e = std::getenv("JANUS_TEST_ORSET_COMMIT_FAIL");
    return e && e[0] == '1';
}
#else
constexpr bool test_commit_fail() { return false; }
#endif
constexpr size_t kTask = 2048;

// Every wave, empty ones too: the figures reset, names pending from the last commit dropped, the uid table's
// registrations and the tracker's adds to the device, the staging arenas reused.
void wave_prologue(jg_node* nd, jg_tracker* tr, double* tp) {
    nd->stats = jg_apply_stats{};
    tp[0] = now_s();
    if (nd->orset) jg::orset_node_no_names(nd->orset);
    tp[1] = now_s();
    nd->sync_table();
    tp[2] = now_s();
    if (tr) tr->flush();
    tp[3] = now_s();
    nd->arena_i = nd->arena_off = 0;  // the previous wave's chunks are no longer referenced
    nd->dmap.clear();
}

// A wave holds its node's stores (and tracker) from wave_begin to the end of wave_end / wave_abort: the calls that
// would write them or reuse the scratch the wave keeps are refused meanwhile (jg::require_writable).
void hold(jg_node* nd, jg_tracker* tr, bool on) {
    if (nd->pnc) nd->pnc->node_open = on;
    if (nd->orset) nd->orset->node_open = on;
    if (tr) tr->waves += on ? 1 : -1;
}

// Setup: the prologue, buffers for `n` messages / `total_bytes` payload bytes and up to `max_chunks` chunks, both
// parsers opened.
void wave_begin(jg_node* nd, WaveRun& r, jg_tracker* tr, uint64_t n, uint64_t total_bytes, uint64_t max_chunks, bool block_mode, bool filter) {
    jg::require_writable(nd->pnc, "jg_apply");  // another node's streamed wave holds a shared store
    jg::require_writable(nd->orset, "jg_apply");
    r = WaveRun{};
    r.t_begin = now_s();
    r.tr = tr;
    r.n = n;
    r.total_bytes = total_bytes;
    r.block_mode = block_mode;
    r.filter = filter;
    r.rank = nd->shard_rank;
    r.world = nd->shard_world;
    jg_ctx* ctx = nd->ctx;
    static const bool trace = std::getenv("JANUS_TRACE_APPLY") != nullptr;  // setup phases to stderr
    r.trace = trace;
    double tp[8];
    wave_prologue(nd, tr, tp);
    // chunks: ~48 MB of payload each (sized from the previous wave's bytes per message), the last 16k
    // messages a chunk of their own (its upload + passes are the part no host work overlaps)
    // (read per call: tests narrow them)
    const char* ce = std::getenv("JANUS_WAVE_CHUNK");
    const size_t chunk_env = ce ? std::max<size_t>(1, std::strtoull(ce, nullptr, 10)) : size_t{0};
    const char* pe = std::getenv("JANUS_HOST_PAR_MIN");  // below this many messages a chunk is gathered on the caller alone
    r.min_par = pe ? (size_t)std::strtoull(pe, nullptr, 10) : size_t{8192};
    r.chunk_msgs = chunk_env ? chunk_env : std::clamp<size_t>((size_t)((48u << 20) / std::max(nd->avg_msg_bytes, 64.0)), 8192, 131072);
    r.tail = std::max<size_t>(1, std::min<size_t>(16384, r.chunk_msgs / 8));
    r.tcnt.assign((r.chunk_msgs + kTask - 1) / kTask + 2, 0);
    r.tbytes.assign(r.tcnt.size(), 0);
    tp[4] = now_s();
    ensure(nd->bytes, ((total_bytes + 15) & ~15ull) + 64);  // the parsers read aligned 16-byte windows
    ensure(nd->off, (n + 1) * 8);
    ensure(nd->uid, n * 16);
    ensure(nd->seq, n * 8);
    ensure(nd->type, n);
    ensure(nd->rows, n * 4);
    ensure(nd->mset, n * 4);
    ensure(nd->tslot, n * 4);
    ensure(nd->status, 64);
    r.meta_cap = n * 33 + 72 * (max_chunks + 1);  // per chunk: 33 m + 8 bytes, 64-B aligned
    ensure(nd->meta, r.meta_cap);
    r.do_pnc = nd->pnc && nd->n_pnc > 0;
    r.do_orset = nd->orset && nd->n_orset > 0;
    r.du = DevUids{nd->dtab.as<UidSlot>(), nd->htab.size() - 1};
    r.dt = tr && tr->cap ? tr->dev() : DevTrack{nullptr, nullptr, 0};
    // the copy queue must not overwrite buffers kernels queued earlier on the compute stream still read:
    // it waits for the stream's tail on the device (a host sync here also waited for the tracker adds
    // just queued, 0.3-0.4 ms of every C5 wave before the first gather)
    if (!nd->drained) JG_HIP(hipEventCreateWithFlags(&nd->drained, hipEventDisableTiming));
    JG_HIP(hipEventRecord(nd->drained, ctx->stream));
    JG_HIP(hipStreamWaitEvent(ctx->copy, nd->drained, 0));
    tp[5] = now_s();
    JG_HIP(hipMemsetAsync(nd->off.as<uint64_t>(), 0, 8, ctx->stream));
    JG_HIP(hipMemsetAsync(nd->status.as<unsigned long long>(), 0xFF, 64, ctx->stream));
    if (r.do_pnc) jg::pnc_node_begin(nd->pnc, n);
    tp[6] = now_s();
    if (r.do_orset) jg::orset_node_begin(nd->orset, nd->bytes.as<uint8_t>(), nd->off.as<uint64_t>(), nd->mset.as<uint32_t>(), n, total_bytes, nd->max_set);
    tp[7] = now_s();
    if (trace)
        std::fprintf(stderr, "apply setup: checks %.0f us, names %.0f, uid table %.0f, tracker adds %.0f, sizes %.0f, buffers %.0f, pnc begin %.0f, orset begin %.0f\n",
                     (tp[0] - r.t_begin) * 1e6, (tp[1] - tp[0]) * 1e6, (tp[2] - tp[1]) * 1e6, (tp[3] - tp[2]) * 1e6, (tp[4] - tp[3]) * 1e6,
                     (tp[5] - tp[4]) * 1e6, (tp[6] - tp[5]) * 1e6, (tp[7] - tp[6]) * 1e6);
    if (filter) nd->dmap.resize(n);
    // trace mode: timing events on the copy queue before the first upload and after the last one
    if (trace) {
        for (hipEvent_t& e : r.up_ev) JG_HIP(hipEventCreate(&e));
        JG_HIP(hipEventRecord(r.up_ev[0], ctx->copy));
    }
    r.t_loop = now_s();
    nd->stats.setup_s = r.t_loop - r.t_begin;
    r.active = true;
    hold(nd, tr, true);
}

// A wave rejected mid-loop (offsets checked chunk by chunk) or a device error: what pass A applied is undone, and the chunks
// already classified took first-occurrence claims on tracker slots; release them for the next wave.
void wave_abort(jg_node* nd, WaveRun& r, uint64_t claimed) {
    jg_ctx* ctx = nd->ctx;
    if (r.dt.tab && claimed)
        hipLaunchKernelGGL(k_claim_reset, dim3(blocks_for(claimed)), dim3(kBlock), 0, ctx->stream, nd->tslot.as<uint32_t>(), claimed, r.dt.claim);
    // the chunks' pass A applied the PN-Counter states it proved (fused): taken back, the store as before the wave
    if (r.do_pnc) {
        try {
            jg::pnc_node_undo(nd->pnc, nd->rows.as<uint32_t>());
        } catch (...) {
        }
    }
    (void)hipStreamSynchronize(ctx->copy);
    (void)hipStreamSynchronize(ctx->stream);
    if (r.do_orset) jg::orset_node_abort(nd->orset);
    for (hipEvent_t& e : r.up_ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    if (r.active || r.held) hold(nd, r.tr, false);
    r.active = r.held = false;
}

// Messages [c0, c1) of part `w` (commit indices gbase + i): gathered into page-locked staging (or uploaded in place
// when the part's payloads are page-locked and contiguous), then classify and both parses of the chunk.
void wave_chunk(jg_node* nd, WaveRun& r, const jg_commit* w, uint64_t gbase, uint64_t c0, uint64_t c1, bool direct) {
    jg_ctx* ctx = nd->ctx;
    jg::WorkerPool& pool = nd->workers();
    const bool filter = r.filter;
    const uint32_t rank = r.rank, world = r.world;
    auto pay = [&](uint64_t i) -> const uint8_t* { return w->off ? w->bytes + w->off[i] : w->ptr[i]; };
    auto plen = [&](uint64_t i) -> uint64_t { return w->off ? w->off[i + 1] - w->off[i] : w->len[i]; };
    auto keep = [&](uint64_t i) { return !filter || shard_of(w->uid[i].lo, w->uid[i].hi, world) == rank; };
    uint8_t* d_bytes = nd->bytes.as<uint8_t>();
    uint64_t* d_off = nd->off.as<uint64_t>();
    std::vector<uint64_t>& tcnt = r.tcnt;
    std::vector<uint64_t>& tbytes = r.tbytes;
    const size_t ntask = (size_t)((c1 - c0 + kTask - 1) / kTask);
    if (tcnt.size() < ntask + 1) tcnt.resize(ntask + 1), tbytes.resize(ntask + 1);
    const bool par = c1 - c0 >= r.min_par;
    const double tg = now_s();
    // pass 1: kept messages and their bytes per task (and, for contiguous payloads, that the offsets
    // never decrease: the wave is rejected before anything of it is applied)
    std::atomic<uint64_t> bad_off{UINT64_MAX};
    jg::deal(pool, par, ntask, [&](size_t q, int) {
        uint64_t k = 0, b = 0;
        const uint64_t e = std::min(c1, c0 + (q + 1) * kTask);
        for (uint64_t i = c0 + q * kTask; i < e; ++i)
            if (keep(i)) ++k, b += plen(i);
        if (w->off)
            for (uint64_t i = c0 + q * kTask; i < e; ++i)
                if (w->off[i + 1] < w->off[i]) {
                    uint64_t cur = bad_off.load();
                    while (i < cur && !bad_off.compare_exchange_weak(cur, i)) {
                    }
                    break;
                }
        tcnt[q + 1] = k;
        tbytes[q + 1] = b;
    });
    JG_REQUIRE(bad_off.load() == UINT64_MAX, JG_EINVAL, "jg_apply: offsets decrease at message %llu", (unsigned long long)(gbase + bad_off.load()));
    // monotone on [0, c1] and within off[n]: every chunk so far fits the buffers sized from off[n]
    JG_REQUIRE(!w->off || w->off[c1] <= w->off[w->n], JG_EINVAL, "jg_apply: offsets decrease after message %llu", (unsigned long long)(gbase + c1 - 1));
    tcnt[0] = tbytes[0] = 0;
    for (size_t q = 0; q < ntask; ++q) tcnt[q + 1] += tcnt[q], tbytes[q + 1] += tbytes[q];
    const uint64_t m = tcnt[ntask], nb = tbytes[ntask];
    if (m == 0) {
        r.t_gather += now_s() - tg;
        return;
    }
    JG_REQUIRE(r.m0 + m <= r.n && r.b0 + nb <= r.total_bytes, JG_EINVAL,
               "jg_apply_stream_append: %llu messages / %llu payload bytes pass the %llu / %llu declared at begin", (unsigned long long)(r.m0 + m),
               (unsigned long long)(r.b0 + nb), (unsigned long long)r.n, (unsigned long long)r.total_bytes);
    const uint64_t meta_bytes = (m + 1) * 8 + m * 25;  // offsets, uids (16), identities (8), types (1)
    JG_REQUIRE(r.mo + meta_bytes <= r.meta_cap, JG_EINVAL, "jg_apply_stream_append: more chunks than the wave was sized for");
    const uint64_t nb_pad = direct ? 0 : (nb + 15) & ~15ull;
    char* buf = nd->stage(nb_pad + (m + 1) * 8 + m * 16 + m * 8 + m + 64);
    auto* soff = reinterpret_cast<uint64_t*>(buf + nb_pad);
    auto* suid = reinterpret_cast<jg_guid*>(soff + m + 1);
    auto* sseq = reinterpret_cast<uint64_t*>(suid + m);
    auto* stype = reinterpret_cast<uint8_t*>(sseq + m);
    soff[0] = 0;
    const uint64_t m0 = r.m0, b0 = r.b0;
    // pass 2: payloads (non-temporal lines), chunk-relative end offsets, uids, identities, types
    jg::deal(pool, par, ntask, [&](size_t q, int) {
        uint64_t j = tcnt[q], o = tbytes[q];
        jg::LineStream out(buf, o);
        const uint64_t e = std::min(c1, c0 + (q + 1) * kTask);
        for (uint64_t i = c0 + q * kTask; i < e; ++i) {
            if (!direct && i + 8 < e) {  // every line of the payload 8 messages ahead
                const uint8_t* pq = pay(i + 8);
                for (uint64_t x = 0, L = plen(i + 8); x < L; x += 64) __builtin_prefetch(pq + x);
            }
            if (!keep(i)) continue;
            const uint64_t L = plen(i);
            if (!direct) out.put(reinterpret_cast<const char*>(pay(i)), L);
            o += L;
            soff[j + 1] = o;
            suid[j] = w->uid[i];
            sseq[j] = w->seq ? w->seq[i] : 0;
            stype[j] = w->type[i];
            if (filter) nd->dmap[m0 + j] = gbase + i;
            ++j;
        }
        if (!direct) out.finish();
    });
    r.t_gather += now_s() - tg;
    // upload (copy stream), then classify and both parses of the chunk (compute stream)
    const uint8_t* src = direct ? w->bytes + w->off[c0] : reinterpret_cast<const uint8_t*>(buf);
    if (nb) JG_HIP(hipMemcpyAsync(d_bytes + b0, src, nb, hipMemcpyHostToDevice, ctx->copy));
    uint8_t* d_meta = nd->meta.as<uint8_t>() + r.mo;
    JG_HIP(hipMemcpyAsync(d_meta, soff, meta_bytes, hipMemcpyHostToDevice, ctx->copy));
    r.mo += (meta_bytes + 63) & ~63ull;
    jg::upload_done(ctx);
    JG_HIP(hipEventRecord(nd->event(2 * r.n_ev), ctx->stream));
    hipLaunchKernelGGL(k_unstage, dim3(blocks_for(m)), dim3(kBlock), 0, ctx->stream, d_meta, m, m0, b0, d_off, nd->uid.as<Guid16>(),
                       nd->seq.as<uint64_t>(), nd->type.as<uint8_t>());
    hipLaunchKernelGGL(k_classify, dim3(blocks_for(m)), dim3(kBlock), 0, ctx->stream, nd->uid.as<Guid16>(), nd->type.as<uint8_t>(),
                       nd->seq.as<unsigned long long>(), m0, m0 + m, r.du, r.dt, nd->rows.as<uint32_t>(), nd->mset.as<uint32_t>(),
                       nd->tslot.as<uint32_t>(), nd->status.as<unsigned long long>());
    JG_HIP(hipGetLastError());
    if (r.do_pnc) jg::pnc_node_scan(nd->pnc, d_bytes, d_off, nd->rows.as<uint32_t>(), m0, m0 + m);
    if (r.do_orset) jg::orset_node_parse(nd->orset, m0, m0 + m);
    JG_HIP(hipEventRecord(nd->event(2 * r.n_ev + 1), ctx->stream));
    ++r.n_ev;
    r.m0 += m;
    r.b0 += nb;
    ++nd->stats.chunks;
}

// Part `w` (commit indices gbase..) in chunks: ~48 MB of payload each, a small first chunk (the first upload starts
// after ~0.1 ms of gathering instead of a full chunk's) and, on the wave's end (`last`), its last `tail` messages
// a chunk of their own (the part no host work overlaps).
void wave_part(jg_node* nd, WaveRun& r, const jg_commit* w, uint64_t gbase, bool last) {
    const uint64_t n = w->n;
    if (n == 0) return;
    JG_REQUIRE(w->uid && w->type && (w->off ? w->bytes != nullptr || w->off[n] == 0 : (w->ptr && w->len)), JG_EINVAL, "jg_apply: NULL array in the wave");
    if (w->off) JG_REQUIRE(w->off[0] == 0, JG_EINVAL, "jg_apply: off[0] must be 0");  // monotonicity: checked by the chunks' first pass
    const bool direct = w->off && !r.filter && host_pinned(w->bytes);  // payload uploaded from the caller's pinned buffer
    std::vector<uint64_t> cb{0};
    const uint64_t first = gbase == 0 && n > 4 * r.tail ? r.tail : r.chunk_msgs;
    // (measured, round 5: planning the last chunks from the end — a `tail` chunk after a 2 x `tail` one, so each
    // chunk's kernels hide under the next upload — moved neither the OR-Set nor the C5 wave, interleaved A/B)
    for (uint64_t c0 = first; c0 < n; c0 += r.chunk_msgs) cb.push_back(c0);
    if (last && n > cb.back() + 2 * r.tail) cb.push_back(n - r.tail);
    cb.push_back(n);
    for (size_t c = 0; c + 1 < cb.size(); ++c) wave_chunk(nd, r, w, gbase, cb[c], cb[c + 1], direct);
}

// The final phase: the cut (the first state the reference's loop would throw at), both commits, the safe-update
// completions of the messages before the cut in commit order, the figures.
void wave_end(jg_node* nd, WaveRun& r, uint64_t* completed, uint64_t* n_completed, uint64_t* stopped_at) {
    jg_ctx* ctx = nd->ctx;
    jg_tracker* tr = r.tr;
    const DevTrack dt = r.dt;
    const bool do_pnc = r.do_pnc, do_orset = r.do_orset, filter = r.filter, trace = r.trace;
    uint8_t* d_bytes = nd->bytes.as<uint8_t>();
    uint64_t* d_off = nd->off.as<uint64_t>();
    uint32_t* d_rows = nd->rows.as<uint32_t>();
    uint32_t* d_mset = nd->mset.as<uint32_t>();
    unsigned long long* d_status = nd->status.as<unsigned long long>();
    const uint64_t nn = r.m0;  // messages on the device
    const uint64_t b0 = r.b0;
    const size_t n_ev = r.n_ev;
    hipEvent_t* up_ev = r.up_ev;
    if (trace) JG_HIP(hipEventRecord(up_ev[1], ctx->copy));
    nd->stats.gather_s = r.t_gather;
    nd->stats.msgs_uploaded = nn;
    nd->stats.bytes_uploaded = b0;
    if (nn) nd->avg_msg_bytes = (double)b0 / (double)nn;
    const double t_dev = now_s();
    nd->stats.loop_s = t_dev - r.t_loop;
    r.active = false;
    r.held = true;
    struct Release {  // every way out of wave_end lets the stores go (wave_abort on the failure paths does too)
        jg_node* nd;
        WaveRun& r;
        ~Release() {
            if (r.held) hold(nd, r.tr, false), r.held = false;
        }
    } release_{nd, r};

    // the cut: the first state the reference's loop would throw at
    JG_HIP(hipEventRecord(nd->event(2 * n_ev), ctx->stream));  // the final phase's kernels start after the chunks'
    double te[6] = {now_s()};
    uint64_t cut = nn;
    int code = JG_OK;
    std::string why;
    try {
        if (r.block_mode) {
            unsigned long long unk;
            JG_HIP(hipMemcpyAsync(&unk, d_status, 8, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            if (unk < nn) {
                cut = unk;
                code = JG_EINVAL;
                why = "The given key was not present in the dictionary (a CRDT state of an uid the node does not hold)";
            }
        }
        if (do_orset) {
            uint64_t bad = UINT64_MAX;
            std::string w2;
            const int rc = jg::orset_node_check(nd->orset, nn, b0, &bad, &w2);  // over the messages uploaded
            te[1] = now_s();
            if (rc != JG_OK) {
                if (bad == UINT64_MAX) jg::fail(rc, "%s", w2.c_str());
                if (bad < cut) cut = bad, code = rc, why = w2;
            }
        }
        if (do_pnc) {
            uint64_t bad = UINT64_MAX;
            std::string w3;
            int rc = cut < nn ? jg::pnc_node_prefix(nd->pnc, d_bytes, d_off, d_rows, cut, &bad, &w3)
                              : jg::pnc_node_finish(nd->pnc, d_bytes, d_off, d_rows, nn, &bad, &w3);
            if (rc != JG_OK) {
                cut = bad, code = rc, why = w3;
                rc = jg::pnc_node_prefix(nd->pnc, d_bytes, d_off, d_rows, cut, &bad, &w3);
                if (rc != JG_OK) jg::fail(JG_EHIP, "jg_apply: the prefix before message %llu failed again: %s", (unsigned long long)cut, w3.c_str());
            }
        }
        te[2] = now_s();
        if (do_orset) jg::orset_node_commit(nd->orset, cut);
        if (do_orset && nd->orset->counts_pending && test_commit_fail())  // tests: the commit's union reports a broken precondition
            JG_HIP(hipMemsetAsync(ctx->flags.p, 0x04, 1, ctx->stream));
        te[3] = now_s();
    } catch (...) {
        // an internal failure past the chunk loop (a check that could not name a message, a prefix that failed
        // again, a device error): the classified chunks' first-occurrence claims are released as in the loop's
        // catch, or a stale claim below the next wave's index would keep that safe update from completing
        // (ADVICE r03).  The OR-Set commit's one data-dependent failure (a set's element ids running out) is
        // ruled out by orset_node_check before the PN-Counter commit, so what is left here is a device error.
        wave_abort(nd, r, nn);
        throw;
    }

    // safe-update completions of the messages before the cut, in commit order
    uint64_t ndone = 0;
    int late_code = JG_OK;  // the OR-Set commit's deferred error flag, raised once the completions are out
    std::string late_why;
    bool orset_pending = false;  // the OR-Set commit's union counts ride on this phase's page-locked read
    JG_HIP(hipMemsetAsync(d_status + 2, 0, 8, ctx->stream));
    if (cut) hipLaunchKernelGGL(k_count_applied, dim3((unsigned)std::min<uint64_t>(1024, blocks_for(cut))), dim3(kBlock), 0, ctx->stream, d_rows, d_mset, cut,
                                d_status + 2);
    JG_HIP(hipGetLastError());
    if (dt.tab && cut > 0) {
        ensure(nd->origin, nn * 8 + 8);
        ensure(nd->done, nn * 8 + 8);
        auto* d_origin = nd->origin.as<unsigned long long>();
        auto* d_done = nd->done.as<unsigned long long>();
        hipLaunchKernelGGL(k_complete, dim3(blocks_for(cut)), dim3(kBlock), 0, ctx->stream, nd->tslot.as<uint32_t>(), cut, dt, d_origin);
        hipLaunchKernelGGL(k_claim_reset, dim3(blocks_for(nn)), dim3(kBlock), 0, ctx->stream, nd->tslot.as<uint32_t>(), nn, dt.claim);
        JG_HIP(hipGetLastError());
        size_t temp = 0;
        JG_HIP(hipcub::DeviceSelect::If(nullptr, temp, d_origin, d_done, d_status + 1, (int)cut, NonZero(), ctx->stream));
        ensure(nd->cub, temp + 256);
        JG_HIP(hipcub::DeviceSelect::If(nd->cub.p, temp, d_origin, d_done, d_status + 1, (int)cut, NonZero(), ctx->stream));
        hipLaunchKernelGGL(k_count_sub, dim3(1), dim3(1), 0, ctx->stream, tr->count.as<unsigned long long>(), d_status + 1);
        JG_HIP(hipGetLastError());
        unsigned long long k = 0;
        jg::pin_get(ctx, 0, d_status + 1, 16);  // the completions' count and the applied count
        orset_pending = do_orset && jg::orset_pin_pending(nd->orset, 64);  // and the OR-Set commit's union counts
        jg::pin_sync(ctx);
        if (orset_pending) {
            // k_complete / k_count_sub have already taken these completions off the tracker: a union failure is
            // reported AFTER they reach the caller, or they would be lost for good
            try {
                jg::orset_settle_pending(nd->orset, 64);
            } catch (const jg::Error& e) {
                late_code = e.code;
                late_why = e.msg;
            }
            orset_pending = false;
        }
        std::memcpy(&k, jg::pin_at(ctx, 0), 8);
        ndone = k;
        if (completed && k) {
            JG_HIP(hipMemcpyAsync(completed, d_done, k * 8, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
        }
    } else {
        if (dt.tab && nn) {
            hipLaunchKernelGGL(k_claim_reset, dim3(blocks_for(nn)), dim3(kBlock), 0, ctx->stream, nd->tslot.as<uint32_t>(), nn, dt.claim);
            JG_HIP(hipGetLastError());
        }
        jg::pin_get(ctx, 8, d_status + 2, 8);  // the applied count with the final sync
        orset_pending = do_orset && jg::orset_pin_pending(nd->orset, 64);  // and the OR-Set commit's union counts
        jg::pin_sync(ctx);
    }
    JG_HIP(hipEventRecord(nd->event(2 * n_ev + 1), ctx->stream));
    unsigned long long applied = 0;
    JG_HIP(hipEventSynchronize(nd->event(2 * n_ev + 1)));
    std::memcpy(&applied, jg::pin_at(ctx, 8), 8);
    if (orset_pending) jg::orset_settle_pending(nd->orset, 64);
    nd->stats.msgs_applied = applied;
    te[4] = now_s();
    if (trace) {
        if (!do_orset) te[1] = te[0];
        std::fprintf(stderr, "apply tail: orset check %.0f us, pnc finish %.0f, orset commit %.0f, completions %.0f (after the loop's last upload: %.0f us host)\n",
                     (te[1] - te[0]) * 1e6, (te[2] - te[1]) * 1e6, (te[3] - te[2]) * 1e6, (te[4] - te[3]) * 1e6, (te[4] - te[0]) * 1e6);
        // device clock: the copy queue from its first upload to the last one's end, and from there to the end of
        // the wave's last kernel (the final phase's event pair)
        float up_ms = 0, after_ms = 0, first_ms = 0;
        JG_HIP(hipEventElapsedTime(&up_ms, up_ev[0], up_ev[1]));
        JG_HIP(hipEventElapsedTime(&after_ms, up_ev[1], nd->ev[2 * n_ev + 1]));
        JG_HIP(hipEventElapsedTime(&first_ms, up_ev[0], nd->ev[0]));
        std::fprintf(stderr, "apply device: uploads %.0f us (%llu chunks, %.1f GB/s of payload over the span), first chunk's kernels at +%.0f us, "
                     "last kernel %.0f us after the last upload\n",
                     up_ms * 1e3, (unsigned long long)nd->stats.chunks, up_ms > 0 ? b0 / (up_ms * 1e-3) / 1e9 : 0.0, first_ms * 1e3, after_ms * 1e3);
        for (hipEvent_t& e : r.up_ev) (void)hipEventDestroy(e), e = nullptr;
    }
    double busy = 0;
    for (size_t k = 0; k <= n_ev; ++k) {
        float ms = 0;
        JG_HIP(hipEventElapsedTime(&ms, nd->ev[2 * k], nd->ev[2 * k + 1]));
        busy += ms * 1e-3;
        if (k == n_ev) nd->stats.tail_busy_s = ms * 1e-3;  // the final phase's pair
    }
    nd->stats.device_busy_s = busy;
    nd->stats.chunk_busy_s = busy - nd->stats.tail_busy_s;
    if (do_orset) jg::orset_free_retired(nd->orset);  // the wave has drained: blocks its growth retired go now
    if (n_completed) *n_completed = ndone;
    *stopped_at = cut < nn ? (filter ? nd->dmap[cut] : cut) : UINT64_MAX;
    const double t_end = now_s();
    nd->stats.device_wait_s = t_end - t_dev;
    nd->stats.total_s = t_end - r.t_begin;
    if (late_code != JG_OK) jg::fail(late_code, "%s (the wave's OR-Set commit; its safe-update completions were reported)", late_why.c_str());
    if (code != JG_OK) jg::fail(code, "%s (commit index %llu)", why.c_str(), (unsigned long long)*stopped_at);
}

// The apply loop over one wave in one call (jg_apply_committed / jg_apply_block).
void apply_wave(jg_node* nd, jg_tracker* tr, const jg_commit* w, bool block_mode, uint64_t* completed, uint64_t* n_completed, uint64_t* stopped_at) {
    const uint64_t n = w->n;
    JG_REQUIRE(n < 0x7FFFFFF0ull, JG_EINVAL, "jg_apply: at most 2^31 - 16 messages per wave");
    JG_REQUIRE(n == 0 || (w->uid && w->type && (w->off ? w->bytes != nullptr || w->off[n] == 0 : (w->ptr && w->len))), JG_EINVAL,
               "jg_apply: NULL array in the wave");
    if (w->off) JG_REQUIRE(w->off[0] == 0, JG_EINVAL, "jg_apply: off[0] must be 0");
    WaveRun& r = nd->run;
    JG_REQUIRE(!r.active, JG_EINVAL, "jg_apply: a streamed wave is open on this node (jg_apply_stream_end first)");
    if (n == 0) {  // the uid table, names and tracker adds still go to the device (the next wave finds them there)
        double tp[8];
        wave_prologue(nd, tr, tp);
        *stopped_at = UINT64_MAX;
        return;
    }
    // capacity for the whole wave (payload bytes: an upper bound when the shard shortcut drops states)
    uint64_t total_bytes = 0;
    if (w->off) {
        total_bytes = w->off[n];
    } else {
        jg::WorkerPool& pool = nd->workers();
        const uint64_t per = std::max<uint64_t>(65536, (n + 63) / 64);  // few large tasks: this pass only sums lengths
        const size_t ntask = (size_t)((n + per - 1) / per);
        std::vector<uint64_t> part(ntask);
        jg::deal(pool, n >= 8192, ntask, [&](size_t q, int) {
            uint64_t b = 0;
            for (uint64_t i = q * per, e = std::min<uint64_t>(n, (q + 1) * per); i < e; ++i) b += w->len[i];
            part[q] = b;
        });
        for (uint64_t b : part) total_bytes += b;
    }
    const bool filter = !block_mode && nd->shortcut();
    const size_t chunk_guess = std::clamp<size_t>((size_t)((48u << 20) / std::max(nd->avg_msg_bytes, 64.0)), 8192, 131072);
    const char* ce = std::getenv("JANUS_WAVE_CHUNK");
    const size_t cm = ce ? std::max<size_t>(1, std::strtoull(ce, nullptr, 10)) : chunk_guess;
    wave_begin(nd, r, tr, n, total_bytes, n / cm + 4, block_mode, filter);
    try {
        wave_part(nd, r, w, 0, true);
    } catch (...) {
        wave_abort(nd, r, r.m0);
        throw;
    }
    wave_end(nd, r, completed, n_completed, stopped_at);
}
}  // namespace

extern "C" {

int jg_node_create(jg_pnc* pnc, jg_orset* orset, jg_node** out) {
    return jg::guard([&] {
        JG_REQUIRE(out && (pnc || orset), JG_EINVAL, "jg_node_create: NULL argument (one store at least)");
        JG_REQUIRE(!pnc || !orset || pnc->ctx == orset->ctx, JG_EINVAL, "jg_node_create: the stores belong to different contexts");
        jg_ctx* ctx = pnc ? pnc->ctx : orset->ctx;
        auto lk_ = jg::lock(ctx);
        jg::ensure_device(ctx);
        auto* nd = new jg_node();
        nd->ctx = ctx;
        nd->pnc = pnc;
        nd->orset = orset;
        *out = nd;
    });
}

int jg_node_destroy(jg_node* nd) {
    return jg::guard([&] {
        if (!nd) return;
        auto lk_ = jg::lock(nd->ctx);
        jg::ensure_device(nd->ctx);
        if (nd->run.active) wave_abort(nd, nd->run, nd->run.m0);  // an open streamed wave: undone, its stores let go
        JG_HIP(hipStreamSynchronize(nd->ctx->stream));
        JG_HIP(hipStreamSynchronize(nd->ctx->copy));
        delete nd;
    });
}

int jg_node_register(jg_node* nd, uint64_t n, const jg_guid* uid, const uint8_t* type, const uint32_t* idx) {
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd, JG_EINVAL, "jg_node_register: node is NULL");
        if (n == 0) return;
        JG_REQUIRE(uid && type && idx, JG_EINVAL, "jg_node_register: NULL argument");
        std::unordered_set<uint64_t> batch;  // repeats inside the call (hash of the uid; exact check below)
        for (uint64_t i = 0; i < n; ++i) {
            JG_REQUIRE((uid[i].lo | uid[i].hi) != 0, JG_EINVAL, "jg_node_register: entry %llu is Guid.Empty (the key space itself)", (unsigned long long)i);
            JG_REQUIRE(type[i] <= 1, JG_EINVAL, "jg_node_register: entry %llu: type %u (0 PNCounter, 1 ORSet)", (unsigned long long)i, type[i]);
            if (type[i] == 0) {
                JG_REQUIRE(nd->pnc, JG_EINVAL, "jg_node_register: entry %llu is a PNCounter but the node has no PN-Counter store", (unsigned long long)i);
                JG_REQUIRE(idx[i] < nd->pnc->n_keys, JG_EINVAL, "jg_node_register: entry %llu: row %u >= n_keys %llu", (unsigned long long)i, idx[i],
                           (unsigned long long)nd->pnc->n_keys);
            } else {
                JG_REQUIRE(nd->orset, JG_EINVAL, "jg_node_register: entry %llu is an ORSet but the node has no OR-Set store", (unsigned long long)i);
                JG_REQUIRE(idx[i] < 0x7FFFFFF0u, JG_EINVAL, "jg_node_register: entry %llu: set id %u out of range", (unsigned long long)i, idx[i]);
            }
            JG_REQUIRE(!nd->find(uid[i].lo, uid[i].hi), JG_EINVAL, "jg_node_register: entry %llu: uid already registered", (unsigned long long)i);
            if (!batch.insert(uid_hash(uid[i].lo, uid[i].hi)).second)
                for (uint64_t j = 0; j < i; ++j)
                    JG_REQUIRE(!(uid[j].lo == uid[i].lo && uid[j].hi == uid[i].hi), JG_EINVAL, "jg_node_register: entry %llu repeats entry %llu",
                               (unsigned long long)i, (unsigned long long)j);
        }
        nd->grow(nd->n_keys + n);
        for (uint64_t i = 0; i < n; ++i) {
            nd->insert(UidSlot{uid[i].lo, uid[i].hi, type[i] ? (idx[i] | kOrSetBit) : idx[i], 0, 0});
            if (type[i]) ++nd->n_orset, nd->max_set = std::max(nd->max_set, idx[i]);
            else ++nd->n_pnc;
            if (nd->shard_world > 1 && shard_of(uid[i].lo, uid[i].hi, nd->shard_world) != nd->shard_rank) nd->foreign = true;
        }
        nd->n_keys += n;
    });
}

int jg_node_set_shard(jg_node* nd, uint32_t rank, uint32_t world) {
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd && world >= 1 && rank < world, JG_EINVAL, "jg_node_set_shard: need rank < world");
        nd->shard_rank = rank;
        nd->shard_world = world;
        nd->foreign = false;
        if (world > 1)
            for (const UidSlot& s : nd->htab)
                if ((s.lo | s.hi) != 0 && shard_of(s.lo, s.hi, world) != rank) {
                    nd->foreign = true;  // a registered key of another shard: the table decides again
                    break;
                }
    });
}

int jg_shard_of(const jg_guid* uid, uint32_t world, uint32_t* rank) {
    return jg::guard([&] {
        JG_REQUIRE(uid && rank && world >= 1, JG_EINVAL, "jg_shard_of: bad argument");
        *rank = shard_of(uid->lo, uid->hi, world);
    });
}

int jg_global_key(const jg_guid* uid, uint32_t world, uint32_t local, uint32_t* global) {
    return jg::guard([&] {
        JG_REQUIRE(uid && global && world >= 1, JG_EINVAL, "jg_global_key: bad argument");
        const uint64_t g = (uint64_t)local * world + jg::shard_of_uid(uid->lo, uid->hi, world);
        JG_REQUIRE(g < 0xFFFFFFF0ull, JG_EINVAL, "jg_global_key: local key %u x world %u leaves the 32-bit key space", local, world);
        *global = (uint32_t)g;
    });
}

int jg_node_last_stats(jg_node* nd, jg_apply_stats* out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd && out, JG_EINVAL, "jg_node_last_stats: NULL argument");
        *out = nd->stats;
    });
}

int jg_tracker_create(jg_ctx* ctx, jg_tracker** out) {
    return jg::guard([&] {
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_tracker_create: NULL argument");
        auto lk_ = jg::lock(ctx);
        jg::ensure_device(ctx);
        auto* t = new jg_tracker();
        t->ctx = ctx;
        *out = t;
    });
}

int jg_tracker_destroy(jg_tracker* t) {
    return jg::guard([&] {
        if (!t) return;
        auto lk_ = jg::lock(t->ctx);
        JG_REQUIRE(t->waves == 0, JG_EINVAL, "jg_tracker_destroy: a node wave (jg_apply_stream_begin .. _end) is using the tracker");
        jg::ensure_device(t->ctx);
        JG_HIP(hipStreamSynchronize(t->ctx->stream));
        delete t;
    });
}

int jg_tracker_add(jg_tracker* t, uint64_t n, const uint64_t* seq, const uint64_t* origin) {
    return jg::guard([&] {
        JG_REQUIRE(t, JG_EINVAL, "jg_tracker_add: tracker is NULL");
        if (n == 0) return;
        JG_REQUIRE(seq && origin, JG_EINVAL, "jg_tracker_add: NULL argument");
        for (uint64_t i = 0; i < n; ++i) {
            JG_REQUIRE(seq[i] != 0 && seq[i] != kTomb, JG_EINVAL, "jg_tracker_add: identity %llu is reserved", (unsigned long long)seq[i]);
            JG_REQUIRE(origin[i] != 0, JG_EINVAL, "jg_tracker_add: origin 0 is the default connection (never tracked, SafeCRDT.cs:55)");
        }
        std::lock_guard<std::mutex> g(t->pend_mu);
        t->append(n, seq, origin);
    });
}

int jg_tracker_size(jg_tracker* t, uint64_t* n) {
    return jg::guard([&] {
        JG_REQUIRE(t && n, JG_EINVAL, "jg_tracker_size: NULL argument");
        auto lk_ = jg::lock(t->ctx);
        jg::ensure_device(t->ctx);
        t->flush();
        unsigned long long c = 0;
        JG_HIP(hipMemcpyAsync(&c, t->count.p, 8, hipMemcpyDeviceToHost, t->ctx->stream));
        JG_HIP(hipStreamSynchronize(t->ctx->stream));
        *n = c;
    });
}

int jg_tracker_contains(jg_tracker* t, uint64_t n, const uint64_t* seq, uint8_t* out) {
    return jg::guard([&] {
        JG_REQUIRE(t, JG_EINVAL, "jg_tracker_contains: tracker is NULL");
        if (n == 0) return;
        JG_REQUIRE(seq && out, JG_EINVAL, "jg_tracker_contains: NULL argument");
        auto lk_ = jg::lock(t->ctx);
        jg_ctx* ctx = t->ctx;
        jg::ensure_device(ctx);
        t->flush();
        char* st = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * 9 + 512));
        auto* ds = reinterpret_cast<unsigned long long*>(st);
        auto* dout = reinterpret_cast<uint8_t*>(st + ((n * 8 + 255) & ~255ull));
        JG_HIP(hipMemcpyAsync(ds, seq, n * 8, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_track_lookup, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, t->dev(), ds, n, dout);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(out, dout, n, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_apply_committed(jg_node* nd, jg_tracker* tr, const jg_commit* wave, uint64_t* completed, uint64_t* n_completed, uint64_t* stopped_at) {
    uint64_t dummy = 0;
    if (!stopped_at) stopped_at = &dummy;
    *stopped_at = UINT64_MAX;
    if (n_completed) *n_completed = 0;
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd && wave, JG_EINVAL, "jg_apply_committed: NULL argument");
        JG_REQUIRE(!tr || tr->ctx == nd->ctx, JG_EINVAL, "jg_apply_committed: the tracker belongs to another context");
        jg::ensure_device(nd->ctx);
        apply_wave(nd, tr, wave, false, completed, n_completed, stopped_at);
    });
}

int jg_apply_stream_begin(jg_node* nd, jg_tracker* tr, uint64_t n_max, uint64_t bytes_max) {
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd, JG_EINVAL, "jg_apply_stream_begin: NULL node");
        JG_REQUIRE(!tr || tr->ctx == nd->ctx, JG_EINVAL, "jg_apply_stream_begin: the tracker belongs to another context");
        JG_REQUIRE(!nd->run.active, JG_EINVAL, "jg_apply_stream_begin: a streamed wave is already open on this node");
        JG_REQUIRE(n_max > 0 && n_max < 0x7FFFFFF0ull, JG_EINVAL, "jg_apply_stream_begin: 1 .. 2^31 - 16 messages per wave");
        jg::ensure_device(nd->ctx);
        // every part may make a chunk of its own: the meta area is sized for one chunk per message at most
        wave_begin(nd, nd->run, tr, n_max, bytes_max, n_max + 1, false, false);
    });
}

int jg_apply_stream_append(jg_node* nd, const jg_commit* part) {
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd && part, JG_EINVAL, "jg_apply_stream_append: NULL argument");
        WaveRun& r = nd->run;
        JG_REQUIRE(r.active, JG_EINVAL, "jg_apply_stream_append: no streamed wave open (jg_apply_stream_begin)");
        jg::ensure_device(nd->ctx);
        try {
            wave_part(nd, r, part, r.seen, false);
            r.seen += part->n;
        } catch (...) {  // the wave is rejected as a whole, nothing of it applied (the one-call path's rule)
            wave_abort(nd, r, r.m0);
            throw;
        }
    });
}

int jg_apply_stream_end(jg_node* nd, uint64_t* completed, uint64_t* n_completed, uint64_t* stopped_at) {
    uint64_t dummy = 0;
    if (!stopped_at) stopped_at = &dummy;
    *stopped_at = UINT64_MAX;
    if (n_completed) *n_completed = 0;
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd, JG_EINVAL, "jg_apply_stream_end: NULL node");
        JG_REQUIRE(nd->run.active, JG_EINVAL, "jg_apply_stream_end: no streamed wave open (jg_apply_stream_begin)");
        jg::ensure_device(nd->ctx);
        wave_end(nd, nd->run, completed, n_completed, stopped_at);
    });
}

int jg_apply_block(jg_node* nd, const jg_commit* wave, uint64_t* stopped_at) {
    uint64_t dummy = 0;
    if (!stopped_at) stopped_at = &dummy;
    *stopped_at = UINT64_MAX;
    return jg::guard([&] {
        auto lk_ = jg::lock(nd);
        JG_REQUIRE(nd && wave, JG_EINVAL, "jg_apply_block: NULL argument");
        jg::ensure_device(nd->ctx);
        apply_wave(nd, nullptr, wave, true, nullptr, nullptr, stopped_at);
    });
}

}  // extern "C"
