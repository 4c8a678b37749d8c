// janus_host.cpp — see janus_host.hpp.
#include "janus_host.hpp"

#include <emmintrin.h>
#include <sys/mman.h>

#include <cstdio>
#include <cstring>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <limits>
#include <memory>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "wire.hpp"

namespace janus {

namespace {
std::string last_error() {
    char buf[1024];
    jg_last_error(buf, sizeof buf);
    return buf;
}
}  // namespace

void GpuStableStore::check(int rc) const {
    if (rc != JG_OK) throw EngineError(rc, last_error());
}

GpuStableStore::GpuStableStore(int device, uint32_t max_keys, uint32_t replicas, uint32_t elem_bytes)
    : max_keys_(max_keys), R_(replicas), eb_(elem_bytes) {
    check(jg_open(device, &ctx_));
    check(jg_pnc_create(ctx_, max_keys, replicas, elem_bytes, &pnc_));
    check(jg_orset_create(ctx_, 0, 0, &orset_));
}

GpuStableStore::~GpuStableStore() {
    for (auto& a : arenas_) jg_host_free(a.first);
    if (orset_) jg_orset_destroy(orset_);
    if (pnc_) jg_pnc_destroy(pnc_);
    if (ctx_) jg_close(ctx_);
}


const GpuStableStore::KeyRef* GpuStableStore::UidTable::find(const Guid& g) const {
    if (slots_.empty()) return nullptr;
    const size_t mask = slots_.size() - 1;
    for (size_t i = GuidHash()(g) & mask;; i = (i + 1) & mask) {
        const Slot& s = slots_[i];
        if (!s.used) return nullptr;
        if (s.key == g) return &s.val;
    }
}

bool GpuStableStore::UidTable::insert(const Guid& g, KeyRef v) {
    if ((n_ + 1) * 2 > slots_.size()) grow();
    const size_t mask = slots_.size() - 1;
    for (size_t i = GuidHash()(g) & mask;; i = (i + 1) & mask) {
        Slot& s = slots_[i];
        if (!s.used) { s.used = 1; s.key = g; s.val = v; ++n_; return true; }
        if (s.key == g) return false;
    }
}

void GpuStableStore::UidTable::grow() {
    std::vector<Slot, TableAlloc<Slot>> old = std::move(slots_);
    slots_.assign(old.empty() ? 1024 : old.size() * 2, Slot{});
    n_ = 0;
    for (const Slot& s : old)
        if (s.used) insert(s.key, s.val);
}

const GpuStableStore::KeyRef& GpuStableStore::ref(const Guid& uid, CrdtType want) const {
    const KeyRef* r = uids_.find(uid);
    if (!r) throw EngineError(JG_EINVAL, "unknown CRDT uid");
    if (r->type != want) throw EngineError(JG_ETYPE, "CRDT uid is of the other type");
    return *r;
}

uint32_t GpuStableStore::elem_id(uint32_t set, const std::optional<std::string>& e, bool create) {
    if (!e) return JG_NULL_ELEM;
    materialize_names();
    SetKey& s = sets_[set];
    for (; s.indexed < s.names.size(); ++s.indexed) s.elems.emplace(s.names[s.indexed], s.indexed);  // ids a wave issued
    auto it = s.elems.find(*e);
    if (it != s.elems.end()) return it->second;
    if (!create) return JG_NULL_ELEM - 1;  // never allocated: no records carry it
    // ids only grow (also across Clear), so ascending id = insertion order into the add Dictionary
    const uint32_t id = (uint32_t)s.names.size();
    if (id >= JG_NULL_ELEM - 1) throw EngineError(JG_ESTATE, "too many elements in one OR-Set");
    s.elems.emplace(*e, id);
    s.names.push_back(*e);
    s.indexed = (uint32_t)s.names.size();
    pending_names_[set].ids.push_back(id);
    return id;
}

void GpuStableStore::CreateSafeCRDT(const Guid& uid, CrdtType type, const Guid& stableReplicaGuid) {
    if (uids_.find(uid)) return;
    if (shard_world_ > 1 && ShardOf(uid, shard_world_) != shard_rank_) foreign_keys_ = true;
    if (type == CrdtType::PNCounter) {
        if (next_row_ >= max_keys_) throw EngineError(JG_ESTATE, "PNCounter store full");
        const uint32_t row = next_row_++;
        reg_rows_.push_back(row);  // {self: 0} — the row is zero already; column 0 once flushed
        reg_guids_.push_back(jg_guid{stableReplicaGuid.lo, stableReplicaGuid.hi});
        uids_.insert(uid, KeyRef{type, row});
    } else {
        uids_.insert(uid, KeyRef{type, next_set_++});
        sets_.emplace_back();
    }
}

void GpuStableStore::flush_registrations() {
    if (reg_rows_.empty()) return;
    std::vector<uint32_t> cols(reg_rows_.size());
    check(jg_pnc_intern(pnc_, reg_rows_.size(), reg_rows_.data(), reg_guids_.data(), cols.data()));
    reg_rows_.clear();
    reg_guids_.clear();
}


namespace {
double wall_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

// Persistent host workers (thread creation per phase cost ~0.3 ms per phase; a wave runs ~20).
class WorkerPool {
  public:
    explicit WorkerPool(int n) : n_(n) {
        for (int t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    // fn(t) for every worker t in [0, n); t = 0 runs on the caller.  Returns when all are done.
    void run(const std::function<void(int)>& fn) {
        if (n_ == 1) { fn(0); return; }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                job = job_;
            }
            (*job)(t);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

namespace {
// One worker's contiguous output range in a pinned staging buffer, written with non-temporal stores in
// whole 64-B lines: the staging is read once by the H2D copy engine, so a line written through the cache
// costs a read for ownership first.  Bytes are collected into `line` until it is full; a payload part
// that starts on an empty, aligned line streams straight from the source.  The range's first and last
// partial lines (shared with the neighbouring workers' ranges) are written with ordinary stores.
class LineStream {
  public:
    LineStream(char* base, size_t pos) : base_(base), pos_(pos) {}
    void put(const char* src, size_t n) {
        if (head_) {  // up to the range's first line boundary: ordinary stores
            const size_t c = std::min(n, (64 - (pos_ & 63)) & 63);
            std::memcpy(base_ + pos_, src, c);
            pos_ += c, src += c, n -= c;
            if ((pos_ & 63) == 0) head_ = false;
            if (head_ || n == 0) return;
        }
        if (fill_) {
            const size_t c = std::min(n, 64 - fill_);
            std::memcpy(line_ + fill_, src, c);
            fill_ += c, pos_ += c, src += c, n -= c;
            if (fill_ < 64) return;
            stream(base_ + pos_ - 64, line_);
            fill_ = 0;
        }
        for (; n >= 64; pos_ += 64, src += 64, n -= 64) stream(base_ + pos_, src);
        std::memcpy(line_, src, n);
        fill_ = n, pos_ += n;
    }
    void finish() {  // the range's last partial line, then order the streamed lines before the join
        if (fill_) std::memcpy(base_ + pos_ - fill_, line_, fill_);
        _mm_sfence();
    }

  private:
    static void stream(char* dst, const char* src) {
        for (int k = 0; k < 4; ++k)
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst) + k, _mm_loadu_si128(reinterpret_cast<const __m128i*>(src) + k));
    }
    char* base_;
    size_t pos_;
    bool head_ = true;
    size_t fill_ = 0;
    alignas(64) char line_[64];
};

// Static contiguous split of [0, n) over the pool's workers: fn(begin, end, worker).  Worker t's
// range precedes worker t+1's, so per-worker results concatenated in worker order keep message order.
template <class F> void parallel_ranges(WorkerPool& pool, size_t n, F&& fn) {
    static const size_t min_par = [] {  // below this many messages a phase runs inline
        const char* e = std::getenv("JANUS_HOST_PAR_MIN");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : size_t{8192};
    }();
    const int T = pool.size();
    if (T <= 1 || n < min_par || n < (size_t)T) {
        fn(size_t{0}, n, 0);
        for (int t = 1; t < T; ++t) fn(n, n, t);
        return;
    }
    pool.run([&](int t) { fn(n * t / T, n * (t + 1) / T, t); });
}
}  // namespace

int GpuStableStore::host_threads() {
    if (const char* e = std::getenv("JANUS_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return v;
    }
    unsigned cap = std::thread::hardware_concurrency();
    cap = std::min(cap ? cap : 1u, 16u);
    // A cgroup CPU quota (cgroup v2 cpu.max "quota period", e.g. 16 CPUs of time on a 256-CPU host)
    // throttles every thread of the process once exceeded: at most that many workers (the caller is
    // worker 0; the HIP runtime's threads sleep through a wave).  On the GPU box 16 workers ran the C5
    // wave in 17.6-18.9 ms against 17.7-25.2 ms with 14, alternated, the cgroup never throttling either.
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (std::fscanf(f, "%31s %llu", q, &period) == 2 && std::strcmp(q, "max") != 0 && period) {
            const unsigned long long cpus = std::strtoull(q, nullptr, 10) / period;
            if (cpus >= 1) cap = std::min<unsigned>(cap, (unsigned)cpus);
        }
        std::fclose(f);
    }
    return (int)std::max(1u, cap);
}

WorkerPool& GpuStableStore::pool() {
    if (!pool_ || pool_->size() != host_threads()) pool_ = std::make_unique<WorkerPool>(host_threads());
    return *pool_;
}

void GpuStableStore::flush_names() {
    if (pending_names_.empty()) return;
    materialize_names();
    std::vector<uint32_t> set, next, nset, nid;
    std::vector<uint8_t> cleared, bytes;
    std::vector<uint64_t> off{0};
    for (const auto& kv : pending_names_) {
        const SetKey& sk = sets_[kv.first];
        set.push_back(kv.first);
        next.push_back((uint32_t)sk.names.size());
        cleared.push_back(kv.second.cleared ? 1 : 0);
        for (uint32_t id : kv.second.ids) {
            const std::string& nm = sk.names[id];
            nset.push_back(kv.first);
            nid.push_back(id);
            bytes.insert(bytes.end(), nm.begin(), nm.end());
            off.push_back(bytes.size());
        }
    }
    if (bytes.empty()) bytes.push_back(0);
    check(jg_orset_names_sync(orset_, set.size(), set.data(), next.data(), cleared.data(), nid.size(), nset.data(), nid.data(), off.data(),
                              bytes.data()));
    pending_names_.clear();
}

// The element ids the last wave issued (sorted by set, then id), copied out of the engine; they join the
// host tables in materialize_names.
void GpuStableStore::take_wave_names() {
    uint64_t n = 0, nb = 0;
    check(jg_orset_wave_names(orset_, &n, &nb, nullptr, nullptr, nullptr, nullptr));
    if (n == 0) return;
    WaveNames w;
    w.set.resize(n);
    w.id.resize(n);
    w.off.resize(n + 1);
    w.bytes.resize(std::max<uint64_t>(nb, 1));
    check(jg_orset_wave_names(orset_, &n, &nb, w.set.data(), w.id.data(), w.off.data(), w.bytes.data()));
    wave_names_.push_back(std::move(w));
}

// Pending wave names appended to the SetKey tables, wave after wave, the sets split over the workers in
// contiguous ranges.
void GpuStableStore::materialize_names() {
    if (wave_names_.empty()) return;
    for (const WaveNames& w : wave_names_) {
        const size_t n = w.set.size();
        const std::vector<uint32_t>& set = w.set;
        std::vector<int> bad(pool().size(), 0);
        parallel_ranges(pool(), n, [&](size_t b, size_t e, int t) {
            while (b < n && b > 0 && set[b - 1] == set[b]) ++b;  // that set belongs to the previous worker
            while (e < n && e > 0 && set[e - 1] == set[e]) ++e;
            for (size_t i = b; i < e; ++i) {
                SetKey& sk = sets_[set[i]];
                if (w.id[i] != sk.names.size()) { bad[t] = 1; return; }
                sk.names.emplace_back(reinterpret_cast<const char*>(w.bytes.data()) + w.off[i], w.off[i + 1] - w.off[i]);  // elems: lazily
            }
        });
        for (int x : bad)
            if (x) throw EngineError(JG_ESTATE, "element ids of the engine and the host tables disagree");
    }
    wave_names_.clear();
}

// Pinned staging for wave chunks: arenas carved front to back each wave and kept for the next; a wave
// bigger than all arenas adds one as large as the pool so far (the pool doubles), so a steady stream of
// waves stops allocating pinned memory (hipHostMalloc costs ~0.3 ms per MB) after its first few waves.
char* GpuStableStore::stage(size_t bytes) {
    bytes = (bytes + 255) & ~size_t(255);
    while (arena_i_ < arenas_.size() && arena_off_ + bytes > arenas_[arena_i_].second) {
        ++arena_i_;
        arena_off_ = 0;
    }
    if (arena_i_ == arenas_.size()) {
        size_t total = 0;
        for (const auto& a : arenas_) total += a.second;
        const size_t cap = std::max({bytes, total, size_t(64) << 20});
        void* p = nullptr;
        check(jg_host_alloc(ctx_, cap, &p));
        arenas_.emplace_back(static_cast<char*>(p), cap);
        arena_off_ = 0;
    }
    char* r = arenas_[arena_i_].first + arena_off_;
    arena_off_ += bytes;
    return r;
}


std::vector<uint64_t> GpuStableStore::ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker) {
    const double t0 = wall_s();
    // the wave's messages in commit order: block offsets first, then the blocks filled in parallel into
    // a buffer kept across waves (a fresh 8 MB vector per 1M-message wave cost its page faults)
    blocks_.clear();
    for (const auto& list : updates)
        for (const auto& block : list) blocks_.push_back(&block);
    block_off_.resize(blocks_.size() + 1);
    block_off_[0] = 0;
    for (size_t b = 0; b < blocks_.size(); ++b) block_off_[b + 1] = block_off_[b] + blocks_[b]->update.size();
    std::vector<const NetworkProtocol*>& msgs = msgs_;
    // wave scratch grows with headroom: an exact fit reallocated (and page-faulted in) 8 MB whenever a
    // wave held a few more messages than the largest before it
    if (msgs.capacity() < block_off_.back()) msgs.reserve(block_off_.back() + block_off_.back() / 4);
    msgs.resize(block_off_.back());
    // split by messages, not blocks (a wave is ~1000 blocks of ~1000 messages: split by block count it
    // ran on one thread, 0.8 ms per 1M-message wave)
    parallel_ranges(pool(), msgs.size(), [&](size_t i0, size_t i1, int) {
        if (i0 >= i1) return;
        size_t b = (size_t)(std::upper_bound(block_off_.begin(), block_off_.end(), i0) - block_off_.begin()) - 1;
        for (size_t i = i0; i < i1; ++b) {
            const NetworkProtocol* u = blocks_[b]->update.data() + (i - block_off_[b]);
            for (const size_t e = std::min(i1, block_off_[b + 1]); i < e; ++i) msgs[i] = u++;
        }
    });
    if (std::getenv("JANUS_TRACE_WAVE")) std::fprintf(stderr, "wave: flatten %.2f ms\n", 1e3 * (wall_s() - t0));
    return apply_msgs(msgs, tracker, t0);
}

void GpuStableStore::ReceivedBlock(const std::vector<UpdateMessage>& block) {
    const double t0 = wall_s();
    std::vector<const NetworkProtocol*> msgs;
    for (const auto& um : block)
        for (const auto& u : um.update) msgs.push_back(&u);
    // ReplicationManager.cs:327-330: objectLookupTable[uid] throws KeyNotFoundException for a CRDT
    // message of an unknown object; the states before it were merged (one at a time, RM:333-336).
    size_t cut = msgs.size();
    for (size_t i = 0; i < msgs.size(); ++i) {
        const NetworkProtocol& u = *msgs[i];
        if (u.syncMsgType == NetworkProtocol::CRDTMsg && !u.uid.is_empty() && !uids_.find(u.uid)) { cut = i; break; }
    }
    if (cut == msgs.size()) {
        apply_msgs(msgs, nullptr, t0);
        return;
    }
    msgs.resize(cut);
    apply_msgs(msgs, nullptr, t0);
    throw ApplyError(JG_EINVAL, "The given key was not present in the dictionary. (unknown CRDT uid)", cut, {});
}

std::vector<uint64_t> GpuStableStore::apply_msgs(const std::vector<const NetworkProtocol*>& msgs, SafeUpdateTracker* tracker, double t0) {
    flush_registrations();
    flush_names();
    arena_i_ = arena_off_ = 0;  // the previous wave's staged chunks are no longer referenced
    const size_t n = msgs.size();
    WorkerPool& wp = pool();
    const int T = wp.size();
    phase_s_[0] = wall_s() - t0;
    if (std::getenv("JANUS_TRACE_WAVE")) std::fprintf(stderr, "wave: setup %.2f ms\n", 1e3 * phase_s_[0]);
    constexpr uint32_t kSkip = UINT32_MAX, kSet = UINT32_MAX - 1;
    // Chunks of ~48 MB of payload (sized from the previous wave's bytes per message): the staging
    // buffers stay few and reusable, and the first chunk's upload starts early.
    static const size_t chunk_env = [] {
        const char* e = std::getenv("JANUS_WAVE_CHUNK");
        return e ? std::max<size_t>(1, std::strtoull(e, nullptr, 10)) : size_t{0};
    }();
    const size_t chunk_msgs = chunk_env ? chunk_env : std::clamp<size_t>((size_t)((48u << 20) / std::max(avg_msg_bytes_, 64.0)), 8192, 131072);

    // Both kinds of states are uploaded undecoded and streamed in chunks of commit order: the host
    // workers classify + gather chunk c (per kind, into its pinned buffer) while the engine uploads and
    // runs the validation pass of chunk c-1 (the append calls return once queued).  A chunk's pinned
    // buffer: [payload | pad 16 | off (m+1) u64 | rows or set ids u32]; untouched until commit / abort.
    // cls[i]: PNC row, kSet (sid[i] = the set), or kSkip (create / keyspace / unknown uid, :133-136).
    if (cls_.size() < n) cls_.resize(n + n / 4), sid_.resize(n + n / 4);  // kept across waves, with headroom (no page faults)
    uint32_t* cls = cls_.data();
    uint32_t* sid = sid_.data();
    struct Chunk { size_t m; char* buf; uint64_t* off; uint32_t* rows; uint8_t* bytes; };
    std::vector<Chunk> chunks[2];
    // where_[kind][j]: commit index of the kind's j-th message (wave order); nw[kind] entries
    size_t nw[2] = {0, 0};
    for (auto& w : where_)
        if (w.size() < n) w.resize(n + n / 4);
    // Chunk boundaries: full chunks, then the remainder, whose last `tail` messages form a chunk of their
    // own — the last chunk's upload and pass A are the part of the engine that no host work overlaps.
    const size_t tail = std::max<size_t>(1, std::min<size_t>(16384, chunk_msgs / 8));
    std::vector<size_t> cb{0};
    for (size_t c0 = chunk_msgs; c0 < n; c0 += chunk_msgs) cb.push_back(c0);
    if (n > cb.back() + 2 * tail) cb.push_back(n - tail);
    if (n > 0) cb.push_back(n);
    const size_t n_chunks = cb.size() - 1;
    // Work inside a chunk is dealt in tasks of kTask messages from a shared counter (a static split made
    // every phase wait for the slowest of 16 workers on a shared host); per-task counts keep commit order.
    constexpr size_t kTask = 2048;
    const size_t max_tasks = (chunk_msgs + kTask - 1) / kTask;
    std::vector<size_t> tcnt(2 * max_tasks), tbytes(2 * max_tasks), tmbase(2 * (max_tasks + 1)), tbbase(2 * (max_tasks + 1));
    bool open[2] = {false, false};
    // The safe-update completions (safeUpdateTracker.TryRemove + notify, :141-142) are claimed in the
    // classify pass, which already has each message in cache: (message, origin) per (chunk, task), so
    // concatenating the lists in that order keeps commit order; claims at or past the cut go back.
    const bool sweep = tracker && tracker->size();
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> part(sweep ? n_chunks * max_tasks : 0);
    struct GiveBack {  // any throw before the cut is known: nothing of the wave counts as applied
        const std::vector<std::vector<std::pair<uint64_t, uint64_t>>>& part;
        const NetworkProtocol* const* msgs;
        SafeUpdateTracker* tracker;
        bool armed = true;
        ~GiveBack() {
            if (armed)
                for (const auto& p : part)
                    for (const auto& [i, o] : p) tracker->add(msgs[i]->seq, o);
        }
    } give_back{part, msgs.data(), tracker};
    // Chunk c's engine append runs on the caller (worker 0) at the start of chunk c+1's classify, while
    // the other workers already classify; its error is rethrown once the phase has joined.
    Chunk pend[2] = {};
    size_t pend_m[2] = {0, 0}, pend_nb[2] = {0, 0};
    int append_rc = JG_OK;
    std::string append_why;
    auto append = [&] {
        for (int kind = 0; kind < 2 && append_rc == JG_OK; ++kind) {
            if (pend_m[kind] == 0) continue;
            pend[kind].off[pend_m[kind]] = pend_nb[kind];
            int rc = JG_OK;
            if (!open[kind]) {
                const uint64_t cap_m = std::max<size_t>(pend_m[kind] * n_chunks, 1), cap_b = std::max<size_t>(pend_nb[kind] * n_chunks, 1);
                rc = kind ? jg_orset_wave_begin(orset_, cap_m, cap_b) : jg_pnc_wave_begin(pnc_, cap_m, cap_b);
                if (rc == JG_OK) open[kind] = true;
            }
            if (rc == JG_OK)
                rc = kind ? jg_orset_wave_append(orset_, pend_m[kind], pend[kind].rows, pend[kind].off, pend[kind].bytes)
                          : jg_pnc_wave_append(pnc_, pend_m[kind], pend[kind].rows, pend[kind].off, pend[kind].bytes);
            if (rc != JG_OK) {
                append_rc = rc;
                append_why = last_error();
                break;
            }
            chunks[kind].push_back(pend[kind]);
        }
        pend_m[0] = pend_m[1] = 0;
    };
    auto append_failed = [&] {
        if (append_rc == JG_OK) return;
        if (open[0]) jg_pnc_wave_abort(pnc_);
        if (open[1]) jg_orset_wave_abort(orset_);
        throw EngineError(append_rc, append_why);
    };
    static const size_t min_par = [] {  // below this many messages a chunk runs on the caller alone
        const char* e = std::getenv("JANUS_HOST_PAR_MIN");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : size_t{8192};
    }();
    // states of other shards' uids are skipped from the uid alone (SetShard), before any table line
    const uint32_t sw = shard_world_ > 1 && !foreign_keys_ ? shard_world_ : 1, sr = shard_rank_;
    std::vector<std::vector<size_t>> cand(T);  // per worker: the current task's messages that may be tracked
    double t_classify = 0, t_gather = 0;
    for (size_t c = 0; c < n_chunks; ++c) {
        const size_t c0 = cb[c], c1 = cb[c + 1];
        const size_t ntask = (c1 - c0 + kTask - 1) / kTask;
        const bool par = T > 1 && c1 - c0 >= min_par;
        auto run = [&](const std::function<void(int)>& fn) {
            if (par) wp.run(fn);
            else fn(0);
        };
        const double ta = wall_s();
        std::atomic<size_t> next{0};
        run([&](int t) {
            if (t == 0) append();  // the previous chunk's upload + pass A, queued
            for (size_t q; (q = next.fetch_add(1, std::memory_order_relaxed)) < ntask;) {
                const size_t e = std::min(c1, c0 + (q + 1) * kTask);
                size_t k[2] = {0, 0}, bytes[2] = {0, 0};
                for (size_t i = c0 + q * kTask; i < e; ++i) {
                    if (i + 16 < e) __builtin_prefetch(msgs[i + 16]);
                    if (i + 8 < e && (sw == 1 || ShardOf(msgs[i + 8]->uid, sw) == sr)) {
                        uids_.prefetch(msgs[i + 8]->uid);
                        if (sweep) tracker->prefetch_claim(msgs[i + 8]->seq);
                    }
                    const NetworkProtocol& u = *msgs[i];
                    uint32_t cl = kSkip;
                    if (u.syncMsgType != NetworkProtocol::ManagerMsg_Create && !u.uid.is_empty() &&  // :133-134
                        (sw == 1 || ShardOf(u.uid, sw) == sr)) {
                        if (const KeyRef* kr = uids_.find(u.uid)) {                                  // :136
                            const int kind = kr->type == CrdtType::PNCounter ? 0 : 1;
                            if (kind == 0) cl = kr->idx;
                            else { cl = kSet; sid[i] = kr->idx; }
                            ++k[kind];
                            bytes[kind] += u.message.size();
                        }
                    }
                    cls[i] = cl;
                    if (sweep && cl != kSkip && tracker->maybe(u.seq)) cand[t].push_back(i);
                }
                // the task's claims after its lookups: each claim is a locked compare-exchange, which
                // drains the core's outstanding loads — inside the loop above it stalled every
                // prefetched lookup behind it (the loop ran 2-3x slower with claims in it)
                for (const size_t i : cand[t]) {
                    uint64_t o;
                    if (tracker->claim(msgs[i]->seq, &o)) part[c * max_tasks + q].emplace_back(i, o);
                }
                cand[t].clear();
                for (int kind = 0; kind < 2; ++kind) {
                    tcnt[kind * max_tasks + q] = k[kind];
                    tbytes[kind * max_tasks + q] = bytes[kind];
                }
            }
        });
        append_failed();
        size_t m[2], nb[2];
        for (int kind = 0; kind < 2; ++kind) {
            size_t* mb = &tmbase[kind * (max_tasks + 1)];
            size_t* bb = &tbbase[kind * (max_tasks + 1)];
            mb[0] = bb[0] = 0;
            for (size_t q = 0; q < ntask; ++q) { mb[q + 1] = mb[q] + tcnt[kind * max_tasks + q]; bb[q + 1] = bb[q] + tbytes[kind * max_tasks + q]; }
            m[kind] = mb[ntask];
            nb[kind] = bb[ntask];
        }
        const double tb = wall_s();
        t_classify += tb - ta;
        Chunk ch[2] = {};
        size_t w0[2];
        for (int kind = 0; kind < 2; ++kind) {
            if (m[kind] == 0) continue;
            const size_t nb_pad = (nb[kind] + 15) & ~size_t(15);
            char* buf = stage(nb_pad + (m[kind] + 1) * 8 + m[kind] * 4 + 64);
            ch[kind] = Chunk{m[kind], buf, reinterpret_cast<uint64_t*>(buf + nb_pad), nullptr, reinterpret_cast<uint8_t*>(buf)};
            ch[kind].rows = reinterpret_cast<uint32_t*>(ch[kind].off + m[kind] + 1);
            w0[kind] = nw[kind];
            nw[kind] += m[kind];
        }
        const double tg = wall_s();
        next.store(0, std::memory_order_relaxed);
        run([&](int) {
            for (size_t q; (q = next.fetch_add(1, std::memory_order_relaxed)) < ntask;) {
                const size_t e = std::min(c1, c0 + (q + 1) * kTask);
                size_t j[2] = {tmbase[q], tmbase[(max_tasks + 1) + q]};
                uint64_t o[2] = {tbbase[q], tbbase[(max_tasks + 1) + q]};
                LineStream out[2] = {LineStream(reinterpret_cast<char*>(ch[0].bytes), o[0]), LineStream(reinterpret_cast<char*>(ch[1].bytes), o[1])};
                for (size_t i = c0 + q * kTask; i < e; ++i) {
                    if (i + 8 < e && cls[i + 8] != kSkip) {  // every line of the payload 8 messages ahead (one prefetch left the rest to miss)
                        const std::string& pq = msgs[i + 8]->message;
                        for (size_t x = 0; x < pq.size(); x += 64) __builtin_prefetch(pq.data() + x);
                    }
                    if (cls[i] == kSkip) continue;
                    const int kind = cls[i] == kSet ? 1 : 0;
                    const std::string& p = msgs[i]->message;
                    Chunk& k = ch[kind];
                    out[kind].put(p.data(), p.size());
                    k.off[j[kind]] = o[kind];
                    k.rows[j[kind]] = kind ? sid[i] : cls[i];
                    where_[kind][w0[kind] + j[kind]] = i;
                    o[kind] += p.size();
                    ++j[kind];
                }
                out[0].finish();
                out[1].finish();
            }
        });
        t_gather += wall_s() - tg;
        for (int kind = 0; kind < 2; ++kind) {
            pend[kind] = ch[kind];
            pend_m[kind] = m[kind];
            pend_nb[kind] = nb[kind];
        }
        if (std::getenv("JANUS_TRACE_WAVE"))
            std::fprintf(stderr, "chunk %zu: classify (+ previous append) %.2f ms, buffers %.2f ms, gather %.2f ms (%zu + %zu msgs, %zu + %zu bytes)\n", c,
                         1e3 * (tb - ta), 1e3 * (tg - tb), 1e3 * (wall_s() - tg), m[0], m[1], nb[0], nb[1]);
    }
    append();  // the last chunk
    append_failed();
    phase_s_[1] = t_classify;
    phase_s_[2] = t_classify + t_gather;
    {
        size_t tot_m = 0, tot_b = 0;
        for (int kind = 0; kind < 2; ++kind)
            for (const Chunk& ch : chunks[kind]) { tot_m += ch.m; tot_b += (size_t)ch.off[ch.m]; }
        if (tot_m) avg_msg_bytes_ = (double)tot_b / (double)tot_m;
    }

    size_t cut = n;
    int cut_code = JG_OK;
    std::string cut_why;
    double to0 = 0, to1 = 0, t1 = 0;
    auto device_side = [&] {
        // OR-Set states: end the device validation; the first rejected state cuts the wave (the reference's
        // loop stops at the state whose Decode / Merge throws).
        to0 = wall_s();
        if (open[1]) {
            uint64_t bad = UINT64_MAX;
            const int rc = jg_orset_wave_check(orset_, &bad);
            if (rc != JG_OK) {
                const std::string why = last_error();
                if (bad == UINT64_MAX) {
                    if (open[0]) jg_pnc_wave_abort(pnc_);
                    jg_orset_wave_abort(orset_);
                    throw EngineError(rc, why);
                }
                cut = where_[1][bad];
                cut_code = rc;
                cut_why = why;
            }
        }
        to1 = wall_s();
        phase_s_[3] = wall_s() - t0;

        t1 = wall_s();
        // Re-stream the first `limit` PNC messages (the reference's loop applied the messages before the
        // one that threw; the engine's PN-Counter waves are all or nothing).
        auto submit_prefix = [&](size_t limit) {
            if (limit == 0) return;
            check(jg_pnc_wave_begin(pnc_, limit, 1));
            size_t left = limit;
            for (const Chunk& ch : chunks[0]) {
                if (!left) break;
                const size_t k = std::min(left, ch.m);
                check(jg_pnc_wave_append(pnc_, k, ch.rows, ch.off, ch.bytes));
                left -= k;
            }
            check(jg_pnc_wave_commit(pnc_, nullptr));
        };
        if (open[0]) {
            if (cut < n) {  // an OR-Set state before some of these PNC states was rejected
                check(jg_pnc_wave_abort(pnc_));
                submit_prefix((size_t)(std::lower_bound(where_[0].begin(), where_[0].begin() + nw[0], (uint64_t)cut) - where_[0].begin()));
            } else {
                uint64_t bad = UINT64_MAX;
                const int rc = jg_pnc_wave_commit(pnc_, &bad);
                if (rc != JG_OK) {
                    if (bad == UINT64_MAX) {
                        if (open[1]) jg_orset_wave_abort(orset_);
                        check(rc);
                    }
                    cut = where_[0][bad];
                    cut_code = rc;
                    cut_why = last_error();
                    submit_prefix(bad);
                }
            }
        }
        pnc_bytes_ = 0;
        for (const Chunk& ch : chunks[0]) pnc_bytes_ += ch.off[ch.m];

        // OR-Set states before the cut: element strings interned in commit order, records unioned into the
        // store (device); then the ids the wave issued join the host tables.
        double to2 = wall_s(), to3 = to2;
        if (open[1]) {
            const uint64_t limit = (uint64_t)(std::lower_bound(where_[1].begin(), where_[1].begin() + nw[1], (uint64_t)cut) - where_[1].begin());
            check(jg_orset_wave_commit(orset_, limit));
            to3 = wall_s();
            take_wave_names();
        }
        orset_phase_s_[0] = to1 - to0;
        orset_phase_s_[1] = to3 - to2;
        orset_phase_s_[2] = wall_s() - to3;
    };
    const double tt = wall_s();
    device_side();
    give_back.armed = false;
    std::vector<uint64_t> completed;
    if (sweep) {
        // parts are in commit order (chunk, task), each ascending: those wholly before the cut are copied
        // on the workers at offsets from a prefix over their sizes (a serial push_back of ~500k
        // completions per C5 wave took ~1 ms); the part reaching the cut and those after it, serially
        const size_t np = part.size();
        std::vector<size_t> at(np + 1, 0);
        size_t whole = np;
        for (size_t k = 0; k < np; ++k) {
            at[k + 1] = at[k] + part[k].size();
            if (whole == np && !part[k].empty() && part[k].back().first >= cut) whole = k;
        }
        completed.resize(at[whole]);
        std::atomic<size_t> next{0};
        auto copy = [&](int) {
            for (size_t k; (k = next.fetch_add(1, std::memory_order_relaxed)) < whole;)
                for (size_t x = 0; x < part[k].size(); ++x) completed[at[k] + x] = part[k][x].second;
        };
        if (T > 1 && at[whole] >= 8 * min_par) wp.run(copy);
        else copy(0);
        size_t kept = at[whole];
        for (size_t k = whole; k < np; ++k)
            for (const auto& [i, o] : part[k]) {
                if (i < cut) completed.push_back(o), ++kept;
                else tracker->add(msgs[i]->seq, o);  // past the cut: not applied, still pending
            }
        tracker->settle(kept);
    }
    host_s_ = t1 - t0;
    engine_s_ = wall_s() - t1;
    if (std::getenv("JANUS_TRACE_WAVE"))
        std::fprintf(stderr, "wave: device side + completions %.2f ms (orset check %.2f commit %.2f names %.2f)\n", 1e3 * (wall_s() - tt),
                     1e3 * orset_phase_s_[0], 1e3 * orset_phase_s_[1], 1e3 * orset_phase_s_[2]);
    if (cut < n) throw ApplyError(cut_code, cut_why, cut, std::move(completed));
    return completed;
}

std::vector<uint8_t> GpuStableStore::ApplyOps(const std::vector<ClientOp>& ops) {
    materialize_names();
    std::vector<uint8_t> result(ops.size(), 1);
    std::vector<uint32_t> pkey, pcol;
    std::vector<int64_t> pdelta;
    std::vector<uint8_t> pisn;
    std::vector<uint32_t> oset, oelem;
    std::vector<uint8_t> oop;
    std::vector<uint64_t> olo, ohi;
    std::vector<size_t> oidx;
    for (size_t i = 0; i < ops.size(); ++i) {  // validate everything first: no partial application
        const KeyRef* kr = uids_.find(ops[i].uid);
        if (!kr) throw EngineError(JG_EINVAL, "unknown CRDT uid");
        const int hi = kr->type == CrdtType::PNCounter ? 2 : 3;
        if (ops[i].opId < 1 || ops[i].opId > hi)
            throw EngineError(JG_EINVAL, kr->type == CrdtType::PNCounter ? "Invalid PNC method name" : "Invalid ORSet method name");
    }
    for (size_t i = 0; i < ops.size(); ++i) {
        const ClientOp& op = ops[i];
        const KeyRef& kr = *uids_.find(op.uid);
        if (kr.type == CrdtType::PNCounter) {
            pkey.push_back(kr.idx);
            pcol.push_back(0);
            pdelta.push_back(eb_ == 4 ? (int64_t)(int32_t)op.amount : op.amount);
            pisn.push_back(op.opId == 2 ? 1 : 0);
        } else {
            SetKey& sk = sets_[kr.idx];
            oset.push_back(kr.idx);
            // Add interns (first insertion); Remove of an unknown element addresses an id no record
            // carries (Contains is false, ORSet.cs:174); Clear empties the Dictionaries, so elements
            // added afterwards take new, larger ids in their new insertion order (ORSet.cs:192-198)
            uint32_t id = 0;
            if (op.opId == 1) id = elem_id(kr.idx, op.elem, true);
            else if (op.opId == 2) id = elem_id(kr.idx, op.elem, false);
            else {
                sk.elems.clear();
                sk.indexed = (uint32_t)sk.names.size();  // every id issued so far is dead
                PendingNames& pn = pending_names_[kr.idx];
                pn.cleared = true;
                pn.ids.clear();
            }
            oelem.push_back(id);
            oop.push_back((uint8_t)op.opId);
            olo.push_back(op.tag.lo);
            ohi.push_back(op.tag.hi);
            oidx.push_back(i);
        }
    }
    if (!pkey.empty()) check(jg_pnc_apply_ops(pnc_, pkey.size(), pkey.data(), pcol.data(), pdelta.data(), pisn.data()));
    if (!oset.empty()) {
        std::vector<uint8_t> r(oset.size());
        check(jg_orset_apply_ops(orset_, oset.size(), oset.data(), oelem.data(), oop.data(), olo.data(), ohi.data(), r.data()));
        for (size_t j = 0; j < oidx.size(); ++j) result[oidx[j]] = r[j];
    }
    return result;
}

int64_t GpuStableStore::QueryStablePNC(const Guid& uid) {
    const uint32_t row = ref(uid, CrdtType::PNCounter).idx;
    int64_t v = 0;
    uint8_t ovf = 0;
    check(jg_pnc_values(pnc_, &row, 1, &v, &ovf));
    if (ovf) throw EngineError(JG_EOVERFLOW, "Arithmetic operation resulted in an overflow.");
    return v;
}

bool GpuStableStore::QueryStableORSet(const Guid& uid, const std::optional<std::string>& elem) {
    const uint32_t set = ref(uid, CrdtType::ORSet).idx;
    const uint32_t id = elem_id(set, elem, false);
    uint8_t out = 0;
    check(jg_orset_contains(orset_, &set, &id, 1, &out));
    return out != 0;
}

std::vector<std::string> GpuStableStore::EncodePNCStates(const std::vector<Guid>& uids) {
    flush_registrations();
    std::vector<uint32_t> rows;
    rows.reserve(uids.size());
    for (const Guid& u : uids) rows.push_back(ref(u, CrdtType::PNCounter).idx);
    std::vector<uint64_t> off(rows.size() + 1, 0);
    check(jg_pnc_encode_json(pnc_, rows.size(), rows.data(), off.data(), nullptr, 0));
    std::string buf(off.back(), '\0');
    check(jg_pnc_encode_json(pnc_, rows.size(), rows.data(), off.data(), reinterpret_cast<uint8_t*>(buf.data()), buf.size()));
    std::vector<std::string> out;
    out.reserve(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) out.emplace_back(buf, off[i], off[i + 1] - off[i]);
    return out;
}

std::vector<std::string> GpuStableStore::EncodeORSetStates(const std::vector<Guid>& uids) {
    materialize_names();
    std::vector<uint32_t> sets;
    sets.reserve(uids.size());
    for (const Guid& u : uids) sets.push_back(ref(u, CrdtType::ORSet).idx);
    const size_t n = sets.size();
    std::vector<uint64_t> ao(n + 1, 0), ro(n + 1, 0);
    check(jg_orset_read_sets(orset_, n, sets.data(), ao.data(), nullptr, 0, ro.data(), nullptr, 0));
    std::vector<jg_tagrec> a(std::max<uint64_t>(ao[n], 1)), r(std::max<uint64_t>(ro[n], 1));
    check(jg_orset_read_sets(orset_, n, sets.data(), ao.data(), a.data(), a.size(), ro.data(), r.data(), r.size()));
    std::vector<std::string> out;
    out.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        const SetKey& sk = sets_[sets[i]];
        ORSetState st;
        // records come sorted by (elem id, tag): one run per element.  Tags enumerate in ascending
        // (ord, tag) (HashSet<Guid> insertion order); addSet elements in ascending id (= the add
        // Dictionary's insertion order); removeSet elements by their first tombstone's ord (= when the
        // element entered the remove Dictionary), ties by id; null last (its own HashSet member).
        auto fill = [&](jg_tagrec* b, jg_tagrec* e, std::vector<std::pair<std::string, std::vector<Guid>>>& dict, std::vector<Guid>& nulls,
                        bool by_first_ord) {
            struct Run { jg_tagrec* b; jg_tagrec* e; uint32_t id; uint64_t first; };
            std::vector<Run> runs;
            for (jg_tagrec* x = b; x < e;) {
                const uint32_t id = (uint32_t)x->key;
                jg_tagrec* y = x;
                uint64_t first = UINT64_MAX;
                for (; y < e && (uint32_t)y->key == id; ++y) first = std::min(first, y->ord);
                std::sort(x, y, [](const jg_tagrec& p, const jg_tagrec& q) {
                    return p.ord != q.ord ? p.ord < q.ord : p.tag_lo != q.tag_lo ? p.tag_lo < q.tag_lo : p.tag_hi < q.tag_hi;
                });
                runs.push_back(Run{x, y, id, first});
                x = y;
            }
            if (by_first_ord)
                std::stable_sort(runs.begin(), runs.end(), [](const Run& p, const Run& q) { return p.first < q.first; });
            for (const Run& r : runs) {
                std::vector<Guid> tags;
                tags.reserve(r.e - r.b);
                for (const jg_tagrec* x = r.b; x < r.e; ++x) tags.push_back(Guid{x->tag_lo, x->tag_hi});
                if (r.id == JG_NULL_ELEM) nulls = std::move(tags);
                else dict.emplace_back(sk.names.at(r.id), std::move(tags));
            }
        };
        fill(a.data() + ao[i], a.data() + ao[i + 1], st.addSet, st.nullAddGuid, false);
        fill(r.data() + ro[i], r.data() + ro[i + 1], st.removeSet, st.nullRemoveGuid, true);
        out.push_back(wire::EncodeORSetMsg(st));
    }
    return out;
}

std::vector<uint8_t> GpuStableStore::SubmitClientUpdates(const std::vector<ClientUpdate>& ups, int clientBatchSize,
                                                         std::vector<UpdateMessage>& submitted,
                                                         SafeUpdateTracker& tracker) {
    const size_t n = ups.size();
    for (const ClientUpdate& u : ups) {  // the wrappers' checks, before anything is applied or queued
        const KeyRef* kr = uids_.find(u.op.uid);
        if (!kr) throw EngineError(JG_EINVAL, "unknown CRDT uid");
        const int hi = kr->type == CrdtType::PNCounter ? 2 : 3;
        if (u.op.opId < 1 || u.op.opId > hi)
            throw EngineError(JG_EINVAL, kr->type == CrdtType::PNCounter ? "Invalid PNC method name" : "Invalid ORSet method name");
    }
    // 1. The batcher over message identities (SafeCRDTManager.cs:165-198); states are filled in below.
    //    q entries: (message, op index or -1 for a message queued by an earlier call).
    constexpr int64_t kOld = -1;
    std::vector<std::pair<NetworkProtocol, int64_t>> q;
    for (auto& np : batch_queue_) q.emplace_back(std::move(np), kOld);
    batch_queue_.clear();
    struct Flush { std::vector<std::pair<NetworkProtocol, int64_t>> msgs; };
    std::vector<Flush> flushes;
    size_t head = 0;  // q[head..] is the live queue
    for (size_t i = 0; i < n; ++i) {
        NetworkProtocol np;
        np.uid = ups[i].op.uid;
        np.syncMsgType = NetworkProtocol::CRDTMsg;
        np.seq = next_seq_++;
        if (ups[i].isSafe && ups[i].origin != 0) tracker.add(np.seq, ups[i].origin);  // SafeCRDT.cs:55-56
        q.emplace_back(std::move(np), (int64_t)i);
        if ((int)(q.size() - head) >= clientBatchSize || ups[i].now_ms - last_submit_ms_ > 100.0) {
            std::vector<std::pair<NetworkProtocol, int64_t>> safe, appeared;
            std::unordered_map<Guid, size_t, GuidHash> pos;  // uid -> slot in `appeared` (first appearance)
            while (head < q.size()) {
                auto e = std::move(q[head++]);                       // TryDequeue first ...
                if (!((int)safe.size() < clientBatchSize)) break;     // ... so this one is lost (:175)
                if (!tracker.contains(e.first.seq)) {
                    auto it = pos.find(e.first.uid);
                    if (it == pos.end()) { pos.emplace(e.first.uid, appeared.size()); appeared.push_back(std::move(e)); }
                    else appeared[it->second] = std::move(e);        // last state wins, position kept
                } else {
                    safe.push_back(std::move(e));
                }
            }
            for (auto& e : appeared) safe.push_back(std::move(e));
            if (!safe.empty()) {
                flushes.push_back(Flush{std::move(safe)});
                last_submit_ms_ = ups[i].now_ms;
            }
        }
    }
    // 2. Which ops' snapshots are needed: those submitted now or still queued.
    std::vector<uint8_t> need(n, 0);
    for (const Flush& f : flushes)
        for (const auto& e : f.msgs)
            if (e.second != kOld) need[(size_t)e.second] = 1;
    for (size_t j = head; j < q.size(); ++j)
        if (q[j].second != kOld) need[(size_t)q[j].second] = 1;
    // 3. Apply the ops in chunks that end at every needed snapshot whose uid is touched again later
    //    in the chunk, encode the needed snapshots after each chunk (on the device).
    std::vector<uint8_t> result(n, 1);
    std::vector<std::string> snap(n);
    size_t c0 = 0;
    while (c0 < n) {
        std::unordered_map<Guid, size_t, GuidHash> last_need;  // uid -> needed op in this chunk
        size_t c1 = c0;
        for (; c1 < n; ++c1) {
            if (last_need.count(ups[c1].op.uid)) break;
            if (need[c1]) last_need.emplace(ups[c1].op.uid, c1);
        }
        std::vector<ClientOp> ops;
        ops.reserve(c1 - c0);
        for (size_t i = c0; i < c1; ++i) ops.push_back(ups[i].op);
        const auto r = ApplyOps(ops);
        std::copy(r.begin(), r.end(), result.begin() + c0);
        std::vector<Guid> pu, ou;
        std::vector<size_t> pi, oi;
        for (const auto& kv : last_need) {
            if (uids_.find(kv.first)->type == CrdtType::PNCounter) { pu.push_back(kv.first); pi.push_back(kv.second); }
            else { ou.push_back(kv.first); oi.push_back(kv.second); }
        }
        if (!pu.empty()) {
            auto enc = EncodePNCStates(pu);
            for (size_t j = 0; j < pi.size(); ++j) snap[pi[j]] = std::move(enc[j]);
        }
        if (!ou.empty()) {
            auto enc = EncodeORSetStates(ou);
            for (size_t j = 0; j < oi.size(); ++j) snap[oi[j]] = std::move(enc[j]);
        }
        c0 = c1;
    }
    // 4. Submitted UpdateMessages and the remaining queue carry the snapshots; each new UpdateMessage
    //    gets its digest (the constructor's ComputeDigest, DAGUpdateMessage.cs:25-30).
    const size_t s0 = submitted.size();
    for (Flush& f : flushes) {
        UpdateMessage um;
        for (auto& e : f.msgs) {
            if (e.second != kOld) e.first.message = snap[(size_t)e.second];
            um.update.push_back(std::move(e.first));
        }
        submitted.push_back(std::move(um));
    }
    ComputeDigests(ctx_, submitted, s0);
    for (size_t j = head; j < q.size(); ++j) {
        if (q[j].second != kOld) q[j].first.message = snap[(size_t)q[j].second];
        batch_queue_.push_back(std::move(q[j].first));
    }
    return result;
}

void ComputeDigests(jg_ctx* ctx, std::vector<UpdateMessage>& msgs, size_t first) {
    if (first >= msgs.size()) return;
    std::vector<uint64_t> off{0}, upd{0};
    for (size_t u = first; u < msgs.size(); ++u) {
        for (const auto& np : msgs[u].update) off.push_back(off.back() + np.message.size());
        upd.push_back(off.size() - 1);
    }
    std::string bytes;
    bytes.reserve(off.back());
    for (size_t u = first; u < msgs.size(); ++u)
        for (const auto& np : msgs[u].update) bytes += np.message;
    std::vector<uint8_t> dig(32 * (msgs.size() - first));
    const int rc = jg_update_digests(ctx, off.size() - 1, off.data(), reinterpret_cast<const uint8_t*>(bytes.data()), nullptr, upd.size() - 1,
                            upd.data(), nullptr, dig.data());
    if (rc != JG_OK) throw EngineError(rc, last_error());
    for (size_t u = first; u < msgs.size(); ++u) std::memcpy(msgs[u].digest.data(), dig.data() + 32 * (u - first), 32);
}

std::vector<std::optional<std::string>> GpuStableStore::QueryStableLookupAll(const Guid& uid) {
    materialize_names();
    const uint32_t set = ref(uid, CrdtType::ORSet).idx;
    uint64_t off[2] = {0, 0};
    check(jg_orset_lookup_all(orset_, 1, &set, off, nullptr, 0));
    std::vector<uint32_t> ids(off[1] ? off[1] : 1);
    check(jg_orset_lookup_all(orset_, 1, &set, off, ids.data(), ids.size()));
    std::vector<std::optional<std::string>> out;
    const SetKey& sk = sets_[set];
    for (uint64_t i = 0; i < off[1]; ++i) {
        if (ids[i] == JG_NULL_ELEM) out.emplace_back(std::nullopt);
        else out.emplace_back(sk.names.at(ids[i]));
    }
    return out;
}

}  // namespace janus
