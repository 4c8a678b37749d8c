// janus_host.cpp — see janus_host.hpp.
#include "janus_host.hpp"

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
bool rec_less(const jg_tagrec& a, const jg_tagrec& b) {
    if (a.key != b.key) return a.key < b.key;
    if (a.tag_lo != b.tag_lo) return a.tag_lo < b.tag_lo;
    return a.tag_hi < b.tag_hi;
}
bool rec_eq(const jg_tagrec& a, const jg_tagrec& b) { return a.key == b.key && a.tag_lo == b.tag_lo && a.tag_hi == b.tag_hi; }
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
    for (auto& c : chunks_)
        if (c.first) jg_host_free(c.first);
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
    std::vector<Slot> old = std::move(slots_);
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

uint32_t GpuStableStore::elem_id(SetKey& s, const std::optional<std::string>& e, bool create) {
    if (!e) return JG_NULL_ELEM;
    auto it = s.elems.find(*e);
    if (it != s.elems.end()) return it->second;
    if (!create) return JG_NULL_ELEM - 1;  // never allocated: no records carry it
    // ids only grow (also across Clear), so ascending id = insertion order into the add Dictionary
    const uint32_t id = (uint32_t)s.names.size();
    if (id >= JG_NULL_ELEM - 1) throw EngineError(JG_ESTATE, "too many elements in one OR-Set");
    s.elems.emplace(*e, id);
    s.names.push_back(*e);
    return id;
}

void GpuStableStore::CreateSafeCRDT(const Guid& uid, CrdtType type, const Guid& stableReplicaGuid) {
    if (uids_.find(uid)) return;
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
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
}

WorkerPool& GpuStableStore::pool() {
    if (!pool_ || pool_->size() != host_threads()) pool_ = std::make_unique<WorkerPool>(host_threads());
    return *pool_;
}

char* GpuStableStore::chunk_buffer(size_t c, size_t bytes) {
    if (chunks_.size() <= c) chunks_.resize(c + 1, {nullptr, 0});
    auto& s = chunks_[c];
    if (s.second < bytes) {
        if (s.first) jg_host_free(s.first);
        s = {nullptr, 0};
        void* p = nullptr;
        const size_t want = bytes + bytes / 4 + 4096;
        check(jg_host_alloc(ctx_, want, &p));
        s = {static_cast<char*>(p), want};
    }
    return s.first;
}

std::vector<uint64_t> GpuStableStore::ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates,
                                                     std::unordered_map<uint64_t, uint64_t>* tracker) {
    const double t0 = wall_s();
    std::vector<const NetworkProtocol*> msgs;
    size_t n_msgs = 0;
    for (const auto& list : updates)
        for (const auto& block : list) n_msgs += block.update.size();
    msgs.reserve(n_msgs);
    for (const auto& list : updates)
        for (const auto& block : list)
            for (const auto& u : block.update) msgs.push_back(&u);
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

std::vector<uint64_t> GpuStableStore::apply_msgs(const std::vector<const NetworkProtocol*>& msgs,
                                                 std::unordered_map<uint64_t, uint64_t>* tracker, double t0) {
    flush_registrations();
    const size_t n = msgs.size();
    WorkerPool& wp = pool();
    const int T = wp.size();
    phase_s_[0] = wall_s() - t0;
    constexpr uint32_t kSkip = UINT32_MAX, kSet = UINT32_MAX - 1;
    static const size_t chunk_msgs = [] {
        const char* e = std::getenv("JANUS_WAVE_CHUNK");
        return e ? std::max<size_t>(1, std::strtoull(e, nullptr, 10)) : size_t{131072};
    }();

    // The wave is streamed in chunks of commit order: classify + gather chunk c on the host workers
    // while the engine uploads and scans chunk c-1 (jg_pnc_wave_append returns once queued).
    // A chunk's pinned buffer: [payload | pad 16 | off (m+1) u64 | rows u32]; it stays untouched
    // until the wave is committed or aborted.
    std::vector<uint32_t> cls(n);
    struct Chunk { size_t m; char* buf; uint64_t* off; uint32_t* rows; uint8_t* bytes; };
    std::vector<Chunk> chunks;
    std::vector<uint64_t> where;  // PNC message (wave order) -> commit index
    std::vector<size_t> cnt(T), nbytes(T), mbase(T + 1), bbase(T + 1);
    const size_t n_chunks = (n + chunk_msgs - 1) / chunk_msgs;
    bool open = false;
    double t_classify = 0, t_gather = 0;
    for (size_t c = 0; c < n_chunks; ++c) {
        const size_t c0 = c * chunk_msgs, c1 = std::min(n, c0 + chunk_msgs);
        const double ta = wall_s();
        parallel_ranges(wp, c1 - c0, [&](size_t b, size_t e, int t) {
            size_t k = 0, bytes = 0;
            for (size_t i = c0 + b; i < c0 + e; ++i) {
                if (i + 16 < c0 + e) __builtin_prefetch(msgs[i + 16]);
                if (i + 8 < c0 + e) uids_.prefetch(msgs[i + 8]->uid);
                const NetworkProtocol& u = *msgs[i];
                uint32_t cl = kSkip;
                if (u.syncMsgType != NetworkProtocol::ManagerMsg_Create && !u.uid.is_empty()) {  // :133-134
                    if (const KeyRef* kr = uids_.find(u.uid)) {                                  // :136
                        if (kr->type == CrdtType::PNCounter) { cl = kr->idx; ++k; bytes += u.message.size(); }
                        else cl = kSet;
                    }
                }
                cls[i] = cl;
            }
            cnt[t] = k;
            nbytes[t] = bytes;
        });
        for (int t = 0; t < T; ++t) { mbase[t + 1] = mbase[t] + cnt[t]; bbase[t + 1] = bbase[t] + nbytes[t]; }
        const size_t m = mbase[T], nb = bbase[T], nb_pad = (nb + 15) & ~size_t(15);
        const double tb = wall_s();
        t_classify += tb - ta;
        if (m == 0) continue;
        char* buf = chunk_buffer(chunks.size(), nb_pad + (m + 1) * 8 + m * 4 + 64);
        Chunk ch{m, buf, reinterpret_cast<uint64_t*>(buf + nb_pad), nullptr, reinterpret_cast<uint8_t*>(buf)};
        ch.rows = reinterpret_cast<uint32_t*>(ch.off + m + 1);
        const size_t w0 = where.size();
        where.resize(w0 + m);
        parallel_ranges(wp, c1 - c0, [&](size_t b, size_t e, int t) {
            size_t j = mbase[t];
            uint64_t o = bbase[t];
            for (size_t i = c0 + b; i < c0 + e; ++i) {
                if (i + 8 < c0 + e) __builtin_prefetch(msgs[i + 8]->message.data());
                if (cls[i] >= kSet) continue;
                const std::string& p = msgs[i]->message;
                std::memcpy(ch.bytes + o, p.data(), p.size());
                ch.off[j] = o;
                ch.rows[j] = cls[i];
                where[w0 + j] = i;
                o += p.size();
                ++j;
            }
        });
        ch.off[m] = nb;
        t_gather += wall_s() - tb;
        if (!open) {
            check(jg_pnc_wave_begin(pnc_, std::max<size_t>(m * n_chunks, 1), std::max<size_t>(nb * n_chunks, 1)));
            open = true;
        }
        const int rc = jg_pnc_wave_append(pnc_, m, ch.rows, ch.off, ch.bytes);
        if (rc != JG_OK) {
            jg_pnc_wave_abort(pnc_);
            check(rc);
        }
        chunks.push_back(ch);
    }
    phase_s_[1] = t_classify;
    phase_s_[2] = t_classify + t_gather;

    // OR-Set states: one parse per payload, straight into element interning and records (no decoded
    // ORSetState).  Sets are independent, so the states are grouped by set (stable: commit order
    // within a set) and the sets split into contiguous id ranges over the workers; each worker interns
    // its sets' elements in commit order and keeps each set's distinct records (a full-state message
    // repeats most of them), sorted.  Worker outputs concatenated in worker order are sorted by
    // (set, elem, tag).  A payload the reader rejects cuts the wave at the first one in commit order:
    // the records of later states are dropped and the element ids they issued are withdrawn.
    std::vector<size_t> set_msgs;
    for (size_t i = 0; i < n; ++i)
        if (cls[i] == kSet) set_msgs.push_back(i);
    std::vector<size_t> first_bad(T, SIZE_MAX);
    std::vector<int> bad_code(T, JG_OK);
    std::vector<std::string> why(T);
    std::vector<std::vector<jg_tagrec>> wadd(T), wrem(T);
    auto rollback = [](SetKey& sk, size_t names0) {  // withdraw the ids issued since names0
        for (size_t q = names0; q < sk.names.size(); ++q) sk.elems.erase(sk.names[q]);
        sk.names.resize(names0);
    };
    std::vector<uint32_t> names_at_start(next_set_);
    for (uint32_t q = 0; q < next_set_; ++q) names_at_start[q] = (uint32_t)sets_[q].names.size();
    const double to0 = wall_s();
    auto intern_pass = [&](size_t n_set) {  // the first n_set OR-Set states (commit order)
        std::vector<uint32_t> set_of(n_set);
        for (size_t j = 0; j < n_set; ++j) set_of[j] = uids_.find(msgs[set_msgs[j]]->uid)->idx;
        std::vector<uint32_t> first(next_set_ + 1, 0);  // counting sort by set id
        for (size_t j = 0; j < n_set; ++j) ++first[set_of[j] + 1];
        for (uint32_t q = 0; q < next_set_; ++q) first[q + 1] += first[q];
        std::vector<uint32_t> grouped(n_set);
        {
            std::vector<uint32_t> at(first.begin(), first.end() - 1);
            for (size_t j = 0; j < n_set; ++j) grouped[at[set_of[j]]++] = (uint32_t)j;
        }
        // worker t takes the sets whose grouped messages start in [n_set*t/T, n_set*(t+1)/T)
        parallel_ranges(wp, n_set, [&](size_t b, size_t e, int t) {
            if (b >= e) return;
            // whole sets only: start at the first set beginning at or after b, end at the first set at or after e
            uint32_t s0 = set_of[grouped[b]], s1 = e < n_set ? set_of[grouped[e]] : next_set_;
            if (b > 0 && set_of[grouped[b - 1]] == s0) ++s0;  // that set belongs to the previous worker
            if (e < n_set && set_of[grouped[e - 1]] == s1) ++s1;
            // A full-state message repeats most of its set's records: each set's records pass a per-side
            // hash set before they are stored, so only distinct records are kept and sorted.
            struct RecSet {
                std::vector<jg_tagrec> slot;
                std::vector<uint32_t> gen;  // slot is live iff gen == cur (O(1) reset per set)
                uint32_t cur = 1;
                size_t n = 0;
                static uint64_t h(const jg_tagrec& r) {
                    uint64_t x = r.key * 0x9E3779B97F4A7C15ull ^ r.tag_lo ^ (r.tag_hi * 0xBF58476D1CE4E5B9ull);
                    x ^= x >> 31;
                    x *= 0x94D049BB133111EBull;
                    return x ^ (x >> 29);
                }
                void reset() {
                    if (++cur == 0) { std::fill(gen.begin(), gen.end(), 0u); cur = 1; }
                    n = 0;
                }
                bool insert(const jg_tagrec& r) {  // true if new
                    if ((n + 1) * 2 > slot.size()) grow();
                    const size_t mask = slot.size() - 1;
                    for (size_t i = h(r) & mask;; i = (i + 1) & mask) {
                        if (gen[i] != cur) { gen[i] = cur; slot[i] = r; ++n; return true; }
                        if (rec_eq(slot[i], r)) return false;
                    }
                }
                void grow() {
                    std::vector<jg_tagrec> old;
                    std::vector<uint32_t> og;
                    old.swap(slot);
                    og.swap(gen);
                    const size_t sz = old.empty() ? 1024 : old.size() * 2;
                    slot.assign(sz, jg_tagrec{0, 0, 0});
                    gen.assign(sz, 0u);
                    const uint32_t was = cur;
                    cur = 1;
                    n = 0;
                    for (size_t i = 0; i < old.size(); ++i)
                        if (og[i] == was) insert(old[i]);
                }
            };
            struct Ctx {
                GpuStableStore* self;
                SetKey* sk;
                uint64_t hi;
                std::vector<jg_tagrec>* out[2];
                RecSet seen[2];
            } c{this, nullptr, 0, {&wadd[t], &wrem[t]}, {}};
            for (uint32_t sid = s0; sid < s1 && sid < next_set_; ++sid) {
                if (first[sid] == first[sid + 1]) continue;
                c.sk = &sets_[sid];
                c.hi = (uint64_t)sid << 32;
                c.seen[0].reset();
                c.seen[1].reset();
                const size_t a0 = wadd[t].size(), r0 = wrem[t].size();
                for (uint32_t x = first[sid]; x < first[sid + 1]; ++x) {
                    const size_t i = set_msgs[grouped[x]];
                    const size_t names0 = c.sk->names.size();
                    try {
                        wire::ScanORSetMsg(msgs[i]->message,
                                           [](void* p, int side, std::string_view name, bool is_null, const Guid* tags, size_t nt) {
                                               Ctx& k = *static_cast<Ctx*>(p);
                                               if (side == 0 && !is_null && nt == 0)
                                                   throw EngineError(JG_ESTATE, "empty add tag set (not produced by ORSet.Add)");
                                               const uint64_t key = k.hi | (is_null ? JG_NULL_ELEM : k.self->elem_id(*k.sk, std::string(name), true));
                                               for (size_t q = 0; q < nt; ++q) {
                                                   const jg_tagrec r{key, tags[q].lo, tags[q].hi};
                                                   if (k.seen[side].insert(r)) k.out[side]->push_back(r);
                                               }
                                           },
                                           &c);
                    } catch (const EngineError& err) {
                        // the reference's loop stops at this state; later states of this set come after it
                        rollback(*c.sk, names0);
                        if (i < first_bad[t]) { first_bad[t] = i; why[t] = err.what(); bad_code[t] = err.code; }
                        break;
                    }
                }
                auto dedup = [](std::vector<jg_tagrec>& v, size_t from) {
                    std::sort(v.begin() + from, v.end(), rec_less);
                    v.erase(std::unique(v.begin() + from, v.end(), rec_eq), v.end());
                };
                dedup(wadd[t], a0);
                dedup(wrem[t], r0);
            }
        });
    };
    intern_pass(set_msgs.size());
    size_t cut = n;
    int cut_code = JG_OK;
    std::string cut_why;
    for (int t = 0; t < T; ++t)
        if (first_bad[t] < cut) { cut = first_bad[t]; cut_why = why[t]; cut_code = bad_code[t]; }
    phase_s_[3] = wall_s() - t0;

    const double t1 = wall_s();
    // Re-stream the first `limit` PNC messages (the reference's loop applied the messages before the
    // one that threw; the engine's waves are all or nothing).
    auto submit_prefix = [&](size_t limit) {
        if (limit == 0) return;
        check(jg_pnc_wave_begin(pnc_, limit, 1));
        size_t left = limit;
        for (const Chunk& ch : chunks) {
            if (!left) break;
            const size_t k = std::min(left, ch.m);
            check(jg_pnc_wave_append(pnc_, k, ch.rows, ch.off, ch.bytes));
            left -= k;
        }
        check(jg_pnc_wave_commit(pnc_, nullptr));
    };
    if (open) {
        if (cut < n) {  // an OR-Set state before some of these PNC states was rejected
            check(jg_pnc_wave_abort(pnc_));
            submit_prefix((size_t)(std::lower_bound(where.begin(), where.end(), (uint64_t)cut) - where.begin()));
        } else {
            uint64_t bad = UINT64_MAX;
            const int rc = jg_pnc_wave_commit(pnc_, &bad);
            if (rc != JG_OK) {
                if (bad == UINT64_MAX) check(rc);
                cut = where[bad];
                cut_code = rc;
                cut_why = last_error();
                submit_prefix(bad);
            }
        }
    }
    pnc_bytes_ = 0;
    for (const Chunk& ch : chunks) pnc_bytes_ += ch.off[ch.m];

    // A cut (a rejected OR-Set or PN-Counter state) before some OR-Set state: redo the OR-Set part over
    // the states before it, from the element tables as they were.
    if (!set_msgs.empty() && set_msgs.back() >= cut) {
        for (uint32_t q = 0; q < next_set_; ++q) rollback(sets_[q], names_at_start[q]);
        for (int t = 0; t < T; ++t) { wadd[t].clear(); wrem[t].clear(); first_bad[t] = SIZE_MAX; }
        size_t n_set = 0;
        while (n_set < set_msgs.size() && set_msgs[n_set] < cut) ++n_set;
        intern_pass(n_set);
    }
    std::vector<jg_tagrec> adds, rems;
    {
        size_t na = 0, nr = 0;
        for (int t = 0; t < T; ++t) { na += wadd[t].size(); nr += wrem[t].size(); }
        adds.reserve(na);
        rems.reserve(nr);
        for (int t = 0; t < T; ++t) {
            adds.insert(adds.end(), wadd[t].begin(), wadd[t].end());
            rems.insert(rems.end(), wrem[t].begin(), wrem[t].end());
        }
    }
    const double to1 = wall_s();
    double to2 = to1;
    if (!adds.empty() || !rems.empty()) {
        to2 = wall_s();
        check(jg_orset_merge(orset_, adds.data(), adds.size(), rems.data(), rems.size()));
    }
    orset_phase_s_[0] = to1 - to0;
    orset_phase_s_[1] = to2 - to1;
    orset_phase_s_[2] = wall_s() - to2;
    std::vector<uint64_t> completed;
    if (tracker)
        for (size_t i = 0; i < cut; ++i) {
            if (cls[i] == kSkip) continue;
            auto tr = tracker->find(msgs[i]->seq);
            if (tr != tracker->end()) { completed.push_back(tr->second); tracker->erase(tr); }
        }
    host_s_ = t1 - t0;
    engine_s_ = wall_s() - t1;
    if (cut < n) throw ApplyError(cut_code, cut_why, cut, std::move(completed));
    return completed;
}

std::vector<uint8_t> GpuStableStore::ApplyOps(const std::vector<ClientOp>& ops) {
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
            if (op.opId == 1) id = elem_id(sk, op.elem, true);
            else if (op.opId == 2) id = elem_id(sk, op.elem, false);
            else sk.elems.clear();
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
    const uint32_t id = elem_id(sets_[set], elem, false);
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
        // records are sorted by (elem id, tag): one run per element, ascending id = insertion order
        auto fill = [&](const jg_tagrec* b, const jg_tagrec* e, std::vector<std::pair<std::string, std::vector<Guid>>>& dict,
                        std::vector<Guid>& nulls) {
            for (const jg_tagrec* x = b; x < e;) {
                const uint32_t id = (uint32_t)x->key;
                const jg_tagrec* y = x;
                std::vector<Guid> tags;
                for (; y < e && (uint32_t)y->key == id; ++y) tags.push_back(Guid{y->tag_lo, y->tag_hi});
                if (id == JG_NULL_ELEM) nulls = std::move(tags);
                else dict.emplace_back(sk.names.at(id), std::move(tags));
                x = y;
            }
        };
        fill(a.data() + ao[i], a.data() + ao[i + 1], st.addSet, st.nullAddGuid);
        fill(r.data() + ro[i], r.data() + ro[i + 1], st.removeSet, st.nullRemoveGuid);
        out.push_back(wire::EncodeORSetMsg(st));
    }
    return out;
}

std::vector<uint8_t> GpuStableStore::SubmitClientUpdates(const std::vector<ClientUpdate>& ups, int clientBatchSize,
                                                         std::vector<UpdateMessage>& submitted,
                                                         std::unordered_map<uint64_t, uint64_t>& tracker) {
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
        if (ups[i].isSafe && ups[i].origin != 0) tracker[np.seq] = ups[i].origin;  // SafeCRDT.cs:55-56
        q.emplace_back(std::move(np), (int64_t)i);
        if ((int)(q.size() - head) >= clientBatchSize || ups[i].now_ms - last_submit_ms_ > 100.0) {
            std::vector<std::pair<NetworkProtocol, int64_t>> safe, appeared;
            std::unordered_map<Guid, size_t, GuidHash> pos;  // uid -> slot in `appeared` (first appearance)
            while (head < q.size()) {
                auto e = std::move(q[head++]);                       // TryDequeue first ...
                if (!((int)safe.size() < clientBatchSize)) break;     // ... so this one is lost (:175)
                if (!tracker.count(e.first.seq)) {
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
    // 4. Submitted UpdateMessages and the remaining queue carry the snapshots.
    for (Flush& f : flushes) {
        UpdateMessage um;
        for (auto& e : f.msgs) {
            if (e.second != kOld) e.first.message = snap[(size_t)e.second];
            um.update.push_back(std::move(e.first));
        }
        submitted.push_back(std::move(um));
    }
    for (size_t j = head; j < q.size(); ++j) {
        if (q[j].second != kOld) q[j].first.message = snap[(size_t)q[j].second];
        batch_queue_.push_back(std::move(q[j].first));
    }
    return result;
}

std::vector<std::optional<std::string>> GpuStableStore::QueryStableLookupAll(const Guid& uid) {
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
