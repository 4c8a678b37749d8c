// janus_host.cpp — see janus_host.hpp.
#include "janus_host.hpp"

#include <cstdio>
#include <cstring>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <limits>
#include <memory>
#include <condition_variable>
#include <functional>
#include <future>
#include <unordered_set>
#include <mutex>
#include <string_view>
#include <thread>

#include "host_pool.hpp"
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
    check(jg_node_create(pnc_, orset_, &node_));
}

GpuStableStore::~GpuStableStore() {
    if (p_bytes_) jg_host_free(p_bytes_);
    if (pin_buf_) jg_host_free(pin_buf_);
    if (pin_aux_) jg_host_free(pin_aux_);
    for (uint8_t* b : pin_more_) jg_host_free(b);
    if (node_) jg_node_destroy(node_);
    if (orset_) jg_orset_destroy(orset_);
    if (pnc_) jg_pnc_destroy(pnc_);
    if (ctx_) jg_close(ctx_);
}


const GpuStableStore::KeyRef& GpuStableStore::ref(const Guid& uid, CrdtType want) const {
    const auto it = uids_.find(uid);
    if (it == uids_.end()) throw EngineError(JG_EINVAL, "unknown CRDT uid");
    if (it->second.type != want) throw EngineError(JG_ETYPE, "CRDT uid is of the other type");
    return it->second;
}

uint32_t GpuStableStore::elem_id(uint32_t set, const std::optional<std::string>& e, bool create) {
    if (!e) return JG_NULL_ELEM;
    materialize_names();
    return elem_id_in(sets_[set], create ? &pending_names_[set] : nullptr, *e, create);
}

// One set's interning (the caller has materialized the names; pn: the set's pending entry, when creating).  Touches
// only this set's tables: the producer path runs it for different sets on different workers.
uint32_t GpuStableStore::elem_id_in(SetKey& s, PendingNames* pn, const std::string& e, bool create) {
    for (; s.indexed < s.names.size(); ++s.indexed) s.elems.emplace(s.names[s.indexed], s.indexed);  // ids a wave issued
    auto it = s.elems.find(e);
    if (it != s.elems.end()) return it->second;
    if (!create) return JG_NULL_ELEM - 1;  // never allocated: no records carry it
    // ids only grow (also across Clear), so ascending id = insertion order into the add Dictionary
    const uint32_t id = (uint32_t)s.names.size();
    if (id >= JG_NULL_ELEM - 1) throw EngineError(JG_ESTATE, "too many elements in one OR-Set");
    s.elems.emplace(e, id);
    s.names.push_back(e);
    s.indexed = (uint32_t)s.names.size();
    pn->ids.push_back(id);
    return id;
}

void GpuStableStore::ensure_uid_index() {
    if (uidx_n_ == uids_.size()) return;
    uint64_t cap = 1024;
    while (cap < 2 * (uint64_t)uids_.size()) cap <<= 1;
    uidx_.assign(cap, UidSlot{0, 0, nullptr, 0});
    uidx_mask_ = cap - 1;
    for (const auto& kv : uids_) {
        uint64_t h = uid_slot0(kv.first);
        while (uidx_[h].kr) h = (h + 1) & uidx_mask_;
        uidx_[h] = UidSlot{kv.first.lo, kv.first.hi, &kv.second, 0};
    }
    uidx_n_ = uids_.size();
}

void GpuStableStore::CreateSafeCRDT(const Guid& uid, CrdtType type, const Guid& stableReplicaGuid) {
    if (uids_.count(uid)) return;
    KeyRef kr{type, 0};
    if (type == CrdtType::PNCounter) {
        if (next_row_ >= max_keys_) throw EngineError(JG_ESTATE, "PNCounter store full");
        kr.idx = next_row_++;
        reg_rows_.push_back(kr.idx);  // {self: 0} — the row is zero already; column 0 once flushed
        reg_guids_.push_back(jg_guid{stableReplicaGuid.lo, stableReplicaGuid.hi});
    } else {
        kr.idx = next_set_++;
        sets_.emplace_back();
    }
    uids_.emplace(uid, kr);
    reg_uid_.push_back(jg_guid{uid.lo, uid.hi});  // safeCRDTsIndexedByuid[uid] (SafeCRDTManager.cs:73, 98)
    reg_type_.push_back(type == CrdtType::PNCounter ? 0 : 1);
    reg_idx_.push_back(kr.idx);
}

void GpuStableStore::flush_registrations() {
    if (!reg_uid_.empty()) {
        check(jg_node_register(node_, reg_uid_.size(), reg_uid_.data(), reg_type_.data(), reg_idx_.data()));
        reg_uid_.clear();
        reg_type_.clear();
        reg_idx_.clear();
    }
    if (reg_rows_.empty()) return;
    std::vector<uint32_t> cols(reg_rows_.size());
    check(jg_pnc_intern(pnc_, reg_rows_.size(), reg_rows_.data(), reg_guids_.data(), cols.data()));
    reg_rows_.clear();
    reg_guids_.clear();
}

uint32_t GpuStableStore::ShardOf(const Guid& uid, uint32_t world) {
    const jg_guid g{uid.lo, uid.hi};
    uint32_t r = 0;
    if (jg_shard_of(&g, world, &r) != JG_OK) throw EngineError(JG_EINVAL, last_error());
    return r;
}

void GpuStableStore::SetShard(uint32_t rank, uint32_t world) {
    flush_registrations();  // the shard rescan sees every key registered so far
    check(jg_node_set_shard(node_, rank, world));
}

SafeUpdateTracker::SafeUpdateTracker(jg_ctx* ctx) {
    if (jg_tracker_create(ctx, &t_) != JG_OK) throw EngineError(JG_EINVAL, last_error());
}
SafeUpdateTracker::~SafeUpdateTracker() { jg_tracker_destroy(t_); }
void SafeUpdateTracker::add(uint64_t seq, uint64_t origin) {
    if (jg_tracker_add(t_, 1, &seq, &origin) != JG_OK) throw EngineError(JG_EINVAL, last_error());
}
void SafeUpdateTracker::add_many(size_t n, const uint64_t* seq, const uint64_t* origin) {
    if (n && jg_tracker_add(t_, n, seq, origin) != JG_OK) throw EngineError(JG_EINVAL, last_error());
}
bool SafeUpdateTracker::contains(uint64_t seq) const {
    uint8_t r = 0;
    if (jg_tracker_contains(t_, 1, &seq, &r) != JG_OK) throw EngineError(JG_EINVAL, last_error());
    return r != 0;
}
size_t SafeUpdateTracker::size() const {
    uint64_t n = 0;
    if (jg_tracker_size(t_, &n) != JG_OK) throw EngineError(JG_EINVAL, last_error());
    return n;
}


namespace {
// Static contiguous split of [0, n) over the pool's workers: fn(begin, end, worker).
// min_items: below this many items the phase runs inline (default JANUS_HOST_PAR_MIN or 8192: element-wise
// loops; a loop over heavy items — a batcher flush of ~1000 messages — passes its own)
template <class F> void parallel_ranges(jg::WorkerPool& pool, size_t n, F&& fn, size_t min_items = 0) {
    static const size_t min_par_default = [] {
        const char* e = std::getenv("JANUS_HOST_PAR_MIN");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : size_t{8192};
    }();
    const size_t min_par = min_items ? min_items : min_par_default;
    const int T = pool.size();
    if (T <= 1 || n < min_par || n < (size_t)T) {
        fn(size_t{0}, n, 0);
        for (int t = 1; t < T; ++t) fn(n, n, t);
        return;
    }
    pool.run([&](int t) { fn(n * t / T, n * (t + 1) / T, t); });
}
}  // namespace

jg::WorkerPool& GpuStableStore::pool() {
    if (!pool_ || pool_->size() != jg::host_threads()) pool_ = std::make_unique<jg::WorkerPool>(jg::host_threads());
    return *pool_;
}

void GpuStableStore::flush_names() {
    if (pending_names_.empty()) return;
    materialize_names();
    // per pending set: its entry, then its names' slots and bytes (counted, then filled by the workers)
    const size_t P = pending_names_.size();
    std::vector<const std::pair<const uint32_t, PendingNames>*> pv;
    pv.reserve(P);
    std::vector<uint32_t> set(P), next(P);
    std::vector<uint8_t> cleared(P);
    std::vector<size_t> nat(P + 1, 0), bat(P + 1, 0);
    for (const auto& kv : pending_names_) {
        const size_t k = pv.size();
        pv.push_back(&kv);
        set[k] = kv.first;
        next[k] = (uint32_t)sets_[kv.first].names.size();
        cleared[k] = kv.second.cleared ? 1 : 0;
        nat[k + 1] = kv.second.ids.size();
    }
    parallel_ranges(pool(), P, [&](size_t b, size_t e, int) {
        for (size_t k = b; k < e; ++k) {
            const SetKey& sk = sets_[pv[k]->first];
            size_t nb = 0;
            for (uint32_t id : pv[k]->second.ids) nb += sk.names[id].size();
            bat[k + 1] = nb;
        }
    }, 64);
    for (size_t k = 0; k < P; ++k) nat[k + 1] += nat[k], bat[k + 1] += bat[k];
    const size_t nn = nat[P];
    std::vector<uint32_t> nset(nn), nid(nn);
    std::vector<uint64_t> off(nn + 1, 0);
    std::vector<uint8_t> bytes(std::max<size_t>(bat[P], 1));
    parallel_ranges(pool(), P, [&](size_t b, size_t e, int) {
        for (size_t k = b; k < e; ++k) {
            const SetKey& sk = sets_[pv[k]->first];
            size_t j = nat[k], at = bat[k];
            for (uint32_t id : pv[k]->second.ids) {
                const std::string& nm = sk.names[id];
                nset[j] = pv[k]->first;
                nid[j] = id;
                std::memcpy(bytes.data() + at, nm.data(), nm.size());
                at += nm.size();
                off[++j] = at;
            }
        }
    }, 64);
    check(jg_orset_names_sync(orset_, P, set.data(), next.data(), cleared.data(), nn, nset.data(), nid.data(), off.data(), bytes.data()));
    names_seen_ += nn;  // caught up before the sync (materialize_names above): the log's new tail is ours
    pending_names_.clear();
}

// The names the engine's waves issued since the last pull (its names log past names_seen_, several waves
// at once), appended to the SetKey tables, the sets split over the workers in contiguous ranges.  The log
// is in issue order: within a set, ids ascend.
void GpuStableStore::materialize_names() {
    if (!orset_) return;
    uint64_t to = 0, nb = 0;
    check(jg_orset_names_since(orset_, names_seen_, &to, &nb, nullptr, nullptr, nullptr, nullptr));
    if (to == names_seen_) return;
    const uint64_t n = to - names_seen_;
    std::vector<uint32_t> set(n), id(n);
    std::vector<uint64_t> off(n + 1);
    std::vector<uint8_t> bytes(std::max<uint64_t>(nb, 1));
    check(jg_orset_names_since(orset_, names_seen_, &to, &nb, set.data(), id.data(), off.data(), bytes.data()));
    // per set the log's ids ascend, but a set's names may interleave with other sets' across waves: group the
    // log's entries by set (stable), then each worker appends whole sets
    std::vector<uint32_t> order(n);
    for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return set[a] < set[b]; });
    std::vector<int> bad(pool().size(), 0);
    parallel_ranges(pool(), n, [&](size_t b, size_t e, int t) {
        while (b < n && b > 0 && set[order[b - 1]] == set[order[b]]) ++b;  // that set belongs to the previous worker
        while (e < n && e > 0 && set[order[e - 1]] == set[order[e]]) ++e;
        for (size_t k = b; k < e; ++k) {
            const uint32_t i = order[k];
            SetKey& sk = sets_[set[i]];
            if (id[i] != sk.names.size()) { bad[t] = 1; return; }
            sk.names.emplace_back(reinterpret_cast<const char*>(bytes.data()) + off[i], off[i + 1] - off[i]);  // elems: lazily
        }
    });
    for (int x : bad)
        if (x) throw EngineError(JG_ESTATE, "element ids of the engine and the host tables disagree");
    names_seen_ = to;
}

std::vector<uint64_t> GpuStableStore::ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker) {
    std::vector<const UpdateMessage*> blocks;
    for (const auto& list : updates)
        for (const auto& block : list) blocks.push_back(&block);
    return apply(blocks, tracker, false);
}

void GpuStableStore::ReceivedBlock(const std::vector<UpdateMessage>& block) {
    std::vector<const UpdateMessage*> blocks;
    for (const auto& um : block) blocks.push_back(&um);
    apply(blocks, nullptr, true);
}

// The wave in commit order (list, block, update) as the jg_commit arrays — what the C# caller builds from
// its List<List<UpdateMessage>> — filled in parallel by messages, then ONE call.
size_t GpuStableStore::index_blocks(const std::vector<const UpdateMessage*>& blocks) {
    block_off_.resize(blocks.size() + 1);
    block_off_[0] = 0;
    for (size_t b = 0; b < blocks.size(); ++b) block_off_[b + 1] = block_off_[b] + blocks[b]->update.size();
    const size_t n = block_off_.back();
    // scratch grows with headroom: an exact fit reallocated (and page-faulted in) the arrays whenever a
    // wave held a few more messages than the largest before it
    if (w_uid_.size() < n) {
        const size_t cap = n + n / 4;
        w_uid_.resize(cap), w_type_.resize(cap), w_seq_.resize(cap), w_ptr_.resize(cap), w_len_.resize(cap);
    }
    return n;
}

size_t GpuStableStore::ApplyCommittedInto(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker,
                                          std::vector<uint64_t>& done) {
    std::vector<const UpdateMessage*> blocks;
    for (const auto& list : updates)
        for (const auto& block : list) blocks.push_back(&block);
    const jg_commit wave = gather_wave(blocks);
    return run_wave_into(wave, tracker, done);
}

// The wave's arrays over the callers' payloads (pointers and lengths, no copy), by the workers.
jg_commit GpuStableStore::gather_wave(const std::vector<const UpdateMessage*>& blocks) {
    flush_registrations();
    flush_names();
    const auto t0 = std::chrono::steady_clock::now();
    const size_t n = index_blocks(blocks);
    parallel_ranges(pool(), n, [&](size_t i0, size_t i1, int) {
        if (i0 >= i1) return;
        size_t b = (size_t)(std::upper_bound(block_off_.begin(), block_off_.end(), i0) - block_off_.begin()) - 1;
        for (size_t i = i0; i < i1; ++b) {
            const NetworkProtocol* u = blocks[b]->update.data() + (i - block_off_[b]);
            for (const size_t e = std::min(i1, block_off_[b + 1]); i < e; ++i, ++u) {
                w_uid_[i] = jg_guid{u->uid.lo, u->uid.hi};
                w_type_[i] = u->syncMsgType == NetworkProtocol::CRDTMsg ? 1 : 0;
                w_seq_[i] = u->seq;
                w_ptr_[i] = reinterpret_cast<const uint8_t*>(u->message.data());
                w_len_[i] = (uint32_t)u->message.size();
            }
        }
    });
    flatten_s_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return jg_commit{n, w_uid_.data(), w_type_.data(), w_seq_.data(), nullptr, nullptr, w_ptr_.data(), w_len_.data()};
}

std::vector<uint64_t> GpuStableStore::apply(const std::vector<const UpdateMessage*>& blocks, SafeUpdateTracker* tracker, bool block_mode) {
    const jg_commit wave = gather_wave(blocks);
    return run_wave(wave, tracker, block_mode);
}

void GpuStableStore::PackCommitted(const std::vector<std::vector<UpdateMessage>>& updates, bool nontemporal) {
    std::vector<const UpdateMessage*> blocks;
    for (const auto& list : updates)
        for (const auto& block : list) blocks.push_back(&block);
    const size_t n = index_blocks(blocks);
    p_off_.resize(n + 1);
    p_off_[0] = 0;
    for (size_t b = 0, i = 0; b < blocks.size(); ++b)
        for (const NetworkProtocol& u : blocks[b]->update) p_off_[i + 1] = p_off_[i] + u.message.size(), ++i;
    const uint64_t nb = p_off_[n];
    if (p_cap_ < nb + 64) {
        if (p_bytes_) check(jg_host_free(p_bytes_));
        p_bytes_ = nullptr;
        void* p = nullptr;
        p_cap_ = nb + nb / 4 + 64;
        check(jg_host_alloc(ctx_, p_cap_, &p));
        p_bytes_ = static_cast<uint8_t*>(p);
    }
    // non-temporal line stores, as a NIC's DMA would leave the buffer: no dirty cache lines for the upload's
    // reads to snoop (plain memcpy here measured the in-place upload at ~41 GB/s instead of 56)
    parallel_ranges(pool(), n, [&](size_t i0, size_t i1, int) {
        if (i0 >= i1) return;
        jg::LineStream out(reinterpret_cast<char*>(p_bytes_), p_off_[i0]);
        size_t b = (size_t)(std::upper_bound(block_off_.begin(), block_off_.end(), i0) - block_off_.begin()) - 1;
        for (size_t i = i0; i < i1; ++b) {
            const NetworkProtocol* u = blocks[b]->update.data() + (i - block_off_[b]);
            for (const size_t e = std::min(i1, block_off_[b + 1]); i < e; ++i, ++u) {
                w_uid_[i] = jg_guid{u->uid.lo, u->uid.hi};
                w_type_[i] = u->syncMsgType == NetworkProtocol::CRDTMsg ? 1 : 0;
                w_seq_[i] = u->seq;
                if (nontemporal) out.put(reinterpret_cast<const char*>(u->message.data()), u->message.size());
                else std::memcpy(p_bytes_ + p_off_[i], u->message.data(), u->message.size());
            }
        }
        if (nontemporal) out.finish();
    });
    p_n_ = n;
}

std::vector<uint64_t> GpuStableStore::ApplyPacked(SafeUpdateTracker* tracker) {
    flush_registrations();
    flush_names();
    flatten_s_ = 0;
    jg_commit wave{p_n_, w_uid_.data(), w_type_.data(), w_seq_.data(), p_off_.data(), p_bytes_, nullptr, nullptr};
    return run_wave(wave, tracker, false);
}

std::vector<uint64_t> GpuStableStore::ApplyArenaStreamed(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker,
                                                         size_t part_msgs, bool nontemporal) {
    flush_registrations();
    flush_names();
    std::vector<const UpdateMessage*> blocks;
    for (const auto& list : updates)
        for (const auto& block : list) blocks.push_back(&block);
    const size_t n = index_blocks(blocks);
    flatten_s_ = 0;
    last_msgs_ = n;
    if (w_done_.size() < n) w_done_.resize(n + n / 4);
    if (n == 0) return ApplyCommitted(updates, tracker);
    p_off_.resize(n + 1);
    p_off_[0] = 0;
    for (size_t b = 0, i = 0; b < blocks.size(); ++b)
        for (const NetworkProtocol& u : blocks[b]->update) p_off_[i + 1] = p_off_[i] + u.message.size(), ++i;
    const uint64_t nb = p_off_[n];
    if (p_cap_ < nb + 64) {
        if (p_bytes_) check(jg_host_free(p_bytes_));
        p_bytes_ = nullptr;
        void* p = nullptr;
        p_cap_ = nb + nb / 4 + 64;
        check(jg_host_alloc(ctx_, p_cap_, &p));
        p_bytes_ = static_cast<uint8_t*>(p);
    }
    static const bool trace = std::getenv("JANUS_TRACE_APPLY") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double tb = trace ? now() : 0;
    check(jg_apply_stream_begin(node_, tracker ? tracker->handle() : nullptr, n, nb));
    double t_copy = 0, t_append = 0;
    size_t n_parts = 0;
    const double t0 = trace ? now() : 0;
    static const size_t copiers = [] {
        const char* e = std::getenv("JANUS_ARENA_COPY_THREADS");
        return e && std::atoi(e) > 0 ? (size_t)std::atoi(e) : SIZE_MAX;
    }();
    std::vector<uint64_t> poff[2];  // the in-flight part's offsets and the next one's
    std::future<int> pending;
    std::string err;
    // parts of whole UpdateMessages, ~part_msgs messages each: the caller's copy of part k + 1 (plain cached copies,
    // what a C# caller's parallel Span.CopyTo does) runs while part k uploads
    for (size_t b0 = 0; b0 < blocks.size();) {
        size_t b1 = b0;
        while (b1 < blocks.size() && (b1 == b0 || block_off_[b1] - block_off_[b0] < part_msgs)) ++b1;
        const size_t i0 = block_off_[b0], i1 = block_off_[b1];
        const double tc = trace ? now() : 0;
        // the copy on `copiers` of the workers (JANUS_ARENA_COPY_THREADS; default all): fewer copiers leave more of the
        // host's memory bandwidth to the part the DMA is reading at the same time
        const size_t m = i1 - i0;
        auto copy_range = [&](size_t a, size_t e) {
            if (a >= e) return;
            a += i0, e += i0;
            jg::LineStream out(reinterpret_cast<char*>(p_bytes_), p_off_[a]);
            size_t b = (size_t)(std::upper_bound(block_off_.begin(), block_off_.end(), a) - block_off_.begin()) - 1;
            for (size_t i = a; i < e; ++b) {
                const NetworkProtocol* u = blocks[b]->update.data() + (i - block_off_[b]);
                for (const size_t f = std::min(e, block_off_[b + 1]); i < f; ++i, ++u) {
                    w_uid_[i] = jg_guid{u->uid.lo, u->uid.hi};
                    w_type_[i] = u->syncMsgType == NetworkProtocol::CRDTMsg ? 1 : 0;
                    w_seq_[i] = u->seq;
                    if (nontemporal) out.put(reinterpret_cast<const char*>(u->message.data()), u->message.size());
                    else std::memcpy(p_bytes_ + p_off_[i], u->message.data(), u->message.size());
                }
            }
            if (nontemporal) out.finish();
        };
        if (copiers >= (size_t)pool().size() || m < 8192) {
            parallel_ranges(pool(), m, [&](size_t a, size_t e, int) { copy_range(a, e); });
        } else {
            pool().run([&](int t) {
                if ((size_t)t < copiers) copy_range(m * t / copiers, m * (t + 1) / copiers);
            });
        }
        const double ta = trace ? now() : 0;
        // the part goes to the library on a helper thread while this thread copies the next part (the previous
        // append has returned first: parts arrive in order)
        if (pending.valid()) {
            const int rc = pending.get();
            if (rc != JG_OK) throw EngineError(rc, err);  // the library closed the stream: nothing applied
        }
        std::vector<uint64_t>& po = poff[n_parts & 1];
        po.resize(i1 - i0 + 1);
        for (size_t i = i0; i <= i1; ++i) po[i - i0] = p_off_[i] - p_off_[i0];
        const jg_commit part{i1 - i0, w_uid_.data() + i0, w_type_.data() + i0, w_seq_.data() + i0, po.data(), p_bytes_ + p_off_[i0], nullptr, nullptr};
        pending = std::async(std::launch::async, [this, part, &err] {
            const int rc = jg_apply_stream_append(node_, &part);
            if (rc != JG_OK) err = last_error();  // the thread's own error message
            return rc;
        });
        if (trace) t_copy += ta - tc, t_append += now() - ta;
        ++n_parts;
        b0 = b1;
    }
    if (pending.valid()) {
        const int rc = pending.get();
        if (rc != JG_OK) throw EngineError(rc, err);
    }
    const double te = trace ? now() : 0;
    uint64_t n_done = 0, at = UINT64_MAX;
    const int rc = jg_apply_stream_end(node_, w_done_.data(), &n_done, &at);
    if (trace)
        std::fprintf(stderr, "ApplyArenaStreamed: begin %.2f ms, %zu parts: copies %.2f ms, append waits %.2f ms, end %.2f ms\n", t0 - tb, n_parts, t_copy,
                     t_append, now() - te);
    const std::string why = rc == JG_OK ? std::string() : last_error();
    jg_node_last_stats(node_, &stats_);
    std::vector<uint64_t> done(w_done_.begin(), w_done_.begin() + (ptrdiff_t)n_done);
    if (rc != JG_OK) {
        if (at == UINT64_MAX) throw EngineError(rc, why);
        throw ApplyError(rc, why, at, std::move(done));
    }
    return done;
}

// The completions straight into the caller's buffer (grown, never shrunk: the first n_done entries are this wave's):
// what a C# caller passing its own reused array to jg_apply_committed pays.  The vector-returning forms copy them
// out of the mirror's buffer into a fresh vector (≈ 0.6–0.9 ms of page faults for C5's 500k completions).
size_t GpuStableStore::run_wave_into(const jg_commit& wave, SafeUpdateTracker* tracker, std::vector<uint64_t>& out) {
    const uint64_t n = wave.n;
    last_msgs_ = n;
    if (out.size() < n) out.resize(n + n / 4);
    uint64_t n_done = 0, at = UINT64_MAX;
    const int rc = jg_apply_committed(node_, tracker ? tracker->handle() : nullptr, &wave, out.data(), &n_done, &at);
    const std::string why = rc == JG_OK ? std::string() : last_error();
    jg_node_last_stats(node_, &stats_);
    if (rc != JG_OK) {
        if (at == UINT64_MAX) throw EngineError(rc, why);
        throw ApplyError(rc, why, at, std::vector<uint64_t>(out.begin(), out.begin() + (ptrdiff_t)n_done));
    }
    return n_done;
}

size_t GpuStableStore::ApplyPackedInto(SafeUpdateTracker* tracker, std::vector<uint64_t>& done) {
    flush_registrations();
    flush_names();
    flatten_s_ = 0;
    jg_commit wave{p_n_, w_uid_.data(), w_type_.data(), w_seq_.data(), p_off_.data(), p_bytes_, nullptr, nullptr};
    return run_wave_into(wave, tracker, done);
}

std::vector<uint64_t> GpuStableStore::run_wave(const jg_commit& wave, SafeUpdateTracker* tracker, bool block_mode) {
    const uint64_t n = wave.n;
    last_msgs_ = n;
    if (!block_mode && w_done_.size() < n) w_done_.resize(n + n / 4);
    uint64_t n_done = 0, at = UINT64_MAX;
    const int rc = block_mode ? jg_apply_block(node_, &wave, &at)
                              : jg_apply_committed(node_, tracker ? tracker->handle() : nullptr, &wave, w_done_.data(), &n_done, &at);
    const std::string why = rc == JG_OK ? std::string() : last_error();
    static const bool trace = std::getenv("JANUS_TRACE_APPLY") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    jg_node_last_stats(node_, &stats_);
    std::vector<uint64_t> done(w_done_.begin(), w_done_.begin() + (ptrdiff_t)n_done);
    if (trace) std::fprintf(stderr, "run_wave: stats + completions %.0f us\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
    // the element ids an OR-Set commit issued join the host tables when something next reads names
    if (rc != JG_OK) {
        if (at == UINT64_MAX) throw EngineError(rc, why);
        throw ApplyError(rc, why, at, std::move(done));  // the prefix before `at` was applied
    }
    return done;
}

std::vector<uint8_t> GpuStableStore::ApplyOps(const std::vector<const ClientOp*>& ops, std::vector<uint64_t>* add_lim, std::vector<uint64_t>* rem_lim,
                                              const KeyRef* const* refs) {
    PreparedOps p = PrepareOps(ops, refs, true);
    return RunOps(p, add_lim, rem_lim);
}

// ApplyOps' host half: every op validated (unless refs are given), the OR-Set ops' element ids interned, the
// engine's arrays built.  Nothing reaches the library but the names pull (materialize).
GpuStableStore::PreparedOps GpuStableStore::PrepareOps(const std::vector<const ClientOp*>& ops, const KeyRef* const* refs, bool materialize) {
    static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double t0 = trace ? now() : 0;
    if (materialize) materialize_names();
    PreparedOps P;
    P.n = ops.size();
    auto& pkey = P.pkey;
    auto& pcol = P.pcol;
    auto& pdelta = P.pdelta;
    auto& pisn = P.pisn;
    auto& oset = P.oset;
    auto& oelem = P.oelem;
    auto& oop = P.oop;
    auto& olo = P.olo;
    auto& ohi = P.ohi;
    auto& oidx = P.oidx;
    std::vector<const KeyRef*> found;
    if (!refs) {
        found.resize(ops.size());
        for (size_t i = 0; i < ops.size(); ++i) {  // validate everything first: no partial application
            const auto it = uids_.find(ops[i]->uid);
            if (it == uids_.end()) throw EngineError(JG_EINVAL, "unknown CRDT uid");
            const KeyRef* kr = &it->second;
            const int hi = kr->type == CrdtType::PNCounter ? 2 : 3;
            if (ops[i]->opId < 1 || ops[i]->opId > hi)
                throw EngineError(JG_EINVAL, kr->type == CrdtType::PNCounter ? "Invalid PNC method name" : "Invalid ORSet method name");
            found[i] = kr;
        }
        refs = found.data();
    }
    pkey.reserve(ops.size()), pcol.reserve(ops.size()), pdelta.reserve(ops.size()), pisn.reserve(ops.size());
    // the OR-Set ops' element ids, interned per set in op order (sets are independent: a large batch by the
    // workers, each taking the sets with set % T == its index; the pending-name entries made first, serially)
    std::vector<uint32_t> oid(ops.size(), 0);
    const bool par = ops.size() >= 4096;
    std::vector<size_t> ors;  // (par) the OR-Set ops, in op order
    if (par) {
        std::vector<PendingNames*> pnp(sets_.size(), nullptr);  // each set's pending-name entry, made once
        const size_t T = (size_t)std::max(1, pool().size());
        std::vector<uint32_t> oset_of;  // (the set of ors[j])
        std::vector<size_t> tat(T + 1, 0);
        for (size_t i = 0; i < ops.size(); ++i)
            if (refs[i]->type == CrdtType::ORSet) {
                ors.push_back(i);
                const uint32_t set = refs[i]->idx;
                oset_of.push_back(set);
                ++tat[set % T + 1];
                if (ops[i]->opId != 2 && !pnp[set]) pnp[set] = &pending_names_[set];
            }
        // each worker's ops (its sets: set % T == its index), op order kept
        for (size_t t = 0; t < T; ++t) tat[t + 1] += tat[t];
        std::vector<uint32_t> tops(ors.size());
        {
            std::vector<size_t> at(tat.begin(), tat.end() - 1);
            for (size_t j = 0; j < ors.size(); ++j) tops[at[oset_of[j] % T]++] = (uint32_t)j;
        }
        std::vector<std::string> err(T);
        parallel_ranges(pool(), T, [&](size_t tb0, size_t te0, int) {
            for (size_t t = tb0; t < te0; ++t)
                try {
                    for (size_t x = tat[t]; x < tat[t + 1]; ++x) {
                        const size_t i = ors[tops[x]];
                        const uint32_t set = oset_of[tops[x]];
                        const ClientOp& op = *ops[i];
                        SetKey& sk = sets_[set];
                        if (op.opId == 3) {
                            sk.elems.clear();
                            sk.indexed = (uint32_t)sk.names.size();  // every id issued so far is dead
                            pnp[set]->cleared = true;
                            pnp[set]->ids.clear();
                        } else if (op.elem) {
                            oid[i] = elem_id_in(sk, op.opId == 1 ? pnp[set] : nullptr, *op.elem, op.opId == 1);
                        } else {
                            oid[i] = JG_NULL_ELEM;
                        }
                    }
                } catch (const std::exception& e) {
                    err[t] = e.what();
                }
        }, 2);
        for (const auto& e : err)
            if (!e.empty()) throw EngineError(JG_ESTATE, e);
        // the OR-Set ops' arrays by the workers (the PN-Counter ops, if any, below)
        const size_t m = ors.size();
        oset.resize(m), oelem.resize(m), oop.resize(m), olo.resize(m), ohi.resize(m), oidx.assign(ors.begin(), ors.end());
        parallel_ranges(pool(), m, [&](size_t b, size_t e, int) {
            for (size_t j = b; j < e; ++j) {
                const size_t i = ors[j];
                const ClientOp& op = *ops[i];
                oset[j] = refs[i]->idx, oelem[j] = oid[i], oop[j] = (uint8_t)op.opId, olo[j] = op.tag.lo, ohi[j] = op.tag.hi;
            }
        });
    }
    for (size_t i = 0; i < ops.size(); ++i) {
        const ClientOp& op = *ops[i];
        const KeyRef& kr = *refs[i];
        if (kr.type == CrdtType::PNCounter) {
            pkey.push_back(kr.idx);
            pcol.push_back(0);
            pdelta.push_back(eb_ == 4 ? (int64_t)(int32_t)op.amount : op.amount);
            pisn.push_back(op.opId == 2 ? 1 : 0);
        } else if (!par) {
            SetKey& sk = sets_[kr.idx];
            oset.push_back(kr.idx);
            // Add interns (first insertion); Remove of an unknown element addresses an id no record
            // carries (Contains is false, ORSet.cs:174); Clear empties the Dictionaries, so elements
            // added afterwards take new, larger ids in their new insertion order (ORSet.cs:192-198)
            // (elem_id_in: the names were materialized by the caller, not once per op — that is a library call)
            uint32_t id = 0;
            if (op.opId != 3 && !op.elem) id = JG_NULL_ELEM;
            else if (op.opId == 1) id = elem_id_in(sk, &pending_names_[kr.idx], *op.elem, true);
            else if (op.opId == 2) id = elem_id_in(sk, nullptr, *op.elem, false);
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
    if (trace) P.prep_ms = now() - t0;
    return P;
}

// ApplyOps' library half: the prepared arrays applied (jg_pnc_apply_ops, jg_orset_apply_ops(_ords)); per op its
// result and, with add_lim / rem_lim, its OR-Set snapshot limits.
std::vector<uint8_t> GpuStableStore::RunOps(PreparedOps& P, std::vector<uint64_t>* add_lim, std::vector<uint64_t>* rem_lim) {
    static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double t1 = trace ? now() : 0;
    std::vector<uint8_t> result(P.n, 1);
    if (!P.pkey.empty()) check(jg_pnc_apply_ops(pnc_, P.pkey.size(), P.pkey.data(), P.pcol.data(), P.pdelta.data(), P.pisn.data()));
    if (!P.oset.empty()) {
        std::vector<uint8_t> r(P.oset.size());
        if (add_lim) {  // and each op's snapshot limits (jg_orset_apply_ops_ords)
            std::vector<uint64_t> al(P.oset.size()), rl(P.oset.size());
            check(jg_orset_apply_ops_ords(orset_, P.oset.size(), P.oset.data(), P.oelem.data(), P.oop.data(), P.olo.data(), P.ohi.data(), r.data(),
                                          al.data(), rl.data()));
            add_lim->assign(P.n, 0);
            rem_lim->assign(P.n, 0);
            for (size_t j = 0; j < P.oidx.size(); ++j) (*add_lim)[P.oidx[j]] = al[j], (*rem_lim)[P.oidx[j]] = rl[j];
        } else {
            check(jg_orset_apply_ops(orset_, P.oset.size(), P.oset.data(), P.oelem.data(), P.oop.data(), P.olo.data(), P.ohi.data(), r.data()));
        }
        for (size_t j = 0; j < P.oidx.size(); ++j) result[P.oidx[j]] = r[j];
    }
    if (trace) std::fprintf(stderr, "ApplyOps(%zu): host prep %.1f ms, device %.1f ms\n", P.n, P.prep_ms, now() - t1);
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

uint8_t* GpuStableStore::pinned_buf(size_t bytes) {
    if (pin_cap_ < bytes) {
        if (pin_buf_) check(jg_host_free(pin_buf_));
        pin_buf_ = nullptr;
        void* p = nullptr;
        pin_cap_ = bytes + bytes / 4 + 4096;
        check(jg_host_alloc(ctx_, pin_cap_, &p));
        pin_buf_ = static_cast<uint8_t*>(p);
    }
    return pin_buf_;
}

uint8_t* GpuStableStore::pinned_aux(size_t bytes) {
    if (pin_aux_cap_ < bytes) {
        if (pin_aux_) check(jg_host_free(pin_aux_));
        pin_aux_ = nullptr;
        void* p = nullptr;
        pin_aux_cap_ = bytes + bytes / 4 + 4096;
        check(jg_host_alloc(ctx_, pin_aux_cap_, &p));
        pin_aux_ = static_cast<uint8_t*>(p);
    }
    return pin_aux_;
}

// jg_pnc_apply_ops_encode over consecutive chunks of ops, into page-locked memory: chunk c's states at cbuf[c] (in
// pinned_buf, or a block of its own when the states outgrow the buffer's guess), their offsets at off + start[c] + c
// (chunk-relative, n_c + 1 of them) and their SHA-256s at sha + 32 start[c]; before(c) first (false: stop there),
// on_chunk(c) after each.  Calls in op
// order give what one call would (each chunk's prefixes start from the rows the chunks before it left).  A chunk
// refused for room (JG_ESTATE: nothing of it applied) goes again into a buffer of the size it reported.
void GpuStableStore::ApplyEncodePNC(const uint32_t* rows, const int64_t* delta, const uint8_t* isn, const std::vector<size_t>& start,
                                    const uint64_t*& off, const uint8_t*& sha, std::vector<const uint8_t*>& cbuf,
                                    const std::function<bool(size_t)>& before, const std::function<void(size_t)>& on_chunk) {
    const size_t K = start.size() - 1, n = start[K];
    for (uint8_t* b : pin_more_) check(jg_host_free(b));
    pin_more_.clear();
    uint8_t* aux = pinned_aux((n + K) * 8 + 32 * n + 64);
    auto* o = reinterpret_cast<uint64_t*>(aux);
    uint8_t* h = aux + (n + K) * 8;
    off = o;
    sha = h;
    cbuf.assign(K, nullptr);
    // JANUS_PNC_STATE_GUESS (bytes per state): a test knob that undersizes the first guess, so the refusal paths
    // below (the first chunk's growth, a later chunk's own block) run
    static const double forced = [] {
        const char* e = std::getenv("JANUS_PNC_STATE_GUESS");
        return e ? std::atof(e) : 0.0;
    }();
    const double per = forced > 0 ? forced : last_pnc_bytes_;
    uint8_t* buf = forced > 0 ? pinned_buf((size_t)(n * per) + 4096) : pinned_buf(std::max<size_t>(pin_cap_, (size_t)(n * (per + 8)) + 4096));
    size_t cap = forced > 0 ? (size_t)(n * per) + 4096 : pin_cap_, base = 0, total = 0;
    for (size_t c = 0; c < K; ++c) {
        if (!before(c)) break;  // (the caller's checks stopped the batch: chunks from here on never reach the store)
        const size_t s0 = start[c], m = start[c + 1] - s0;
        uint64_t* oc = o + s0 + c;
        auto call = [&] { return jg_pnc_apply_ops_encode(pnc_, m, rows + s0, 0, delta + s0, isn + s0, oc, buf + base, cap - base, h + 32 * s0); };
        int rc = call();
        if (rc == JG_ESTATE && oc[m] > cap - base) {
            static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;
            if (trace)
                std::fprintf(stderr, "ApplyEncodePNC: chunk %zu refused (%llu bytes, %zu of room): %s\n", c, (unsigned long long)oc[m], cap - base,
                             c == 0 ? "buffer grown" : "a block of its own");
            if (c == 0) {  // nothing read from the buffer yet: grow it
                buf = pinned_buf(oc[m] + (n - m) * (oc[m] / std::max<size_t>(m, 1) + 8));
                cap = pin_cap_;
            } else {       // earlier chunks live in it: the rest goes to a block of its own
                void* p = nullptr;
                const size_t want = oc[m] + (n - start[c + 1]) * (oc[m] / m + 8) + 4096;
                check(jg_host_alloc(ctx_, want, &p));
                pin_more_.push_back(static_cast<uint8_t*>(p));
                buf = static_cast<uint8_t*>(p);
                cap = want;
            }
            base = 0;
            rc = call();
        }
        check(rc);
        cbuf[c] = buf + base;
        base += (oc[m] + 63) & ~size_t(63);
        total += oc[m];
        on_chunk(c);
    }
    if (n) last_pnc_bytes_ = (double)total / (double)n;
}

const uint8_t* GpuStableStore::EncodePNCRowsRaw(const std::vector<uint32_t>& rows, const std::vector<int64_t>& dp, const std::vector<int64_t>& dn,
                                                std::vector<uint64_t>& off, std::vector<uint8_t>* sha) {
    const size_t n = rows.size();
    off.assign(n + 1, 0);
    // one call into a page-locked buffer sized from the last call (a second only if the states outgrew it)
    size_t guess = std::max<size_t>(pin_cap_, (size_t)(n * (last_pnc_bytes_ + 8)) + 4096);
    uint8_t* buf = pinned_buf(guess);
    if (sha) sha->assign(32 * n, 0);  // each state's SHA-256, hashed on the device as it is encoded
    uint8_t* h = sha ? sha->data() : nullptr;
    int rc = jg_pnc_encode_json_before(pnc_, n, rows.data(), 0, dp.data(), dn.data(), off.data(), buf, pin_cap_, h);
    if (rc == JG_ESTATE && off[n] > pin_cap_) {
        buf = pinned_buf(off[n]);
        rc = jg_pnc_encode_json_before(pnc_, n, rows.data(), 0, dp.data(), dn.data(), off.data(), buf, pin_cap_, h);
    }
    check(rc);
    if (n) last_pnc_bytes_ = (double)off[n] / (double)n;
    return buf;
}

void GpuStableStore::EncodePNCRowsBefore(const std::vector<uint32_t>& rows, const std::vector<int64_t>& dp, const std::vector<int64_t>& dn,
                                         const std::vector<size_t>& at, std::vector<std::string>& out,
                                         std::vector<std::array<uint8_t, 32>>* sha, std::vector<uint8_t>* has) {
    static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double t0 = trace ? now() : 0;
    flush_registrations();
    const size_t n = rows.size();
    std::vector<uint64_t> off;
    std::vector<uint8_t> h;
    const uint8_t* buf = EncodePNCRowsRaw(rows, dp, dn, off, sha ? &h : nullptr);
    const double t1 = trace ? now() : 0;
    parallel_ranges(pool(), n, [&](size_t b, size_t e, int) {
        for (size_t i = b; i < e; ++i) {
            out[at[i]].assign(reinterpret_cast<const char*>(buf) + off[i], off[i + 1] - off[i]);
            if (!h.empty()) std::memcpy((*sha)[at[i]].data(), h.data() + 32 * i, 32), (*has)[at[i]] = 1;
        }
    });
    if (trace) std::fprintf(stderr, "EncodePNCRowsBefore(%zu): encode %.1f ms, strings %.1f ms\n", n, t1 - t0, now() - t1);
}

// ComputeDigests of msgs[first..] from per-payload SHA-256s: the ones not given (has[i] = 0: states queued by an earlier
// call) hashed here, then the second level in one call (jg_update_digests_of).
void GpuStableStore::DigestsOf(std::vector<UpdateMessage>& msgs, size_t first, std::vector<std::array<uint8_t, 32>>& sha,
                               const std::vector<uint8_t>& has) {
    if (first >= msgs.size()) return;
    const size_t nu = msgs.size() - first;
    std::vector<uint64_t> upd(nu + 1, 0);
    for (size_t u = 0; u < nu; ++u) upd[u + 1] = upd[u] + msgs[first + u].update.size();
    const size_t nm = upd[nu];
    std::vector<const std::string*> miss;
    std::vector<size_t> miss_at;
    for (size_t u = 0, i = 0; u < nu; ++u)
        for (const auto& np : msgs[first + u].update) {
            if (!has[i]) miss.push_back(&np.message), miss_at.push_back(i);
            ++i;
        }
    if (!miss.empty()) {
        std::vector<uint64_t> off(miss.size() + 1, 0);
        for (size_t k = 0; k < miss.size(); ++k) off[k + 1] = off[k] + miss[k]->size();
        uint8_t* buf = pinned_buf(off.back() + 64);
        for (size_t k = 0; k < miss.size(); ++k) std::memcpy(buf + off[k], miss[k]->data(), miss[k]->size());
        std::vector<uint8_t> h(32 * miss.size());
        check(jg_sha256_batch(ctx_, miss.size(), off.data(), buf, h.data()));
        for (size_t k = 0; k < miss.size(); ++k) std::memcpy(sha[miss_at[k]].data(), h.data() + 32 * k, 32);
    }
    std::vector<uint8_t> dig(32 * nu);
    check(jg_update_digests_of(ctx_, nm, reinterpret_cast<const uint8_t*>(sha.data()), nullptr, nu, upd.data(), dig.data()));
    for (size_t u = 0; u < nu; ++u) std::memcpy(msgs[first + u].digest.data(), dig.data() + 32 * u, 32);
}

// ComputeDigests of msgs[first..] with the payloads gathered into page-locked staging by the workers.
void GpuStableStore::DigestsPinned(std::vector<UpdateMessage>& msgs, size_t first) {
    if (first >= msgs.size()) return;
    const size_t nu = msgs.size() - first;
    std::vector<uint64_t> upd(nu + 1, 0);
    for (size_t u = 0; u < nu; ++u) upd[u + 1] = upd[u] + msgs[first + u].update.size();
    const size_t nm = upd[nu];
    std::vector<uint64_t> off(nm + 1, 0);
    for (size_t u = 0, i = 0; u < nu; ++u)
        for (const auto& np : msgs[first + u].update) off[i + 1] = off[i] + np.message.size(), ++i;
    uint8_t* buf = pinned_buf(off[nm] + 64);
    parallel_ranges(pool(), nu, [&](size_t b, size_t e, int) {
        for (size_t u = b; u < e; ++u) {
            size_t i = upd[u];
            for (const auto& np : msgs[first + u].update) std::memcpy(buf + off[i], np.message.data(), np.message.size()), ++i;
        }
    });
    std::vector<uint8_t> dig(32 * nu);
    check(jg_update_digests(ctx_, nm, off.data(), buf, nullptr, nu, upd.data(), nullptr, dig.data()));
    for (size_t u = 0; u < nu; ++u) std::memcpy(msgs[first + u].digest.data(), dig.data() + 32 * u, 32);
}

std::vector<std::string> GpuStableStore::EncodePNCStatesBefore(const std::vector<Guid>& uids, const std::vector<int64_t>& dp,
                                                               const std::vector<int64_t>& dn) {
    flush_registrations();
    std::vector<uint32_t> rows;
    rows.reserve(uids.size());
    for (const Guid& u : uids) rows.push_back(ref(u, CrdtType::PNCounter).idx);
    std::vector<uint64_t> off(rows.size() + 1, 0);
    check(jg_pnc_encode_json_before(pnc_, rows.size(), rows.data(), 0, dp.data(), dn.data(), off.data(), nullptr, 0, nullptr));
    std::string buf(off.back(), '\0');
    check(jg_pnc_encode_json_before(pnc_, rows.size(), rows.data(), 0, dp.data(), dn.data(), off.data(), reinterpret_cast<uint8_t*>(buf.data()),
                                    buf.size(), nullptr));
    std::vector<std::string> out;
    out.reserve(rows.size());
    for (size_t i = 0; i < rows.size(); ++i) out.emplace_back(buf, off[i], off[i + 1] - off[i]);
    return out;
}

std::vector<std::string> GpuStableStore::EncodeORSetStates(const std::vector<Guid>& uids, const std::vector<uint64_t>* add_lim,
                                                           const std::vector<uint64_t>* rem_lim, std::vector<std::array<uint8_t, 32>>* sha) {
    std::vector<uint32_t> sets;
    sets.reserve(uids.size());
    for (const Guid& u : uids) sets.push_back(ref(u, CrdtType::ORSet).idx);
    const size_t n = sets.size();
    std::vector<size_t> at(n);
    for (size_t i = 0; i < n; ++i) at[i] = i;
    std::vector<std::string> out(n);
    std::vector<uint8_t> has;
    if (sha) sha->resize(n), has.resize(n);
    EncodeORSetSets(sets, add_lim, rem_lim, at, out, sha, sha ? &has : nullptr);
    return out;
}

// ORSetMsg.Encode() of sets[i] (at its ord limits when given) into out[at[i]] (and its SHA-256 into (*sha)[at[i]],
// (*has)[at[i]] = 1): one jg_orset_encode_json into a page-locked buffer kept across calls (a second only if the
// states outgrow it), the strings built by the workers
void GpuStableStore::EncodeORSetSets(const std::vector<uint32_t>& sets, const std::vector<uint64_t>* add_lim, const std::vector<uint64_t>* rem_lim,
                                     const std::vector<size_t>& at, std::vector<std::string>& out, std::vector<std::array<uint8_t, 32>>* sha,
                                     std::vector<uint8_t>* has) {
    static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double t0 = trace ? now() : 0;
    flush_names();  // every element this mirror interned is in the engine's element table
    const double t1 = trace ? now() : 0;
    OrEnc e;
    EncodeORSetSetsDevice(sets, add_lim, rem_lim, sha != nullptr, e);
    const double t2 = trace ? now() : 0;
    EncodeORSetSetsPlace(e, at, out, sha, has);
    if (trace)
        std::fprintf(stderr, "EncodeORSetSets(%zu, %.1f MB): names %.1f ms, encode %.1f ms, strings %.1f ms\n", sets.size(), e.off.back() / 1e6,
                     t1 - t0, t2 - t1, now() - t2);
}

// The library half (no workers, nothing of the mirror's tables but the pinned buffer: it may run beside the workers)
void GpuStableStore::EncodeORSetSetsDevice(const std::vector<uint32_t>& sets, const std::vector<uint64_t>* add_lim, const std::vector<uint64_t>* rem_lim,
                                           bool sha, OrEnc& e) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    const double t0 = now();
    const size_t n = sets.size();
    e.off.assign(n + 1, 0);
    const uint64_t* al = add_lim ? add_lim->data() : nullptr;
    const uint64_t* rl = rem_lim ? rem_lim->data() : nullptr;
    uint8_t* buf = pinned_buf(4096);
    e.h.assign(sha ? 32 * n : 0, 0);  // each state's SHA-256, hashed on the device as it is encoded
    uint8_t* hs = sha ? e.h.data() : nullptr;
    int rc = jg_orset_encode_json(orset_, n, sets.data(), al, rl, e.off.data(), buf, pin_cap_, hs);
    if (rc == JG_ESTATE && e.off[n] > pin_cap_) {
        buf = pinned_buf(e.off[n]);
        rc = jg_orset_encode_json(orset_, n, sets.data(), al, rl, e.off.data(), buf, pin_cap_, hs);
    }
    check(rc);
    e.buf = buf;
    e.ms = now() - t0;
}

void GpuStableStore::EncodeORSetSetsPlace(const OrEnc& e, const std::vector<size_t>& at, std::vector<std::string>& out,
                                          std::vector<std::array<uint8_t, 32>>* sha, std::vector<uint8_t>* has) {
    parallel_ranges(pool(), at.size(), [&](size_t b, size_t x, int) {
        for (size_t i = b; i < x; ++i) {
            out[at[i]].assign(reinterpret_cast<const char*>(e.buf) + e.off[i], e.off[i + 1] - e.off[i]);
            if (sha) std::memcpy((*sha)[at[i]].data(), e.h.data() + 32 * i, 32), (*has)[at[i]] = 1;
        }
    });
}

std::vector<uint8_t> GpuStableStore::SubmitClientUpdates(const std::vector<ClientUpdate>& ups, int clientBatchSize,
                                                         std::vector<UpdateMessage>& submitted,
                                                         SafeUpdateTracker& tracker) {
    const size_t n = ups.size();
    static const bool trace = std::getenv("JANUS_TRACE_SUBMIT") != nullptr;  // phase times to stderr
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e3; };
    double tt[6] = {trace ? now() : 0};
    double t_apply = 0, t_enc_p = 0, t_enc_o = 0;
    size_t n_chunks = 0;
    // Round 6: three things overlap.  A helper thread runs the wrappers' checks on the workers (every op's key resolved,
    // read-only), chunk by chunk, while this thread walks the batcher over message identities (serial, nothing
    // committed until the checks pass); each PN-Counter chunk whose checks passed goes to the device on an encoder
    // thread (jg_pnc_apply_ops_encode: per-key prefixes, every op's snapshot encoded, then the ops applied; no
    // workers) while the next chunk is checked and, later, this thread computes the flushes and the tracker adds and
    // builds the messages of the chunks already encoded.  Only the snapshots the batcher keeps become strings.  A
    // failing check still raises with nothing applied or queued, as the serial loop would: chunks already applied
    // are taken back first.
    std::vector<const KeyRef*> kref(n);
    // each op's key as plain arrays: the serial walks below would chase every KeyRef through the uid map's nodes
    std::vector<uint32_t> krow(n);
    std::vector<uint8_t> kpn(n);  // 1: a PN-Counter key
    std::vector<size_t> first_bad(pool().size(), n);
    ensure_uid_index();
    flush_registrations();  // (the helper's encode needs every registered row's columns on the device)
    struct Spec {  // the helper's device results for a PN-Counter-only batch (page-locked, ApplyEncodePNC)
        bool on = false;           // set with checks_done
        size_t done = 0;           // chunks encoded and applied (under hm)
        std::vector<size_t> start; // chunk c = ops [start[c], start[c + 1])
        std::vector<const uint8_t*> cbuf;
        const uint64_t* off = nullptr;
        const uint8_t* sha = nullptr;
        size_t clen = 1;
        std::string_view state(size_t i) const {  // op i's snapshot
            const size_t c = std::min(i / clen, start.size() - 2);
            const uint64_t* o = off + i + c;
            return {reinterpret_cast<const char*>(cbuf[c]) + o[0], (size_t)(o[1] - o[0])};
        }
    } spec;
    std::vector<int64_t> delta(n);  // each op's amount at the store's width, 1: a Decrement (the check pass fills them)
    std::vector<uint8_t> isn(n);
    std::vector<uint8_t> saw_set(pool().size(), 0);
    std::mutex hm;
    std::condition_variable hcv;
    bool checks_done = false;
    size_t bad = n;
    std::exception_ptr herr;
    double t_chk = 0;
    std::vector<double> t_chunk;
    // The batch in chunks (4 for >= 2^18 ops): the checks run chunk by chunk, and a PN-Counter chunk whose checks
    // passed goes to the device (jg_pnc_apply_ops_encode, on the encoder thread) while the next chunk is checked.  A
    // later failing check, or an OR-Set key (the batch then takes the rounds below), stops the encoder, and the
    // chunks it applied are taken back exactly (the adds wrap: the negated amounts restore every cell) before
    // anything raises or proceeds — the serial loop's all-or-nothing.
    const size_t K = n >= (size_t(1) << 18) ? 4 : 1;
    spec.clen = std::max<size_t>(1, (n + K - 1) / K);
    for (size_t c = 0; c <= K; ++c) spec.start.push_back(std::min(n, c * spec.clen));
    size_t checked = 0;  // chunks checked and all PN-Counter (under hm)
    bool stop = false;   // no further chunk goes to the device (under hm)
    std::thread encoder;
    std::thread helper([&] {
        try {
            bool any_set = false, enc_started = false;
            size_t b = n;
            // JANUS_SUBMIT_LOCKSTEP (tests): chunk c is checked only once the encoder applied chunk c - 1, so a failing
            // check in a later chunk always meets applied chunks and the take-back runs
            static const bool lockstep = std::getenv("JANUS_SUBMIT_LOCKSTEP") != nullptr;
            for (size_t c = 0; c < K && b == n; ++c) {
                if (lockstep && enc_started && c > 0) {
                    std::unique_lock<std::mutex> g(hm);
                    hcv.wait(g, [&] { return spec.done >= c || stop || herr; });
                }
                const size_t c0 = spec.start[c], c1 = spec.start[c + 1];
                parallel_ranges(pool(), c1 - c0, [&](size_t rb, size_t re, int t) {
                    rb += c0, re += c0;
                    constexpr size_t kAhead = 8;  // the slot of op i + kAhead prefetched while op i is looked up
                    for (size_t i = rb; i < std::min(re, rb + kAhead); ++i) __builtin_prefetch(&uidx_[uid_slot0(ups[i].op.uid)]);
                    uint8_t set_seen = 0;  // (one store per range: the workers' flags share a cache line)
                    struct Put {
                        uint8_t& to;
                        uint8_t& v;
                        ~Put() { to |= v; }
                    } put{saw_set[t], set_seen};
                    for (size_t i = rb; i < re; ++i) {
                        if (i + kAhead < re) __builtin_prefetch(&uidx_[uid_slot0(ups[i + kAhead].op.uid)]);
                        const ClientOp& op = ups[i].op;
                        const KeyRef* kr = find_uid(op.uid);
                        kref[i] = kr;
                        if (kr) {
                            const bool pn = kr->type == CrdtType::PNCounter;
                            krow[i] = kr->idx, kpn[i] = pn ? 1 : 0;
                            set_seen |= pn ? 0 : 1;
                            delta[i] = eb_ == 4 ? (int64_t)(int32_t)op.amount : op.amount;
                            isn[i] = op.opId == 2 ? 1 : 0;
                        }
                        if (!kr || op.opId < 1 || op.opId > (kr->type == CrdtType::PNCounter ? 2 : 3)) {
                            first_bad[t] = std::min(first_bad[t], i);
                            return;
                        }
                    }
                }, 0);
                b = *std::min_element(first_bad.begin(), first_bad.end());
                any_set = any_set || std::any_of(saw_set.begin(), saw_set.end(), [](uint8_t x) { return x != 0; });
                {
                    std::lock_guard<std::mutex> g(hm);
                    if (b < n || any_set) stop = true;  // (an OR-Set key: the later chunks are still checked, for the rounds)
                    else checked = c + 1;
                }
                hcv.notify_all();
                if (c == 0 && b == n && !any_set && (enc_started = true))  // the encoder takes the chunks as they pass
                    encoder = std::thread([&] {
                        try {
                            ApplyEncodePNC(krow.data(), delta.data(), isn.data(), spec.start, spec.off, spec.sha, spec.cbuf,
                                           [&](size_t cc) {
                                               std::unique_lock<std::mutex> g(hm);
                                               hcv.wait(g, [&] { return stop || checked > cc || checks_done; });
                                               return !stop && checked > cc;
                                           },
                                           [&](size_t cc) {
                                               {
                                                   std::lock_guard<std::mutex> g(hm);
                                                   spec.done = cc + 1;
                                                   if (trace) t_chunk.push_back(now());
                                               }
                                               hcv.notify_all();
                                           });
                        } catch (...) {
                            std::lock_guard<std::mutex> g(hm);
                            if (!herr) herr = std::current_exception();
                            stop = true;
                            hcv.notify_all();
                        }
                    });
            }
            {
                std::lock_guard<std::mutex> g(hm);
                bad = b;
                spec.on = b == n && n > 0 && !any_set && !stop;
                checks_done = true;
                t_chk = trace ? now() : 0;
            }
            hcv.notify_all();
        } catch (...) {
            std::lock_guard<std::mutex> g(hm);
            if (!herr) herr = std::current_exception();
            stop = true;
            checks_done = true;
            hcv.notify_all();
        }
    });
    struct JoinGuard {  // the helper and the encoder never outlive the call, whatever throws
        std::thread& t;
        ~JoinGuard() {
            if (t.joinable()) t.join();
        }
    } join_enc{encoder}, join_guard{helper};  // (the helper first: it is what starts the encoder)
    // 1. The batcher over message identities (SafeCRDTManager.cs:165-198); states are filled in below.
    //    q entries: message, op index (kOld: queued by an earlier call), and whether SafeCRDT.Update
    //    tracked it.  The batcher's safeUpdateTracker.ContainsKey(msg) (:176) is that flag: a message the
    //    batcher drains has not been submitted yet, so nothing can have removed its entry.
    constexpr int64_t kOld = -1;
    struct QE { int64_t op; uint32_t old; bool tracked; };  // op: a client op of this call, or kOld: oldq[old]
    std::vector<QE> q;
    q.reserve(batch_queue_.size() + n);
    for (size_t k = 0; k < batch_queue_.size(); ++k) q.push_back(QE{kOld, (uint32_t)k, batch_queue_[k].second});
    const uint64_t seq0 = next_seq_;  // op i's message carries seq0 + i (next_seq_++ per Update)
    // (a) serial and light: which queue entries each flush drains, and the one it loses.  A flush drains the whole
    //     queue unless its safe entries reach clientBatchSize first; the entry dequeued then is lost (:175).  The live
    //     queue's safe count is kept as entries arrive and leave, so the entry-by-entry drain runs only in that case.
    struct Range { size_t h0, h1; };
    std::vector<Range> ranges;
    size_t head = 0;  // q[head..] is the live queue
    size_t safe_live = 0;
    for (const QE& e : q) safe_live += e.tracked;
    double last_submit = last_submit_ms_;
    std::vector<uint64_t> t_seq, t_org;  // SafeCRDT.Update's TryAdds, handed to the tracker in one call after the loop
    t_seq.reserve(n);
    t_org.reserve(n);
    const size_t batch = (size_t)std::max(clientBatchSize, 0);
    for (size_t i = 0; i < n; ++i) {
        const bool tracked = ups[i].isSafe && ups[i].origin != 0;  // SafeCRDT.cs:55-56
        if (tracked) t_seq.push_back(seq0 + i), t_org.push_back(ups[i].origin);
        q.push_back(QE{(int64_t)i, 0, tracked});
        safe_live += tracked;
        if (q.size() - head >= batch || ups[i].now_ms - last_submit > 100.0) {
            const size_t h0 = head;
            size_t end = 0, kept = 0;
            if (safe_live < batch) {  // every live entry drains
                kept = q.size() - head;
                end = head = q.size();
                safe_live = 0;
            } else {
                size_t safe_n = 0;
                while (head < q.size()) {
                    const size_t k = head++;                              // TryDequeue first ...
                    safe_live -= q[k].tracked;
                    if (!(safe_n < batch)) break;                         // ... so this one is lost (:175)
                    if (q[k].tracked) ++safe_n;
                    ++kept;
                    end = head;
                }
            }
            if (kept) {
                ranges.push_back(Range{h0, end});
                last_submit = ups[i].now_ms;
            }
        }
    }
    const double t_sim = trace ? now() : 0;
    {
        std::unique_lock<std::mutex> g(hm);
        hcv.wait(g, [&] { return checks_done; });
    }
    if (!spec.on) {
        // the chunks the encoder applied before the checks stopped it, taken back: the adds wrap, so the negated
        // amounts restore every cell exactly — nothing applied, as the serial loop's first throw and the rounds below
        // expect (the helper has set checks_done, so the encoder it may have started exists by now)
        helper.join();
        if (encoder.joinable()) encoder.join();
        const size_t applied = spec.start[spec.done];
        if (applied && !herr) {
            std::vector<uint32_t> zc(applied, 0);
            std::vector<int64_t> neg(applied);
            for (size_t i = 0; i < applied; ++i) neg[i] = (int64_t)(0ull - (uint64_t)delta[i]);
            check(jg_pnc_apply_ops(pnc_, applied, krow.data(), zc.data(), neg.data(), isn.data()));
            if (trace) std::fprintf(stderr, "SubmitClientUpdates: %zu ops of %zu chunks taken back (the checks stopped the batch)\n", applied, spec.done);
        }
        spec.done = 0;
    }
    if (herr || bad < n) {  // nothing applied, nothing queued: the serial loop's first throw
        if (helper.joinable()) helper.join();
        if (encoder.joinable()) encoder.join();
        if (herr) std::rethrow_exception(herr);
        if (!kref[bad]) throw EngineError(JG_EINVAL, "unknown CRDT uid");
        throw EngineError(JG_EINVAL, kref[bad]->type == CrdtType::PNCounter ? "Invalid PNC method name" : "Invalid ORSet method name");
    }
    std::vector<std::pair<NetworkProtocol, bool>> oldq = std::move(batch_queue_);
    batch_queue_.clear();
    next_seq_ += n;
    last_submit_ms_ = last_submit;
    // (b) each flush's messages by the workers (flushes are independent): safe states in queue order, then the
    //     non-safe ones compacted per uid (first appearance keeps its place, the last state wins)
    struct Flush { std::vector<QE> msgs; };
    std::vector<Flush> flushes(ranges.size());
    auto uid_of = [&](const QE& e) -> const Guid& { return e.op == kOld ? oldq[e.old].first.uid : ups[(size_t)e.op].op.uid; };
    parallel_ranges(pool(), ranges.size(), [&](size_t rb, size_t re, int) {
        std::unordered_map<Guid, size_t, GuidHash> pos;  // uid -> slot in `appeared`
        pos.reserve(2 * (size_t)std::max(clientBatchSize, 1));
        std::vector<QE> appeared;
        for (size_t r = rb; r < re; ++r) {
            std::vector<QE>& safe = flushes[r].msgs;
            pos.clear();
            appeared.clear();
            for (size_t k = ranges[r].h0; k < ranges[r].h1; ++k) {
                const QE& e = q[k];
                if (!e.tracked) {
                    auto it = pos.find(uid_of(e));
                    if (it == pos.end()) pos.emplace(uid_of(e), appeared.size()), appeared.push_back(e);
                    else appeared[it->second] = e;
                } else {
                    safe.push_back(e);
                }
            }
            safe.insert(safe.end(), appeared.begin(), appeared.end());
        }
    }, 32);
    const double t_fl = trace ? now() : 0;
    tracker.add_many(t_seq.size(), t_seq.data(), t_org.data());
    if (trace) {
        tt[1] = now();
        std::fprintf(stderr, "SubmitClientUpdates: checks %.1f ms (helper), batcher walk %.1f ms, flushes %.1f ms (after the checks), tracker adds %.1f ms\n",
                     t_chk - tt[0], t_sim - tt[0], t_fl - std::max(t_sim, t_chk), tt[1] - t_fl);
    }
    // 2. Which ops' snapshots are needed: those submitted now or still queued.
    //    (A PN-Counter-only batch encodes every op's: the helper is at it already.)
    std::vector<uint8_t> need(spec.on ? 0 : n, 0);
    if (!spec.on) {
        for (const Flush& f : flushes)
            for (const auto& e : f.msgs)
                if (e.op != kOld) need[(size_t)e.op] = 1;
        for (size_t j = head; j < q.size(); ++j)
            if (q[j].op != kOld) need[(size_t)q[j].op] = 1;
    }
    // 3. Apply the ops in rounds, encode the needed snapshots after each round (on the device).  A PN-Counter
    //    snapshot is the row rewound by the amounts the batch's later ops on that key added to the own column
    //    (jg_pnc_encode_json_before); an OR-Set snapshot is its set's records below the ord limits the apply
    //    reported for its op (jg_orset_apply_ops_ords + jg_orset_encode_json).  Only a Clear of an OR-Set key with a
    //    snapshot needed earlier in the round forces a new round, and only for that key: sets are independent, so an
    //    op's round is the number of such Clears of its own set before it (per-set order kept), and every PN-Counter
    //    op runs in round 0.
    std::vector<uint8_t> result(n, 1);
    if (!spec.on) {  // (the helper ended with the checks; joined above)
        if (herr) std::rethrow_exception(herr);
    }
    // A PN-Counter-only batch is applied and encoded by the helper, chunk by chunk: its snapshots stay in page-locked
    // memory and become the messages' strings where the messages are built (step 4), each flush as soon as the
    // chunks holding its ops are done.
    std::vector<std::string> snap(spec.on ? 0 : n);
    std::vector<std::array<uint8_t, 32>> ssha(spec.on ? 0 : n);  // each snapshot's SHA-256, taken where it was encoded
    std::vector<uint8_t> shas(spec.on ? 0 : n, 0);
    if (spec.on) n_chunks = spec.start.size() - 1;
    std::vector<uint32_t> round(n, 0);
    uint32_t n_rounds = spec.on ? 0 : 1;
    if (!spec.on) {
        std::vector<std::pair<uint32_t, bool>> st(sets_.size());  // OR-Set set -> (its round, a snapshot needed in it)
        for (size_t i = 0; i < n; ++i) {
            if (kpn[i]) continue;
            auto& e = st[krow[i]];
            if (ups[i].op.opId == 3 && e.second) ++e.first, e.second = false;
            round[i] = e.first;
            if (need[i]) e.second = true;
            n_rounds = std::max(n_rounds, e.first + 1);
        }
    }
    // each round's ops in op order, in one pass (a counting sort on the round)
    std::vector<size_t> rbeg(n_rounds + 1, 0), rops(spec.on ? 0 : n);
    if (!spec.on) {
        for (size_t i = 0; i < n; ++i) ++rbeg[round[i] + 1];
        for (uint32_t rd = 0; rd < n_rounds; ++rd) rbeg[rd + 1] += rbeg[rd];
        std::vector<size_t> at(rbeg.begin(), rbeg.end() - 1);
        for (size_t i = 0; i < n; ++i) rops[at[round[i]]++] = i;
    }
    const double t_rounds = trace ? now() : 0;
    double t_prep = 0, t_over = 0;
    // A round's lists (its ops in op order; the OR-Set ops as pointers, no ClientOp copies) and its OR-Set ops
    // prepared (element ids interned in op order, the engine's arrays).  Round r + 1 is prepared on this thread's
    // workers while round r's OR-Set snapshots encode in the library on a helper thread (its device work and D2H):
    // the preparation touches only the mirror's tables, the encode only the library and the page-locked buffer.
    struct Round {
        std::vector<size_t> idx;
        std::vector<const ClientOp*> ops;
        std::vector<const KeyRef*> rr;
        std::vector<size_t> opos, ppos;  // positions in idx of the round's OR-Set / PN-Counter ops
        bool or_snap = false;
        PreparedOps prep;
    };
    auto make_round = [&](uint32_t rd, Round& R) {
        const double tp0 = trace ? now() : 0;
        R.idx.assign(rops.begin() + rbeg[rd], rops.begin() + rbeg[rd + 1]);
        for (size_t j = 0; j < R.idx.size(); ++j) {
            const size_t i = R.idx[j];
            if (kpn[i]) {
                R.ppos.push_back(j);
                continue;
            }
            R.ops.push_back(&ups[i].op);
            R.rr.push_back(kref[i]);
            R.opos.push_back(j);
            R.or_snap |= need[i] != 0;
        }
        if (!R.ops.empty()) R.prep = PrepareOps(R.ops, R.rr.data(), false);
        if (trace) t_prep += now() - tp0;
    };
    if (n_rounds) materialize_names();  // (once: nothing issues names during this call)
    // Round r's OR-Set strings are placed (by the workers) on a helper while round r + 1's ops apply in the library,
    // whose apply runs on threads of its own; the helper is joined before this thread next uses the workers.
    struct Placer {
        OrEnc e;
        std::vector<size_t> at;
        std::thread t;
        std::exception_ptr err;
    };
    std::unique_ptr<Placer> placer;
    struct PlacerGuard {  // (never a joinable thread left to a destructor while an exception unwinds)
        std::unique_ptr<Placer>& p;
        ~PlacerGuard() {
            if (p && p->t.joinable()) p->t.join();
        }
    } placer_guard{placer};
    auto join_placer = [&] {
        if (!placer) return;
        if (placer->t.joinable()) placer->t.join();
        const std::exception_ptr err = placer->err;
        placer.reset();
        if (err) std::rethrow_exception(err);
    };
    Round cur;
    if (n_rounds) make_round(0, cur);
    for (uint32_t rd = 0; rd < n_rounds; ++rd) {
        const std::vector<size_t>& idx = cur.idx;
        std::vector<uint64_t> alim(cur.or_snap ? idx.size() : 0), rlim(cur.or_snap ? idx.size() : 0);
        const double ta = trace ? now() : 0;
        // the round's PN-Counter ops applied, and the rewind of every needed snapshot (the amounts of the key's later
        // ops in the round) computed, in ONE call on the device (jg_pnc_apply_ops_rewind): dp / dn in op order over the
        // needed ops, which is pnc_need's order below
        std::vector<int64_t> dp, dn;
        const std::vector<size_t>& ppos = cur.ppos;
        const std::vector<size_t>& opos = cur.opos;
        if (!ppos.empty()) {
            join_placer();
            std::vector<uint32_t> pkey(ppos.size());
            std::vector<int64_t> pdelta(ppos.size());
            std::vector<uint8_t> pisn(ppos.size()), pneed(ppos.size());
            parallel_ranges(pool(), ppos.size(), [&](size_t b, size_t e, int) {
                for (size_t k = b; k < e; ++k) {
                    const size_t i = idx[ppos[k]];
                    const ClientOp& op = ups[i].op;
                    pkey[k] = krow[i];
                    pdelta[k] = eb_ == 4 ? (int64_t)(int32_t)op.amount : op.amount;
                    pisn[k] = op.opId == 2 ? 1 : 0;
                    pneed[k] = need[i];
                }
            });
            size_t nn = 0;
            for (uint8_t x : pneed) nn += x;
            dp.resize(nn);
            dn.resize(nn);
            check(jg_pnc_apply_ops_rewind(pnc_, pkey.size(), pkey.data(), 0, pdelta.data(), pisn.data(), pneed.data(), dp.data(), dn.data()));
        }
        if (!cur.ops.empty()) {
            std::vector<uint64_t> al, rl;
            const auto r = RunOps(cur.prep, cur.or_snap ? &al : nullptr, cur.or_snap ? &rl : nullptr);
            for (size_t k = 0; k < opos.size(); ++k) {
                result[idx[opos[k]]] = r[k];
                if (cur.or_snap) alim[opos[k]] = al[k], rlim[opos[k]] = rl[k];
            }
        }
        join_placer();  // (the previous round's strings, placed beside this round's library apply)
        const double tb = trace ? now() : 0;
        t_apply += tb - ta;
        ++n_chunks;
        std::vector<size_t> pnc_need, or_need;  // positions in idx
        for (size_t j = 0; j < idx.size(); ++j)
            if (need[idx[j]]) (kpn[idx[j]] ? pnc_need : or_need).push_back(j);
        if (!pnc_need.empty()) {
            std::vector<uint32_t> prow(pnc_need.size());
            std::vector<size_t> at(pnc_need.size());
            for (size_t w = 0; w < pnc_need.size(); ++w) prow[w] = krow[idx[pnc_need[w]]], at[w] = idx[pnc_need[w]];
            const double trw = trace ? now() : 0;
            EncodePNCRowsBefore(prow, dp, dn, at, snap, &ssha, &shas);
            if (trace) std::fprintf(stderr, "SubmitClientUpdates: PN-Counter rows %.1f ms, encode + hashes + strings %.1f ms\n", trw - tb, now() - trw);
        }
        const double tc = trace ? now() : 0;
        t_enc_p += tc - tb;
        // the OR-Set snapshots: names flushed here, the library's encode on the helper while round rd + 1 is prepared
        std::vector<uint32_t> os(or_need.size());
        std::vector<uint64_t> oal(or_need.size()), orl(or_need.size());
        std::vector<size_t> oat(or_need.size());
        for (size_t k = 0; k < or_need.size(); ++k) {
            const size_t j = or_need[k];
            os[k] = krow[idx[j]], oal[k] = alim[j], orl[k] = rlim[j], oat[k] = idx[j];
        }
        OrEnc oe;
        std::exception_ptr eerr;
        std::thread enc;
        if (!or_need.empty()) {
            flush_names();  // every element this mirror interned so far (this round's included) in the engine's table
            enc = std::thread([&] {
                try {
                    EncodeORSetSetsDevice(os, &oal, &orl, true, oe);
                } catch (...) {
                    eerr = std::current_exception();
                }
            });
        }
        struct EncJoin {
            std::thread& t;
            ~EncJoin() {
                if (t.joinable()) t.join();
            }
        } enc_join{enc};
        Round next;
        const double tn = trace ? now() : 0;
        if (rd + 1 < n_rounds) make_round(rd + 1, next);
        const double tn1 = trace ? now() : 0;
        if (enc.joinable()) enc.join();
        if (eerr) std::rethrow_exception(eerr);
        if (trace) {
            t_enc_o += now() - tc - (tn1 - tn);
            t_over += std::min(tn1 - tn, oe.ms);
        }
        if (!or_need.empty()) {
            placer = std::make_unique<Placer>();
            Placer* pl = placer.get();
            pl->e = std::move(oe);
            pl->at = std::move(oat);
            pl->t = std::thread([this, pl, &snap, &ssha, &shas] {
                try {
                    EncodeORSetSetsPlace(pl->e, pl->at, snap, &ssha, &shas);
                } catch (...) {
                    pl->err = std::current_exception();
                }
            });
        }
        cur = std::move(next);
    }
    join_placer();
    if (trace) {
        tt[2] = now();
        std::fprintf(stderr, "SubmitClientUpdates: before the rounds %.1f ms, rounds' op lists + preparation %.1f ms (%.1f ms of it beside the encodes)\n",
                     t_rounds - tt[1], t_prep, t_over);
    }
    // 4. Submitted UpdateMessages and the remaining queue carry the snapshots; each new UpdateMessage
    //    gets its digest (the constructor's ComputeDigest, DAGUpdateMessage.cs:25-30).
    const size_t s0 = submitted.size();
    auto make_np = [&](const QE& e) {  // the queued message with its state (each snapshot goes to one message)
        if (e.op == kOld) return std::move(oldq[e.old].first);
        NetworkProtocol np;
        np.uid = ups[(size_t)e.op].op.uid;
        np.syncMsgType = NetworkProtocol::CRDTMsg;
        np.seq = seq0 + (uint64_t)e.op;
        if (spec.on) {
            np.message.assign(spec.state((size_t)e.op));
        } else {
            np.message = std::move(snap[(size_t)e.op]);
        }
        return np;
    };
    std::vector<size_t> mo(flushes.size() + 1, 0);  // first payload of each new UpdateMessage
    for (size_t f = 0; f < flushes.size(); ++f) mo[f + 1] = mo[f] + flushes[f].msgs.size();
    std::vector<std::array<uint8_t, 32>> msha(mo.back());  // per submitted payload, in UpdateMessage order
    std::vector<uint8_t> mhas(mo.back(), 0);
    submitted.resize(s0 + flushes.size());
    auto build = [&](size_t f0, size_t f1) {  // the UpdateMessages of flushes [f0, f1)
        parallel_ranges(pool(), f1 - f0, [&](size_t fb, size_t fe, int) {
            for (size_t f = f0 + fb; f < f0 + fe; ++f) {
                UpdateMessage& um = submitted[s0 + f];
                um.update.reserve(flushes[f].msgs.size());
                for (size_t j = 0; j < flushes[f].msgs.size(); ++j) {
                    const QE& e = flushes[f].msgs[j];
                    if (e.op != kOld && spec.on) {
                        std::memcpy(msha[mo[f] + j].data(), spec.sha + 32 * (size_t)e.op, 32);
                        mhas[mo[f] + j] = 1;
                    } else if (e.op != kOld && shas[(size_t)e.op]) {
                        msha[mo[f] + j] = ssha[(size_t)e.op], mhas[mo[f] + j] = 1;
                    }
                    um.update.push_back(make_np(e));
                }
            }
        }, 8);
    };
    if (spec.on) {
        const int64_t nold = (int64_t)oldq.size();
        size_t f0 = 0;
        for (size_t c = 1; c < spec.start.size(); ++c) {
            {
                std::unique_lock<std::mutex> g(hm);
                hcv.wait(g, [&] { return spec.done >= c || herr; });
            }
            if (herr) break;  // (a device failure part way: rethrown below)
            const int64_t lim = (int64_t)spec.start[c];  // ops below it are encoded and applied
            size_t f1 = f0;
            while (f1 < flushes.size() && (int64_t)ranges[f1].h1 - 1 - nold < lim) ++f1;
            build(f0, f1);
            f0 = f1;
        }
        helper.join();
        encoder.join();
        if (herr) std::rethrow_exception(herr);
        build(f0, flushes.size());
        if (trace) {
            std::string ct;
            for (double t : t_chunk) ct += " +" + std::to_string(t - tt[0]).substr(0, 5);
            std::fprintf(stderr, "SubmitClientUpdates: helper's chunks (apply + encode + hashes) done at%s ms; all messages built at +%.1f ms\n",
                         ct.c_str(), now() - tt[0]);
        }
    } else {
        build(0, flushes.size());
    }
    if (trace) tt[3] = now();
    DigestsOf(submitted, s0, msha, mhas);
    if (trace) tt[4] = now();
    for (size_t j = head; j < q.size(); ++j) {
        batch_queue_.emplace_back(make_np(q[j]), q[j].tracked);
    }
    if (trace)
        std::fprintf(stderr, "SubmitClientUpdates(%zu ops): checks + batcher %.1f ms, %zu rounds: apply %.1f ms, PN-Counter snapshots %.1f ms, "
                     "OR-Set snapshots %.1f ms (loop %.1f ms), messages %.1f ms, digests %.1f ms, queue %.1f ms\n",
                     n, tt[1] - tt[0], n_chunks, t_apply, t_enc_p, t_enc_o, tt[2] - tt[1], tt[3] - tt[2], tt[4] - tt[3], now() - tt[4]);
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
