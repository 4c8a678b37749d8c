// janus_host.cpp — see janus_host.hpp.
#include "janus_host.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <limits>
#include <memory>
#include <thread>

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
void sort_unique(std::vector<jg_tagrec>& v) {
    std::sort(v.begin(), v.end(), rec_less);
    v.erase(std::unique(v.begin(), v.end(), rec_eq), v.end());
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

uint32_t GpuStableStore::column_nothrow(uint32_t row, const Guid& g, uint32_t hint) {
    Guid* c = &cols_[(size_t)row * R_];
    uint32_t& n = ncols_[row];
    if (hint < n && c[hint] == g) return hint;
    for (uint32_t j = 0; j < n; ++j)
        if (c[j] == g) return j;
    if (n >= R_) return UINT32_MAX;
    c[n] = g;
    return n++;
}

uint32_t GpuStableStore::column(uint32_t row, const Guid& g, uint32_t hint) {
    const uint32_t c = column_nothrow(row, g, hint);
    if (c == UINT32_MAX) throw EngineError(JG_ESTATE, "PNCounter key holds more replicas than the store's columns");
    return c;
}

uint32_t GpuStableStore::find_column(uint32_t row, const Guid& g, uint32_t hint) const {
    const Guid* c = &cols_[(size_t)row * R_];
    const uint32_t n = ncols_[row];
    if (hint < n && c[hint] == g) return hint;
    for (uint32_t j = 0; j < n; ++j)
        if (c[j] == g) return j;
    return UINT32_MAX;
}

uint32_t GpuStableStore::elem_id(SetKey& s, const std::optional<std::string>& e, bool create) {
    if (!e) return JG_NULL_ELEM;
    auto it = s.elems.find(*e);
    if (it != s.elems.end()) return it->second;
    if (!create) return JG_NULL_ELEM - 1;  // never allocated: no records carry it
    const uint32_t id = (uint32_t)s.elems.size();
    if (id >= JG_NULL_ELEM - 1) throw EngineError(JG_ESTATE, "too many elements in one OR-Set");
    s.elems.emplace(*e, id);
    return id;
}

void GpuStableStore::CreateSafeCRDT(const Guid& uid, CrdtType type, const Guid& stableReplicaGuid) {
    if (uids_.find(uid)) return;
    if (type == CrdtType::PNCounter) {
        if (next_row_ >= max_keys_) throw EngineError(JG_ESTATE, "PNCounter store full");
        const uint32_t row = next_row_++;
        if (ncols_.size() <= row) {
            ncols_.resize((size_t)row + 1, 0);
            cols_.resize(((size_t)row + 1) * R_);
        }
        column(row, stableReplicaGuid, 0);  // {self: 0} — the row is zero already
        uids_.insert(uid, KeyRef{type, row});
    } else {
        uids_.insert(uid, KeyRef{type, next_set_++});
        sets_.emplace_back();
    }
}

namespace {
double wall_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

namespace {
// Static contiguous split of [0, n) over up to `threads` workers: fn(begin, end, worker).  Worker t's
// range precedes worker t+1's, so per-worker results concatenated in worker order keep message order.
template <class F> void parallel_ranges(size_t n, int threads, F&& fn) {
    static const size_t min_par = [] {  // below this many messages the wave is decoded inline
        const char* e = std::getenv("JANUS_HOST_PAR_MIN");
        return e ? (size_t)std::strtoull(e, nullptr, 10) : size_t{32768};
    }();
    if (threads <= 1 || n < min_par || n < (size_t)threads) {
        fn(size_t{0}, n, 0);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back([&, t] { fn(n * t / threads, n * (t + 1) / threads, t); });
    fn(size_t{0}, n / threads, 0);
    for (auto& th : pool) th.join();
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

std::vector<uint64_t> GpuStableStore::ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates,
                                                     std::unordered_map<uint64_t, uint64_t>* tracker) {
    const double t0 = wall_s();
    std::vector<const NetworkProtocol*> msgs;
    {
        size_t n_msgs = 0;
        for (const auto& list : updates)
            for (const auto& block : list) n_msgs += block.update.size();
        msgs.reserve(n_msgs);
        for (const auto& list : updates)
            for (const auto& block : list)
                for (const auto& u : block.update) msgs.push_back(&u);
    }
    const size_t n = msgs.size();
    const int T = host_threads();
    phase_s_[0] = wall_s() - t0;
    constexpr uint32_t kSkip = UINT32_MAX, kSet = UINT32_MAX - 1, kBadType = UINT32_MAX - 2;

    // Phase 1 (parallel, read-only): classify every message — PNC row, OR-Set, or skipped (:133-136).
    std::vector<uint32_t> cls(n);
    std::vector<size_t> pnc_count(T, 0), bad(T, SIZE_MAX);
    parallel_ranges(n, T, [&](size_t b, size_t e, int t) {
        size_t cnt = 0;
        for (size_t i = b; i < e; ++i) {
            if (i + 16 < e) __builtin_prefetch(msgs[i + 16]);
            if (i + 8 < e) uids_.prefetch(msgs[i + 8]->uid);
            const NetworkProtocol& u = *msgs[i];
            uint32_t c = kSkip;
            if (u.syncMsgType != NetworkProtocol::ManagerMsg_Create && !u.uid.is_empty()) {
                if (const KeyRef* kr = uids_.find(u.uid)) {
                    if (u.type != kr->type) c = kBadType;  // ORSet.cs:288-291 / the PNCounter cast
                    else if (kr->type == CrdtType::PNCounter) { c = kr->idx; ++cnt; }
                    else c = kSet;
                }
            }
            if (c == kBadType && bad[t] == SIZE_MAX) bad[t] = i;
            cls[i] = c;
        }
        pnc_count[t] = cnt;
    });
    for (int t = 0; t < T; ++t)
        if (bad[t] != SIZE_MAX) throw EngineError(JG_ETYPE, "committed state of the wrong CRDT type for its key");
    phase_s_[1] = wall_s() - t0;

    // Phase 2 (parallel, read-only on the interning): decode PNC states into the SoA batch.  A
    // state naming a replica this row has not seen yet is deferred to phase 3, which appends
    // columns in commit order (first-insertion order, as the stable Dictionary would).
    std::vector<size_t> base(T + 1, 0);
    for (int t = 0; t < T; ++t) base[t + 1] = base[t] + pnc_count[t];
    const size_t n_pnc = base[T];
    const int64_t absent = eb_ == 4 ? (int64_t)std::numeric_limits<int32_t>::min() : std::numeric_limits<int64_t>::min();
    std::unique_ptr<uint32_t[]> rows(new uint32_t[n_pnc ? n_pnc : 1]);
    std::unique_ptr<char[]> Pb(new char[(n_pnc ? n_pnc : 1) * R_ * eb_]), Nb(new char[(n_pnc ? n_pnc : 1) * R_ * eb_]);
    std::vector<std::vector<std::pair<size_t, size_t>>> deferred(T);  // (message, batch position)
    auto put = [&](char* buf, size_t at, int64_t v) {
        if (eb_ == 4) reinterpret_cast<int32_t*>(buf)[at] = (int32_t)v;
        else reinterpret_cast<int64_t*>(buf)[at] = v;
    };
    parallel_ranges(n, T, [&](size_t b, size_t e, int t) {
        size_t p = base[t];
        for (size_t i = b; i < e; ++i) {
            if (i + 16 < e) __builtin_prefetch(msgs[i + 16]);  // software pipeline over the pointer chase
            if (i + 8 < e && cls[i + 8] < kBadType) {
                __builtin_prefetch(&cols_[(size_t)cls[i + 8] * R_]);
                __builtin_prefetch(msgs[i + 8]->pnc.pVector.data());
                __builtin_prefetch(msgs[i + 8]->pnc.nVector.data());
            }
            const uint32_t row = cls[i];
            if (row >= kBadType) continue;
            const NetworkProtocol& u = *msgs[i];
            rows[p] = row;
            for (uint32_t c = 0; c < R_; ++c) { put(Pb.get(), p * R_ + c, absent); put(Nb.get(), p * R_ + c, absent); }
            bool miss = false;
            uint32_t j = 0;
            for (const auto& en : u.pnc.pVector) {
                const uint32_t c = find_column(row, en.first, j++);
                if (c == UINT32_MAX) { miss = true; break; }
                put(Pb.get(), p * R_ + c, en.second);
            }
            j = 0;
            for (const auto& en : u.pnc.nVector) {
                if (miss) break;
                const uint32_t c = find_column(row, en.first, j++);
                if (c == UINT32_MAX) { miss = true; break; }
                put(Nb.get(), p * R_ + c, en.second);
            }
            if (miss) deferred[t].emplace_back(i, p);
            ++p;
        }
    });
    phase_s_[2] = wall_s() - t0;
    // Phase 3 (commit order within each row): states that introduce replicas.  Column order only
    // matters per row, so rows are dealt to workers by row % T and every worker walks the deferred
    // states in commit order, handling its own rows.
    std::vector<std::pair<size_t, size_t>> dlist;
    for (int t = 0; t < T; ++t) dlist.insert(dlist.end(), deferred[t].begin(), deferred[t].end());
    const int T3 = dlist.size() < 4096 ? 1 : T;
    std::vector<uint8_t> full(T3, 0);
    auto run3 = [&](int w) {
        for (const auto& [i, p] : dlist) {
            const uint32_t row = cls[i];
            if ((int)(row % (uint32_t)T3) != w) continue;
            const NetworkProtocol& u = *msgs[i];
            uint32_t j = 0;
            for (const auto& en : u.pnc.pVector) {
                const uint32_t c = column_nothrow(row, en.first, j++);
                if (c == UINT32_MAX) { full[w] = 1; return; }
                put(Pb.get(), p * R_ + c, en.second);
            }
            j = 0;
            for (const auto& en : u.pnc.nVector) {
                const uint32_t c = column_nothrow(row, en.first, j++);
                if (c == UINT32_MAX) { full[w] = 1; return; }
                put(Nb.get(), p * R_ + c, en.second);
            }
        }
    };
    if (T3 == 1) run3(0);
    else {
        std::vector<std::thread> pool;
        for (int w = 1; w < T3; ++w) pool.emplace_back(run3, w);
        run3(0);
        for (auto& th : pool) th.join();
    }
    for (uint8_t f : full)
        if (f) throw EngineError(JG_ESTATE, "PNCounter key holds more replicas than the store's columns");

    phase_s_[3] = wall_s() - t0;
    // OR-Set states and the safe-update tracker, serial in commit order.
    std::vector<jg_tagrec> adds, rems;
    std::vector<uint64_t> completed;
    for (size_t i = 0; i < n; ++i) {
        if (cls[i] == kSkip) continue;
        const NetworkProtocol& u = *msgs[i];
        if (cls[i] == kSet) {
            const KeyRef* kr = uids_.find(u.uid);
            SetKey& s = sets_[kr->idx];
            const uint64_t hi = (uint64_t)kr->idx << 32;
            for (const auto& e : u.orset.addSet) {
                if (e.second.empty()) throw EngineError(JG_ESTATE, "empty add tag set (not produced by ORSet.Add)");
                const uint64_t key = hi | elem_id(s, e.first, true);
                for (const auto& g : e.second) adds.push_back(jg_tagrec{key, g.lo, g.hi});
            }
            for (const auto& e : u.orset.removeSet) {
                const uint64_t key = hi | elem_id(s, e.first, true);
                for (const auto& g : e.second) rems.push_back(jg_tagrec{key, g.lo, g.hi});
            }
            for (const auto& g : u.orset.nullAddGuid) adds.push_back(jg_tagrec{hi | JG_NULL_ELEM, g.lo, g.hi});
            for (const auto& g : u.orset.nullRemoveGuid) rems.push_back(jg_tagrec{hi | JG_NULL_ELEM, g.lo, g.hi});
        }
        if (tracker) {
            auto tr = tracker->find(u.seq);
            if (tr != tracker->end()) { completed.push_back(tr->second); tracker->erase(tr); }
        }
    }
    if (!adds.empty() || !rems.empty()) {
        sort_unique(adds);
        sort_unique(rems);
    }
    const double t1 = wall_s();
    if (n_pnc) check(jg_pnc_merge_rows(pnc_, rows.get(), n_pnc, Pb.get(), Nb.get()));
    if (!adds.empty() || !rems.empty()) check(jg_orset_merge(orset_, adds.data(), adds.size(), rems.data(), rems.size()));
    host_s_ = t1 - t0;
    engine_s_ = wall_s() - t1;
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
            // an element first seen in a Remove gets an id too: its (empty) runs are what Contains sees
            oelem.push_back(op.opId == 3 ? 0u : elem_id(sk, op.elem, true));
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

}  // namespace janus
