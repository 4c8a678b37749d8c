// janus_host.cpp — see janus_host.hpp.
#include "janus_host.hpp"

#include <algorithm>
#include <chrono>
#include <limits>

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
    if (keys_.empty()) return nullptr;
    const size_t mask = keys_.size() - 1;
    for (size_t i = GuidHash()(g) & mask;; i = (i + 1) & mask) {
        if (!used_[i]) return nullptr;
        if (keys_[i] == g) return &vals_[i];
    }
}

bool GpuStableStore::UidTable::insert(const Guid& g, KeyRef v) {
    if ((n_ + 1) * 2 > keys_.size()) grow();
    const size_t mask = keys_.size() - 1;
    for (size_t i = GuidHash()(g) & mask;; i = (i + 1) & mask) {
        if (!used_[i]) { used_[i] = 1; keys_[i] = g; vals_[i] = v; ++n_; return true; }
        if (keys_[i] == g) return false;
    }
}

void GpuStableStore::UidTable::grow() {
    std::vector<Guid> k = std::move(keys_);
    std::vector<KeyRef> v = std::move(vals_);
    std::vector<uint8_t> u = std::move(used_);
    const size_t cap = k.empty() ? 1024 : k.size() * 2;
    keys_.assign(cap, Guid{});
    vals_.assign(cap, KeyRef{CrdtType::PNCounter, 0});
    used_.assign(cap, 0);
    n_ = 0;
    for (size_t i = 0; i < k.size(); ++i)
        if (u[i]) insert(k[i], v[i]);
}

const GpuStableStore::KeyRef& GpuStableStore::ref(const Guid& uid, CrdtType want) const {
    const KeyRef* r = uids_.find(uid);
    if (!r) throw EngineError(JG_EINVAL, "unknown CRDT uid");
    if (r->type != want) throw EngineError(JG_ETYPE, "CRDT uid is of the other type");
    return *r;
}

uint32_t GpuStableStore::column(uint32_t row, const Guid& g, uint32_t hint) {
    Guid* c = &cols_[(size_t)row * R_];
    uint32_t& n = ncols_[row];
    if (hint < n && c[hint] == g) return hint;
    for (uint32_t j = 0; j < n; ++j)
        if (c[j] == g) return j;
    if (n >= R_) throw EngineError(JG_ESTATE, "PNCounter key holds more replicas than the store's columns");
    c[n] = g;
    return n++;
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

std::vector<uint64_t> GpuStableStore::ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates,
                                                     std::unordered_map<uint64_t, uint64_t>* tracker) {
    const double t0 = wall_s();
    std::vector<uint32_t> rows;
    std::vector<int64_t> P64, N64;
    std::vector<int32_t> P32, N32;
    std::vector<jg_tagrec> adds, rems;
    std::vector<uint64_t> completed;
    const int64_t absent = eb_ == 4 ? (int64_t)std::numeric_limits<int32_t>::min() : std::numeric_limits<int64_t>::min();

    size_t n_msgs = 0;
    for (const auto& list : updates)
        for (const auto& block : list) n_msgs += block.update.size();
    rows.reserve(n_msgs);
    if (eb_ == 4) { P32.reserve(n_msgs * R_); N32.reserve(n_msgs * R_); }
    else { P64.reserve(n_msgs * R_); N64.reserve(n_msgs * R_); }

    for (const auto& list : updates)
        for (const auto& block : list)
            for (const auto& u : block.update) {
                if (u.syncMsgType == NetworkProtocol::ManagerMsg_Create || u.uid.is_empty()) continue;
                const KeyRef* kr = uids_.find(u.uid);
                if (!kr) continue;
                if (u.type != kr->type) {  // ORSet.cs:288-291 / the PNCounter cast
                    throw EngineError(JG_ETYPE, "committed state of the wrong CRDT type for its key");
                }
                if (kr->type == CrdtType::PNCounter) {
                    const uint32_t row = kr->idx;
                    const size_t base = rows.size() * R_;
                    rows.push_back(row);
                    if (eb_ == 4) { P32.resize(base + R_, (int32_t)absent); N32.resize(base + R_, (int32_t)absent); }
                    else { P64.resize(base + R_, absent); N64.resize(base + R_, absent); }
                    uint32_t j = 0;
                    for (const auto& e : u.pnc.pVector) {
                        const uint32_t c = column(row, e.first, j++);
                        if (eb_ == 4) P32[base + c] = (int32_t)e.second; else P64[base + c] = e.second;
                    }
                    j = 0;
                    for (const auto& e : u.pnc.nVector) {
                        const uint32_t c = column(row, e.first, j++);
                        if (eb_ == 4) N32[base + c] = (int32_t)e.second; else N64[base + c] = e.second;
                    }
                } else {
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
    if (!rows.empty()) {
        if (eb_ == 4) check(jg_pnc_merge_rows(pnc_, rows.data(), rows.size(), P32.data(), N32.data()));
        else check(jg_pnc_merge_rows(pnc_, rows.data(), rows.size(), P64.data(), N64.data()));
    }
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
