// oracle/oracle.hpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's CRDT state-merge path (MSRG/Janus-CRDT, snapshot
// 2025-03-10, C#/.NET 6).  It is the checker for the HIP engine and the "port" CPU baseline in
// bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
// The product library (janus-crdt_amd/) never links or calls anything here.
//
// Parity pinning: the reference cannot run in this image (no dotnet/mono), so
// this restatement is pinned by the reference's own known-answer tests, transcribed one-for-one
// in oracle/test_kat.cpp (PNCounterTests.cs, ORSetTests.cs, ReplicationManagerTests.cs,
// KVStoreTests.cs convergence invariants).  The reference has no golden vectors or fixed seeds.
//
// Data structures follow the reference on purpose (this is also the CPU baseline):
//   Dictionary<Guid,int>          -> OrderedDict<Guid,T>   (hash map + insertion-ordered entries;
//                                    .NET Dictionary enumerates in insertion order while no entry
//                                    is removed, and the reference never removes single entries)
//   HashSet<Guid>                 -> GuidSet (insertion-ordered: entries array + hash index)
//   Dictionary<T,HashSet<Guid>>   -> OrderedDict<std::string, GuidSet>
//   C# int '+=' (unchecked)       -> wrapping add (two's complement)
//   LINQ Sum (checked)            -> exact prefix sums; any prefix outside T's range = overflow
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <initializer_list>
#include <map>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------------------------
// Guid: 16 opaque bytes compared for equality only (reference: System.Guid; ORSet.cs:138,145,149;
// PNCounters.cs:75).  Ordering is only used for canonical export (lexicographic on the two
// little-endian 64-bit words, the same order the GPU store keeps its tag streams in).
// ---------------------------------------------------------------------------------------------
struct Guid {
    uint64_t lo = 0, hi = 0;  // bytes 0..7 -> lo, 8..15 -> hi (little-endian words)
    bool operator==(const Guid& o) const { return lo == o.lo && hi == o.hi; }
    bool operator!=(const Guid& o) const { return !(*this == o); }
    bool operator<(const Guid& o) const { return lo != o.lo ? lo < o.lo : hi < o.hi; }
    bool is_empty() const { return lo == 0 && hi == 0; }  // Guid.Empty
};

inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31; return x;
}

struct GuidHash {
    size_t operator()(const Guid& g) const { return (size_t)mix64(g.lo ^ mix64(g.hi)); }
};

// Deterministic stand-in for Guid.NewGuid(): the reference only relies on uniqueness.
struct GuidGen {
    uint64_t state;
    explicit GuidGen(uint64_t seed = 0x4A414E5553ull) : state(seed) {}
    Guid next() {
        Guid g;
        state += 0x9E3779B97F4A7C15ull; g.lo = mix64(state);
        state += 0x9E3779B97F4A7C15ull; g.hi = mix64(state);
        if (g.is_empty()) g.lo = 1;
        return g;
    }
};

// HashSet<Guid> with .NET's enumeration order.  A .NET 6 HashSet<T> keeps its entries in an array
// filled front to back; Add appends (when the value is new), enumeration walks that array, and only
// Remove (a free list) could reorder later additions — the reference never removes a single tag:
// ORSet.cs only calls Add (:138,145,149), UnionWith (:165,178,259,272,281-282), the copy constructor
// (:182,263,276; HashSet(IEnumerable) of a HashSet copies the entry array, so the order carries over)
// and Clear (:196-197, which resets the array).  System.Text.Json fills a deserialised HashSet with
// Add in array order (duplicates ignored) and serialises it in enumeration order.  So the order is
// first-insertion order, which this class keeps: a vector of entries plus a hash index.
class GuidSet {
  public:
    GuidSet() = default;
    GuidSet(std::initializer_list<Guid> l) { for (const auto& g : l) insert(g); }
    bool insert(const Guid& g) {  // HashSet.Add: false (and no change) when present
        if (!idx_.insert(g).second) return false;
        items_.push_back(g);
        return true;
    }
    size_t count(const Guid& g) const { return idx_.count(g); }
    size_t size() const { return items_.size(); }
    bool empty() const { return items_.empty(); }
    void clear() { items_.clear(); idx_.clear(); }
    std::vector<Guid>::const_iterator begin() const { return items_.begin(); }
    std::vector<Guid>::const_iterator end() const { return items_.end(); }
    const std::vector<Guid>& items() const { return items_; }

  private:
    std::vector<Guid> items_;
    std::unordered_set<Guid, GuidHash> idx_;
};

inline bool SetEquals(const GuidSet& a, const GuidSet& b) {  // HashSet<T>.SetEquals (order-free)
    if (a.size() != b.size()) return false;
    for (const auto& g : a) if (!b.count(g)) return false;
    return true;
}
// HashSet<T>.UnionWith: src's elements in src's enumeration order, each appended if new.
inline void UnionWith(GuidSet& dst, const GuidSet& src) { for (const auto& g : src) dst.insert(g); }

// ---------------------------------------------------------------------------------------------
// OrderedDict: System.Collections.Generic.Dictionary with insertion-order enumeration.
// ---------------------------------------------------------------------------------------------
template <class K, class V, class H = std::hash<K>>
class OrderedDict {
  public:
    using Item = std::pair<K, V>;
    bool TryGetValue(const K& k, V& out) const {
        auto it = idx_.find(k);
        if (it == idx_.end()) { out = V(); return false; }
        out = items_[it->second].second; return true;
    }
    bool ContainsKey(const K& k) const { return idx_.count(k) != 0; }
    V& operator[](const K& k) {  // indexer set: insert at the end if absent
        auto it = idx_.find(k);
        if (it != idx_.end()) return items_[it->second].second;
        idx_.emplace(k, items_.size());
        items_.emplace_back(k, V());
        return items_.back().second;
    }
    const V& at(const K& k) const {
        auto it = idx_.find(k);
        if (it == idx_.end()) throw std::out_of_range("KeyNotFoundException");
        return items_[it->second].second;
    }
    void Clear() { items_.clear(); idx_.clear(); }
    size_t size() const { return items_.size(); }
    void reserve(size_t n) { items_.reserve(n); idx_.reserve(n); }
    typename std::vector<Item>::const_iterator begin() const { return items_.begin(); }
    typename std::vector<Item>::const_iterator end() const { return items_.end(); }
    typename std::vector<Item>::iterator begin() { return items_.begin(); }
    typename std::vector<Item>::iterator end() { return items_.end(); }

  private:
    std::vector<Item> items_;
    std::unordered_map<K, size_t, H> idx_;
};

// ---------------------------------------------------------------------------------------------
// .NET exception kinds surfaced by the path (SURVEY.md §8b B1 "Errors").
// ---------------------------------------------------------------------------------------------
struct OverflowException : std::runtime_error { OverflowException() : std::runtime_error("Arithmetic operation resulted in an overflow.") {} };
struct InvalidOperationException : std::runtime_error { using std::runtime_error::runtime_error; };
struct NotSupportedException : std::runtime_error { using std::runtime_error::runtime_error; };
struct InvalidCastException : std::runtime_error { using std::runtime_error::runtime_error; };

template <class T> inline T wrap_add(T a, T b) {  // C# unchecked '+=' / '-'
    using U = std::make_unsigned_t<T>;
    return (T)((U)a + (U)b);
}
template <class T> inline T wrap_sub(T a, T b) {
    using U = std::make_unsigned_t<T>;
    return (T)((U)a - (U)b);
}

// LINQ Sum over int/long is `checked`: throws on the first partial sum that leaves T's range.
template <class T, class It> inline T checked_sum(It b, It e) {
    T s = 0;
    for (; b != e; ++b) {
        T r;
        if (__builtin_add_overflow(s, b->second, &r)) throw OverflowException();
        s = r;
    }
    return s;
}

// ---------------------------------------------------------------------------------------------
// PN-Counter — MergeSharp/MergeSharp/CRDTs/PNCounters.cs.  T = int32_t is the reference width;
// T = int64_t is the BASELINE.json variant (same algorithm instantiated at long).
// ---------------------------------------------------------------------------------------------
template <class T>
struct PNCounterMsg {  // PNCounters.cs:13-50 (decoded form; JSON codec is §8f F1)
    OrderedDict<Guid, T, GuidHash> pVector, nVector;
};

template <class T>
class PNCounter {
  public:
    // PNCounters.cs:73-81 — fresh replica Guid, P and N hold {self: 0}.
    explicit PNCounter(GuidGen& gen) : replicaIdx_(gen.next()) { P_[replicaIdx_] = 0; N_[replicaIdx_] = 0; }
    explicit PNCounter(const Guid& self) : replicaIdx_(self) { P_[replicaIdx_] = 0; N_[replicaIdx_] = 0; }

    // PNCounters.cs:87-90 — checked Sum(P) - checked Sum(N); the subtraction is unchecked.
    T Get() const { return wrap_sub(checked_sum<T>(P_.begin(), P_.end()), checked_sum<T>(N_.begin(), N_.end())); }

    void Increment(T i) { P_[replicaIdx_] = wrap_add(P_[replicaIdx_], i); }  // PNCounters.cs:97-101
    void Decrement(T i) { N_[replicaIdx_] = wrap_add(N_[replicaIdx_], i); }  // PNCounters.cs:108-112

    // PNCounters.cs:115-118 returns a message aliasing the live dictionaries; every caller encodes
    // it immediately under the object's lock (SafeCRDT.cs:52), so a copy is observationally equal.
    PNCounterMsg<T> GetLastSynchronizedUpdate() const { return PNCounterMsg<T>{P_, N_}; }

    void ApplySynchronizedUpdate(const PNCounterMsg<T>& m) { Merge(m); }  // PNCounters.cs:121-125

    // PNCounters.cs:131-144 — per received entry: local = TryGetValue (absent -> 0), then
    // this[g] = Math.Max(local, v), inserting g if it was absent.
    void Merge(const PNCounterMsg<T>& received) {
        for (const auto& kv : received.pVector) {
            T value; P_.TryGetValue(kv.first, value);
            P_[kv.first] = std::max(value, kv.second);
        }
        for (const auto& kv : received.nVector) {
            T value; N_.TryGetValue(kv.first, value);
            N_[kv.first] = std::max(value, kv.second);
        }
    }

    const Guid& replicaIdx() const { return replicaIdx_; }
    const OrderedDict<Guid, T, GuidHash>& P() const { return P_; }
    const OrderedDict<Guid, T, GuidHash>& N() const { return N_; }
    OrderedDict<Guid, T, GuidHash>& mutP() { return P_; }
    OrderedDict<Guid, T, GuidHash>& mutN() { return N_; }

  private:
    Guid replicaIdx_;
    OrderedDict<Guid, T, GuidHash> P_, N_;
};

// ---------------------------------------------------------------------------------------------
// OR-Set<string?> — MergeSharp/MergeSharp/CRDTs/ORSet.cs.  Elem = nullopt models C# null.
// ---------------------------------------------------------------------------------------------
using Elem = std::optional<std::string>;

struct ORSetMsg {  // ORSet.cs:15-70 (decoded form)
    OrderedDict<std::string, GuidSet> addSet, removeSet;
    GuidSet nullAddGuid, nullRemoveGuid;
};

class ORSet {
  public:
    // ORSet.cs:134-153 — a fresh tag per Add; null goes to nullAddGuid.
    bool Add(const Elem& item, GuidGen& gen) { return AddTag(item, gen.next()); }
    bool AddTag(const Elem& item, const Guid& tag) {
        if (!item) { nullAdd_.insert(tag); return true; }
        if (addSet_.ContainsKey(*item)) addSet_[*item].insert(tag);
        else { GuidSet s; s.insert(tag); addSet_[*item] = std::move(s); }
        return true;
    }

    // ORSet.cs:161-186.
    bool Remove(const Elem& item) {
        if (!item && ListContains(LookupAll(), item)) {
            UnionWith(nullRem_, nullAdd_);
            return true;
        }
        if (!Contains(item)) return false;
        const GuidSet& toRemove = addSet_.at(*item);
        if (removeSet_.ContainsKey(*item)) UnionWith(removeSet_[*item], toRemove);
        else removeSet_[*item] = GuidSet(toRemove);
        return true;
    }

    void Clear() { addSet_.Clear(); removeSet_.Clear(); nullAdd_.clear(); nullRem_.clear(); }  // ORSet.cs:192-198

    // ORSet.cs:204-227 — add-only keys (add order), then keys in both with !SetEquals (add order),
    // then null if !SetEquals(nullRemove, nullAdd).  Union() de-duplicates.
    std::vector<Elem> LookupAll() const {
        std::vector<Elem> out;
        std::unordered_set<std::string> seen;
        for (const auto& kv : addSet_)  // Except(): distinct, not in removeSet.Keys
            if (!removeSet_.ContainsKey(kv.first) && seen.insert(kv.first).second) out.emplace_back(kv.first);
        for (const auto& kv : addSet_) {  // inner join on key, where !SetEquals
            if (!removeSet_.ContainsKey(kv.first)) continue;
            if (!SetEquals(kv.second, removeSet_.at(kv.first)) && seen.insert(kv.first).second) out.emplace_back(kv.first);
        }
        if (!SetEquals(nullRem_, nullAdd_)) out.emplace_back(std::nullopt);
        return out;
    }
    bool Contains(const Elem& item) const { return ListContains(LookupAll(), item); }  // ORSet.cs:234-237
    int Count() const { return (int)LookupAll().size(); }                               // ORSet.cs:103

    // ORSet.cs:253-283 — per received key: UnionWith into the existing set, else a copy.
    void Merge(const ORSetMsg& received) {
        for (const auto& r : received.addSet) {
            if (addSet_.ContainsKey(r.first)) UnionWith(addSet_[r.first], r.second);
            else addSet_[r.first] = GuidSet(r.second);
        }
        for (const auto& r : received.removeSet) {
            if (removeSet_.ContainsKey(r.first)) UnionWith(removeSet_[r.first], r.second);
            else removeSet_[r.first] = GuidSet(r.second);
        }
        UnionWith(nullAdd_, received.nullAddGuid);
        UnionWith(nullRem_, received.nullRemoveGuid);
    }
    void ApplySynchronizedUpdate(const ORSetMsg& m) { Merge(m); }  // ORSet.cs:286-294 (type check is static here)

    ORSetMsg GetLastSynchronizedUpdate() const { return ORSetMsg{addSet_, removeSet_, nullAdd_, nullRem_}; }  // ORSet.cs:305-308

    const OrderedDict<std::string, GuidSet>& addSet() const { return addSet_; }
    const OrderedDict<std::string, GuidSet>& removeSet() const { return removeSet_; }
    const GuidSet& nullAdd() const { return nullAdd_; }
    const GuidSet& nullRem() const { return nullRem_; }
    OrderedDict<std::string, GuidSet>& mutAddSet() { return addSet_; }
    OrderedDict<std::string, GuidSet>& mutRemoveSet() { return removeSet_; }
    GuidSet& mutNullAdd() { return nullAdd_; }
    GuidSet& mutNullRem() { return nullRem_; }

    static bool ListContains(const std::vector<Elem>& v, const Elem& e) {
        for (const auto& x : v) if (x == e) return true;
        return false;
    }

  private:
    OrderedDict<std::string, GuidSet> addSet_, removeSet_;
    GuidSet nullAdd_, nullRem_;
};

// ---------------------------------------------------------------------------------------------
// Safe-CRDT wrappers — BFT-CRDT/SafeCRDTs/{PNCounterWrapper,ORSetWrapper,SafeCRDT}.cs.
// Boxed `object[]` args become a tagged Arg; a wrong tag is the C# InvalidCastException.
// ---------------------------------------------------------------------------------------------
struct Arg {
    enum Kind { Int, Str, Null } kind = Null;
    int64_t i = 0; std::string s;
    static Arg I(int64_t v) { Arg a; a.kind = Int; a.i = v; return a; }
    static Arg S(std::string v) { Arg a; a.kind = Str; a.s = std::move(v); return a; }
    static Arg N() { return Arg(); }
};

struct Result { enum Kind { Bool, Int } kind = Bool; bool b = false; int64_t i = 0; };

enum class CrdtType { PNCounter, ORSet };

// State message carried by NetworkProtocol.message (SyncProtocol.cs:12-62): the decoded state.
struct StateMsg {
    CrdtType type = CrdtType::PNCounter;
    PNCounterMsg<int32_t> pnc;
    ORSetMsg orset;
};

struct NetworkProtocol {  // MergeSharp/MergeSharp/proto/SyncProtocol.cs:12-62
    enum SyncMsgType { ManagerMsg_Create = 0, CRDTMsg = 1 };
    Guid uid; SyncMsgType syncMsgType = CRDTMsg; uint64_t seq = 0;  // seq: object identity for the tracker
    StateMsg message;   // the state, decoded (what Encode was called on)
    std::string bytes;  // `byte[] message`: GetLastSynchronizedUpdate().Encode() (SafeCRDT.cs:49); when
                        // set, ApplyUpdateStable decodes it with the stable copy's codec (oracle/json.hpp)
};

struct UpdateMessage { std::vector<NetworkProtocol> update; };  // DAGConsensus/DAGUpdateMessage.cs:16-55

class PNCounterWrapper {  // PNCounterWrapper.cs
  public:
    explicit PNCounterWrapper(GuidGen& g) : pnc(g) {}
    Result Query() const { Result r; r.kind = Result::Int; r.i = pnc.Get(); return r; }  // :28
    Result Update(int op, const std::vector<Arg>& args) {                             // :33-47
        if (args.empty() || args[0].kind != Arg::Int) throw InvalidCastException("Specified cast is not valid.");
        int32_t arg = (int32_t)args[0].i;  // cast happens BEFORE the switch (:35)
        switch (op) {
            case 1: pnc.Increment(arg); return Result{Result::Bool, true, 0};
            case 2: pnc.Decrement(arg); return Result{Result::Bool, true, 0};
            default: throw InvalidOperationException("Invalid PNC method name");
        }
    }
    PNCounter<int32_t> pnc;
};

class ORSetWrapper {  // ORSetWrapper.cs
  public:
    Result Query(const std::vector<Arg>& args) const {  // :24-28
        Elem e = args.at(0).kind == Arg::Null ? Elem() : Elem(args[0].s);
        return Result{Result::Bool, orset.Contains(e), 0};
    }
    Result Update(int op, const std::vector<Arg>& args, GuidGen& gen) {  // :30-46
        switch (op) {
            case 1: return Result{Result::Bool, orset.Add(ElemOf(args), gen), 0};
            case 2: return Result{Result::Bool, orset.Remove(ElemOf(args)), 0};
            case 3: orset.Clear(); return Result{Result::Bool, true, 0};
            default: throw InvalidOperationException("Invalid ORSet method name");
        }
    }
    static Elem ElemOf(const std::vector<Arg>& a) {
        if (a.empty()) throw std::out_of_range("IndexOutOfRangeException");
        if (a[0].kind == Arg::Null) return Elem();
        if (a[0].kind != Arg::Str) throw InvalidCastException("Specified cast is not valid.");
        return Elem(a[0].s);
    }
    ORSet orset;
};

class SafeCRDTManager;

// SafeCRDT.cs:19-83 — a stable and a prospective copy per key.
class SafeCRDT {
  public:
    SafeCRDT(Guid uid, std::string key, CrdtType t, GuidGen& gen, SafeCRDTManager* sm);
    Result Update(int op, const std::vector<Arg>& args, bool isSafe, uint64_t origin = 0);  // :39-62
    Result QueryStable(const std::vector<Arg>& args = {}) const;                             // :64-70
    Result QueryProspective(const std::vector<Arg>& args = {}) const;                        // :72-78
    void ApplyUpdateStable(const NetworkProtocol& msg);                                      // :80-83
    StateMsg ProspectiveState() const;

    Guid guid; std::string key; CrdtType type;
    std::optional<PNCounterWrapper> pncStable, pncProspective;
    std::optional<ORSetWrapper> orStable, orProspective;
    GuidGen* gen; SafeCRDTManager* sm;
};

// SafeCRDTManager.cs — committed-batch apply loop and the client batcher.
class SafeCRDTManager {
  public:
    explicit SafeCRDTManager(int clientBatchSize = 1, uint64_t seed = 0x4A414E5553ull) : clientBatchSize(clientBatchSize), gen(seed) {}

    SafeCRDT& CreateSafeCRDT(const std::string& key, CrdtType t);                  // :61-76
    SafeCRDT& CreateSafeCRDT(const std::string& key, CrdtType t, const Guid& uid);  // :86-101

    // :109-160 — ordered triple loop; skip create / Guid.Empty; ApplyUpdateStable; notify safe
    // updates in commit order.  The reference runs it on a Task under a SemaphoreSlim(1,1); the
    // oracle runs it inline (the final state is order independent: max and union are ACI).
    void HandleAfterConsensusUpdates(const std::vector<std::vector<UpdateMessage>>& updates);

    // :165-198 — enqueue; flush when >= clientBatchSize or >100 ms since the last submit.
    // Non-safe messages de-duplicate per uid (last wins, first-appearance order of the uid);
    // safe messages stay individual.  Quirk kept: a message dequeued while msgs is full is lost.
    void ActualPropagateSyncMsg(const NetworkProtocol& msg, double now_ms);

    int clientBatchSize;
    GuidGen gen;
    std::map<std::string, SafeCRDT*> safeCRDTs;
    std::unordered_map<Guid, std::unique_ptr<SafeCRDT>, GuidHash> safeCRDTsIndexedByuid;
    std::unordered_map<uint64_t, uint64_t> safeUpdateTracker;  // msg seq -> client origin
    std::deque<NetworkProtocol> clientUpdateBuffer;
    std::vector<UpdateMessage> submitted;  // what DAG.SubmitMessage received (DAG.cs:180-189)
    std::vector<uint64_t> notified;        // safeUpdateCompleteClientNotifier(origin) calls, in order
    double lastSubmittedMs = 0;
    double clock_ms = 0;  // injected DateTime.Now for the 100 ms flush rule (tests set it)
    uint64_t nextSeq = 1;
};

}  // namespace oracle
