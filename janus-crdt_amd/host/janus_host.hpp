// janus_host.hpp — host-side mirror of the reference's stable-apply surface over the C ABI.
//
// The reference host is C#/.NET (absent from this image), so this C++ layer plays the part the C#
// integration plays: it keeps the reference's names and message shapes and turns
// a DAG-committed wave into ONE batched engine call per CRDT type.
//
//   SafeCRDTManager.CreateSafeCRDT       (BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:61-101)
//   SafeCRDTManager.HandleAfterConsensusUpdates (SafeCRDTManager.cs:109-160)   -> ApplyCommitted
//   SafeCRDT.ApplyUpdateStable / QueryStable    (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:64-83)
//   PNCounterWrapper.Query / ORSetWrapper.Query (PNCounterWrapper.cs:28, ORSetWrapper.cs:24-28)
//
// Interning: key uid -> row (here); per-key replica Guid -> column in first-insertion
// order (= the stable Dictionary's enumeration order, so PNCounter.Get's checked Sum sees the same
// prefix order) in the engine's device replica table (csrc/json.hip); per-set element string -> elem
// id (null -> JG_NULL_ELEM) here.
//
// Committed states arrive as the reference ships them: NetworkProtocol.message = the encoded
// PropagationMessage bytes (System.Text.Json, SafeCRDT.cs:49).  PN-Counter payloads go to the GPU
// undecoded (jg_pnc_merge_json); OR-Set payloads are decoded here (wire.hpp) and merged as records.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "janus_gpu.h"

namespace janus {

class WorkerPool;

struct Guid {
    uint64_t lo = 0, hi = 0;
    bool operator==(const Guid& o) const { return lo == o.lo && hi == o.hi; }
    bool is_empty() const { return lo == 0 && hi == 0; }
};
struct GuidHash {
    size_t operator()(const Guid& g) const {
        uint64_t x = g.lo ^ (g.hi * 0x9E3779B97F4A7C15ull);
        x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
        return (size_t)x;
    }
};

enum class CrdtType { PNCounter, ORSet };

// Decoded ORSetMsg<string?> (ORSet.cs:15-70).
struct ORSetState {
    std::vector<std::pair<std::string, std::vector<Guid>>> addSet, removeSet;
    std::vector<Guid> nullAddGuid, nullRemoveGuid;
};

// NetworkProtocol (MergeSharp/MergeSharp/proto/SyncProtocol.cs:12-62): uid, type, and the encoded
// state (`byte[] message`); the CRDT type of the payload is the type registered for uid (the stable
// copy decodes it with its own DecodePropagationMessage, SafeCRDT.cs:80-83).
struct NetworkProtocol {
    enum SyncMsgType { ManagerMsg_Create = 0, CRDTMsg = 1 };
    Guid uid;
    SyncMsgType syncMsgType = CRDTMsg;
    uint64_t seq = 0;  // identity of the message object for the safe-update tracker
    std::string message;
};
struct UpdateMessage {  // BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:16-55
    std::vector<NetworkProtocol> update;
    std::array<uint8_t, 32> digest{};  // ComputeDigest() (:32-55), filled where the batch is created
};

// `new UpdateMessage(list)` computes its digest (DAGUpdateMessage.cs:25-30): ComputeDigest of every
// message in msgs[first..] in ONE device call (jg_update_digests).
void ComputeDigests(jg_ctx* ctx, std::vector<UpdateMessage>& msgs, size_t first = 0);

// Storage of the apply loop's random-access tables (uid table, safe-update tracker: one random line per
// message each): 2 MiB-aligned and marked for transparent huge pages once at least 2 MiB, so a lookup's
// line does not also miss the TLB (a 1M-key uid table spans 64 MB).
template <class T> struct TableAlloc {
    using value_type = T;
    static constexpr size_t kHuge = size_t(2) << 20;
    TableAlloc() = default;
    template <class U> TableAlloc(const TableAlloc<U>&) {}
    T* allocate(size_t n);
    void deallocate(T* p, size_t n);
    template <class U> bool operator==(const TableAlloc<U>&) const { return true; }
    template <class U> bool operator!=(const TableAlloc<U>&) const { return false; }
};
void* table_alloc(size_t bytes);
void table_free(void* p, size_t bytes);
template <class T> T* TableAlloc<T>::allocate(size_t n) { return static_cast<T*>(table_alloc(n * sizeof(T))); }
template <class T> void TableAlloc<T>::deallocate(T* p, size_t n) { table_free(p, n * sizeof(T)); }

// SafeCRDTManager.safeUpdateTracker (SafeCRDTManager.cs:33, a ConcurrentDictionary<NetworkProtocol,
// (Connection, uint)>): message identity (NetworkProtocol.seq, >= 1) -> client origin.  TryAdd / ContainsKey
// from one thread (the batcher); TryRemove (take) from many threads at once — the apply loop removes a
// wave's completed messages in parallel.  Message identities are issued in order and a committed wave
// carries them roughly in that order, so the entries live in a ring indexed by seq itself (slot =
// seq mod ring size: a wave's claims walk the ring nearly sequentially instead of one random line
// each; a claim empties its slot); a seq whose ring slot holds another live seq goes to an
// open-addressing table (a removed slot there becomes a tombstone, so concurrent takes of different
// keys never move an entry), and the ring doubles once that table holds 1/16 of its size.
class SafeUpdateTracker {
  public:
    SafeUpdateTracker() = default;
    template <class It> SafeUpdateTracker(It b, It e) { for (; b != e; ++b) add(b->first, b->second); }
    SafeUpdateTracker(const SafeUpdateTracker& o) { for (const auto& kv : o.items()) add(kv.first, kv.second); }
    SafeUpdateTracker& operator=(const SafeUpdateTracker& o) {
        if (this != &o) {
            std::vector<std::pair<uint64_t, uint64_t>> kv = o.items();
            clear();
            for (const auto& e : kv) add(e.first, e.second);
        }
        return *this;
    }
    bool add(uint64_t seq, uint64_t origin);          // TryAdd: false if present (seq 0 is not a message)
    bool contains(uint64_t seq) const;
    bool take(uint64_t seq, uint64_t* origin) {       // TryRemove; safe against concurrent take()s
        if (!claim(seq, origin)) return false;
        n_.fetch_sub(1, std::memory_order_relaxed);
        return true;
    }
    // take() without the size update, for parallel sweeps (one shared counter decremented per take
    // serialised 16 workers to ~90 ns a take); settle(k) afterwards with the number claimed
    bool claim(uint64_t seq, uint64_t* origin);
    // false only if seq is certainly not tracked: a plain load of its ring slot (no locked instruction),
    // for callers that batch their claims
    bool maybe(uint64_t seq) const {
        if (used_) return true;
        return !ring_.empty() && ring_[seq & (ring_.size() - 1)].key.load(std::memory_order_relaxed) == seq;
    }
    void settle(size_t k) { n_.fetch_sub(k, std::memory_order_relaxed); }
    void prefetch(uint64_t seq) const {
        if (!ring_.empty()) __builtin_prefetch(&ring_[seq & (ring_.size() - 1)]);
    }
    // the line in exclusive state, for a claim() that will empty it (its CAS then needs no ownership
    // request of its own)
    void prefetch_claim(uint64_t seq) const {
        if (!ring_.empty()) __builtin_prefetch(&ring_[seq & (ring_.size() - 1)], 1);
    }
    size_t size() const { return n_.load(std::memory_order_relaxed); }
    std::vector<std::pair<uint64_t, uint64_t>> items() const;  // live entries (any order)

  private:
    struct Slot { std::atomic<uint64_t> key{0}; uint64_t val = 0; };  // key 0 empty; kTomb removed (table only)
    static constexpr uint64_t kTomb = ~0ull;
    static constexpr size_t kRing0 = size_t(1) << 20;
    static size_t seq_slot(uint64_t x) {
        x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33;
        return (size_t)x;
    }
    void clear() { ring_.clear(); slots_.clear(); n_ = 0; used_ = 0; spill_ = 0; }
    bool table_add(uint64_t seq, uint64_t origin);
    bool table_contains(uint64_t seq) const;
    bool table_claim(uint64_t seq, uint64_t* origin);
    void grow();       // the table: rehash its live entries (tombstones dropped), single-threaded
    void grow_ring();  // twice the ring, every live entry placed again, single-threaded
    std::vector<Slot, TableAlloc<Slot>> ring_;
    std::vector<Slot, TableAlloc<Slot>> slots_;
    std::atomic<size_t> n_{0};
    size_t used_ = 0;   // table: live + tombstones
    size_t spill_ = 0;  // table entries added since the ring was (re)built
};

struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ApplyCommitted stopped at a state its CRDT rejects (JsonException in the reference, whose apply
// Task faults there): every message before `commit_index` was applied and `completed` holds their
// safe-update notifications; nothing at or after it was.
struct ApplyError : EngineError {
    uint64_t commit_index;
    std::vector<uint64_t> completed;
    ApplyError(int c, const std::string& m, uint64_t at, std::vector<uint64_t> done)
        : EngineError(c, m), commit_index(at), completed(std::move(done)) {}
};

// One client operation for PNCounterWrapper.Update / ORSetWrapper.Update
// (BFT-CRDT/SafeCRDTs/PNCounterWrapper.cs:33-47, ORSetWrapper.cs:30-46).
struct ClientOp {
    Guid uid;
    int opId = 0;                     // PNC: 1 Increment, 2 Decrement; ORSet: 1 Add, 2 Remove, 3 Clear
    int64_t amount = 0;               // PNC argument (args[0] as int)
    std::optional<std::string> elem;  // ORSet argument (args[0] as string; nullopt = null)
    Guid tag;                         // ORSet Add: the Guid.NewGuid() drawn for this add
};

// One client update through SafeCRDT.Update (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:39-62).
struct ClientUpdate {
    ClientOp op;
    bool isSafe = false;
    uint64_t origin = 0;  // the client (Connection, id); 0 = default: never tracked (SafeCRDT.cs:55-56)
    double now_ms = 0;    // DateTime.Now when the batcher sees it (the 100 ms flush rule, SafeCRDTManager.cs:170)
};

// One CRDT copy (stable or prospective) of every key of one node, resident on one GPU.
class GpuStableStore {
  public:
    GpuStableStore(int device, uint32_t max_keys, uint32_t replicas, uint32_t elem_bytes);
    ~GpuStableStore();
    GpuStableStore(const GpuStableStore&) = delete;
    GpuStableStore& operator=(const GpuStableStore&) = delete;

    // CreateSafeCRDT: the stable copy is a fresh instance (SafeCRDTManager.cs:68-69, 91-92); a
    // PNCounter's own replica Guid takes column 0 with value 0 (PNCounters.cs:73-81).
    void CreateSafeCRDT(const Guid& uid, CrdtType type, const Guid& stableReplicaGuid = Guid{});

    // HandleAfterConsensusUpdates: walk the committed wave in order, skip ManagerMsg_Create and
    // Guid.Empty (:133-134) and unknown uids (:136), gather the PN-Counter payloads into one pinned
    // staging buffer for ONE jg_pnc_merge_json, decode the OR-Set payloads into one record batch for
    // ONE jg_orset_merge, then report the safe updates that completed, in commit order (:141-142).
    // `tracker` maps message seq -> client origin; matched entries are removed like
    // ConcurrentDictionary.TryRemove.  A rejected payload throws ApplyError after applying the prefix.
    std::vector<uint64_t> ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker = nullptr);

    // ConnectionManager.ReceivedBlock -> ReplicationManager.ReceivedUpdateSyncMsg (BFT-CRDT/Network/
    // DAGConnectionManager.cs:40-50, MergeSharp/MergeSharp/ReplicationManager.cs:290-344): the
    // PROSPECTIVE merge of one received block, one batched engine call per CRDT type.  Creation
    // messages (RM:300-302) and the key-space set (Guid.Empty) are not CRDT states of this store and
    // are skipped; a CRDT state of an unknown uid throws ApplyError(JG_EINVAL) after merging the
    // states before it (KeyNotFoundException at RM:329); a rejected payload throws like ApplyCommitted.
    void ReceivedBlock(const std::vector<UpdateMessage>& block);

    // Wrapper Update, batched: ops run in order (PNC increments commute; OR-Set ops keep their order
    // per set).  Returns each op's bool result.  An unknown op id throws EngineError(JG_EINVAL) (the
    // wrappers' InvalidOperationException) before anything is applied.  A PNC op writes this copy's
    // own replica column (column 0, registered by CreateSafeCRDT).
    std::vector<uint8_t> ApplyOps(const std::vector<ClientOp>& ops);

    // SafeCRDT.Update over a batch of client updates, on this store as the node's PROSPECTIVE copy
    // (SafeCRDT.cs:39-62) followed by the client batcher SafeCRDTManager.ActualPropagateSyncMsg
    // (SafeCRDTManager.cs:165-198): every update is applied in order and its full-state snapshot
    // (GetLastSynchronizedUpdate().Encode()) becomes a NetworkProtocol{uid, CRDTMsg, seq}; safe updates
    // with an origin are tracked (tracker: seq -> origin); the batcher queues them and, when it holds
    // clientBatchSize messages or 100 ms passed since its last submit, drains the queue into one
    // UpdateMessage (appended to `submitted`): safe messages individually in queue order, then the
    // latest message of each non-safe uid in first-appearance order (state compaction), the message
    // dequeued once the safe list is full dropped (:175).  Only the snapshots that survive compaction
    // (or stay queued) are encoded — on the device, after applying the ops up to that point.  Returns
    // each op's bool result; validation failures throw before anything is applied.
    std::vector<uint8_t> SubmitClientUpdates(const std::vector<ClientUpdate>& ups, int clientBatchSize, std::vector<UpdateMessage>& submitted,
                                             SafeUpdateTracker& tracker);
    // ORSet GetLastSynchronizedUpdate().Encode() of OR-Set keys from the device store (jg_orset_read_sets),
    // byte for byte the reference's: Dictionary and HashSet enumeration orders come from the records'
    // arrival ordinals (jg_tagrec.ord; addSet elements in ascending interned id).
    std::vector<std::string> EncodeORSetStates(const std::vector<Guid>& uids);
    // Identity of the next message SubmitClientUpdates creates (NetworkProtocol.seq; the reference keys
    // its safe-update tracker by message object, so identities only need to be unique per process).
    void SetNextMessageSeq(uint64_t seq) { next_seq_ = seq; }

    // QueryStable: PNCounter.Get (throws EngineError JG_EOVERFLOW where the checked Sum would throw
    // OverflowException) and ORSet.Contains.
    int64_t QueryStablePNC(const Guid& uid);
    bool QueryStableORSet(const Guid& uid, const std::optional<std::string>& elem);
    // GetLastSynchronizedUpdate().Encode() of PN-Counter keys, encoded on the device — the payload
    // SafeCRDT.Update ships after a client op (SafeCRDT.cs:49; batch producer).
    std::vector<std::string> EncodePNCStates(const std::vector<Guid>& uids);
    // ORSetWrapper's enumeration / ORSet.LookupAll (ORSet.cs:204-227) in the reference's order.
    std::vector<std::optional<std::string>> QueryStableLookupAll(const Guid& uid);

    // Key-space sharding over `world` GPUs: the shard owning `uid`.  Every rank
    // registers only the keys it owns and applies the same committed waves: states of keys it does
    // not own are skipped exactly like the reference skips unknown uids (SafeCRDTManager.cs:136), so
    // no state crosses GPUs and the data path needs no collective.
    static uint32_t ShardOf(const Guid& uid, uint32_t world) {
        return world <= 1 ? 0u : (uint32_t)((GuidHash()(uid) >> 7) % world);
    }
    // Declare this store the shard `rank` of `world`: the apply loop then skips a state of another
    // shard's uid from the uid alone (ShardOf), without the uid-table and safe-update-tracker lookups —
    // the same skip the table lookup would make, since a shard registers only the uids it owns.  A
    // CreateSafeCRDT of a uid outside the shard turns the shortcut off (the table decides again).
    void SetShard(uint32_t rank, uint32_t world) { shard_rank_ = rank, shard_world_ = world; }

    jg_ctx* ctx() const { return ctx_; }
    jg_pnc* pnc() const { return pnc_; }
    uint32_t pnc_row(const Guid& uid) const { return ref(uid, CrdtType::PNCounter).idx; }
    static int host_threads();  // host workers: JANUS_HOST_THREADS, else min(16, hardware threads)
    // Wall time of the last ApplyCommitted: host work (classify, gather into pinned staging, OR-Set
    // decode; JANUS_HOST_THREADS workers) vs the engine calls (H2D + kernels).
    double last_apply_host_s() const { return host_s_; }
    double last_apply_engine_s() const { return engine_s_; }
    uint64_t last_apply_pnc_bytes() const { return pnc_bytes_; }
    // Cumulative host time at the end of: flatten, classify, gather, OR-Set decode.
    const double* last_apply_phases_s() const { return phase_s_; }
    // OR-Set part of the last ApplyCommitted: element interning, record sort, engine merge call.
    const double* last_apply_orset_phases_s() const { return orset_phase_s_; }

  private:
    struct KeyRef { CrdtType type; uint32_t idx; };  // idx = PNC row or OR-Set set id
    // uid -> KeyRef, open addressing with linear probing: one cache line per lookup on the apply path.
    class UidTable {
      public:
        const KeyRef* find(const Guid& g) const;
        bool insert(const Guid& g, KeyRef v);  // false if present
        void prefetch(const Guid& g) const {
            if (!slots_.empty()) __builtin_prefetch(&slots_[GuidHash()(g) & (slots_.size() - 1)]);
        }
      private:
        struct alignas(32) Slot {  // one cache line holds two slots: a lookup touches one line
            Guid key;
            KeyRef val{CrdtType::PNCounter, 0};
            uint8_t used = 0;
        };
        void grow();
        std::vector<Slot, TableAlloc<Slot>> slots_;
        size_t n_ = 0;
    };
    struct SetKey {
        std::unordered_map<std::string, uint32_t> elems;  // live interning (reset by Clear), indexed lazily:
        uint32_t indexed = 0;                              // names[indexed..] are live but not in elems yet
        std::vector<std::string> names;                   // id -> element, every id ever issued
    };
    uint32_t elem_id(uint32_t set, const std::optional<std::string>& e, bool create);
    // Interning changes made here (ORSet.Add of a new element, Clear) that the engine's element table
    // (the wave path, jg_orset_names_sync) has not seen yet, per set: cleared since the last sync, and
    // the ids issued since then (or since the Clear).
    struct PendingNames { bool cleared = false; std::vector<uint32_t> ids; };
    std::unordered_map<uint32_t, PendingNames> pending_names_;
    void flush_names();
    // Ids the last OR-Set wave issued: copied from the engine right after the commit (the engine keeps
    // only the last commit's), appended to the SetKey tables on first use by anything that reads names
    // (interning for ops, encode, LookupAll, the name sync) — not on the apply path.
    struct WaveNames { std::vector<uint32_t> set, id; std::vector<uint64_t> off; std::vector<uint8_t> bytes; };
    std::vector<WaveNames> wave_names_;
    void take_wave_names();
    void materialize_names();
    const KeyRef& ref(const Guid& uid, CrdtType want) const;
    void check(int rc) const;
    void flush_registrations();             // pending CreateSafeCRDT replica Guids -> jg_pnc_intern
    // The body of ApplyCommitted / ReceivedBlock over the flattened messages (commit order).
    std::vector<uint64_t> apply_msgs(const std::vector<const NetworkProtocol*>& msgs, SafeUpdateTracker* tracker, double t0);
    char* stage(size_t bytes);  // pinned staging of one wave chunk (jg_host_alloc arenas, reused wave after wave)
    WorkerPool& pool();                     // persistent host workers (host_threads())

    jg_ctx* ctx_ = nullptr;
    jg_pnc* pnc_ = nullptr;
    jg_orset* orset_ = nullptr;
    uint32_t max_keys_, R_, eb_;
    uint32_t next_row_ = 0, next_set_ = 0;
    double host_s_ = 0, engine_s_ = 0, phase_s_[4] = {0, 0, 0, 0}, orset_phase_s_[3] = {0, 0, 0};
    uint64_t pnc_bytes_ = 0;
    double avg_msg_bytes_ = 357.0;          // bytes per state message of the last wave (chunk sizing)
    UidTable uids_;
    std::vector<uint32_t> reg_rows_;        // CreateSafeCRDT registrations not yet sent
    std::vector<jg_guid> reg_guids_;
    std::vector<std::pair<char*, size_t>> arenas_;  // pinned staging arenas (base, bytes)
    size_t arena_i_ = 0, arena_off_ = 0;            // carve position of the current wave
    std::vector<uint32_t> cls_, sid_;               // apply_msgs scratch: per message class / set id
    uint32_t shard_rank_ = 0, shard_world_ = 1;
    bool foreign_keys_ = false;  // a uid outside the declared shard was registered
    std::vector<const UpdateMessage*> blocks_;      // ApplyCommitted scratch: the wave's blocks, their
    std::vector<size_t> block_off_;                 //   first message, the messages in commit order
    std::vector<const NetworkProtocol*> msgs_;
    std::vector<uint64_t> where_[2];                //   and per kind, the commit index of its messages
    std::unique_ptr<WorkerPool> pool_;
    std::vector<SetKey> sets_;
    std::vector<NetworkProtocol> batch_queue_;  // clientUpdateBuffer (SafeCRDTManager.cs:167)
    double last_submit_ms_ = 0;                 // lastSumittedTime
    uint64_t next_seq_ = 1;                     // message identity for the safe-update tracker
};

}  // namespace janus
