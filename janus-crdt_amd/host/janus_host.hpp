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
// Interning: key uid -> row; per-key replica Guid -> column in first-insertion
// order (= the stable Dictionary's enumeration order, so PNCounter.Get's checked Sum sees the same
// prefix order); per-set element string -> elem id (null -> JG_NULL_ELEM).
#pragma once

#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "janus_gpu.h"

namespace janus {

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

// Decoded PNCounterMsg (PNCounters.cs:13-50): entries in the message's dictionary order.
struct PNCounterState {
    std::vector<std::pair<Guid, int64_t>> pVector, nVector;
};
// Decoded ORSetMsg<string?> (ORSet.cs:15-70).
struct ORSetState {
    std::vector<std::pair<std::string, std::vector<Guid>>> addSet, removeSet;
    std::vector<Guid> nullAddGuid, nullRemoveGuid;
};

// NetworkProtocol (MergeSharp/MergeSharp/proto/SyncProtocol.cs:12-62), message already decoded.
struct NetworkProtocol {
    enum SyncMsgType { ManagerMsg_Create = 0, CRDTMsg = 1 };
    Guid uid;
    SyncMsgType syncMsgType = CRDTMsg;
    uint64_t seq = 0;  // identity of the message object for the safe-update tracker
    CrdtType type = CrdtType::PNCounter;
    PNCounterState pnc;
    ORSetState orset;
};
struct UpdateMessage {  // BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:16-55
    std::vector<NetworkProtocol> update;
};

struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
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
    // Guid.Empty (:133-134) and unknown uids (:136), decode every state into one SoA batch per CRDT
    // type, apply each batch with ONE engine call, then report the safe updates that completed, in
    // commit order (:141-142).  `tracker` maps message seq -> client origin; matched entries are
    // removed like ConcurrentDictionary.TryRemove.
    std::vector<uint64_t> ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates,
                                         std::unordered_map<uint64_t, uint64_t>* tracker = nullptr);

    // Wrapper Update, batched: ops run in order (PNC increments commute; OR-Set ops keep their order
    // per set).  Returns each op's bool result.  An unknown op id throws EngineError(JG_EINVAL) (the
    // wrappers' InvalidOperationException) before anything is applied.  A PNC op writes this copy's
    // own replica column (column 0, registered by CreateSafeCRDT).
    std::vector<uint8_t> ApplyOps(const std::vector<ClientOp>& ops);

    // QueryStable: PNCounter.Get (throws EngineError JG_EOVERFLOW where the checked Sum would throw
    // OverflowException) and ORSet.Contains.
    int64_t QueryStablePNC(const Guid& uid);
    bool QueryStableORSet(const Guid& uid, const std::optional<std::string>& elem);

    jg_ctx* ctx() const { return ctx_; }
    static int host_threads();  // decode workers: JANUS_HOST_THREADS, else min(16, hardware threads)
    // Wall time of the last ApplyCommitted: host decode/interning (multi-threaded over the wave's
    // messages, JANUS_HOST_THREADS) vs the engine calls (incl. H2D).
    double last_apply_host_s() const { return host_s_; }
    double last_apply_engine_s() const { return engine_s_; }
    // Cumulative host time at the end of: flatten, classify, parallel decode, deferred columns.
    const double* last_apply_phases_s() const { return phase_s_; }

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
        std::vector<Slot> slots_;
        size_t n_ = 0;
    };
    struct SetKey { std::unordered_map<std::string, uint32_t> elems; };
    // Column of replica g in PNC row `row`; `hint` = its position in the message (messages list
    // replicas in the sender's insertion order, which usually equals ours).  Appends new replicas.
    uint32_t column(uint32_t row, const Guid& g, uint32_t hint);
    uint32_t column_nothrow(uint32_t row, const Guid& g, uint32_t hint);  // UINT32_MAX if the row is full
    uint32_t find_column(uint32_t row, const Guid& g, uint32_t hint) const;  // UINT32_MAX if new
    uint32_t elem_id(SetKey& s, const std::optional<std::string>& e, bool create);
    const KeyRef& ref(const Guid& uid, CrdtType want) const;
    void check(int rc) const;

    jg_ctx* ctx_ = nullptr;
    jg_pnc* pnc_ = nullptr;
    jg_orset* orset_ = nullptr;
    uint32_t max_keys_, R_, eb_;
    uint32_t next_row_ = 0, next_set_ = 0;
    double host_s_ = 0, engine_s_ = 0, phase_s_[4] = {0, 0, 0, 0};
    UidTable uids_;
    std::vector<uint32_t> ncols_;  // per PNC row: replica columns in use
    std::vector<Guid> cols_;       // per PNC row: R replica Guids, in first-insertion order
    std::vector<SetKey> sets_;
};

}  // namespace janus
