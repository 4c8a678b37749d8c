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
// PropagationMessage bytes (System.Text.Json, SafeCRDT.cs:49).  A committed wave is flattened here into
// the C ABI's jg_commit arrays and applied by ONE jg_apply_committed call (csrc/node.hip): the uid lookup,
// the safe-update tracker and both kinds' decode + merge run inside the library — exactly the call the
// C# HandleAfterConsensusUpdates makes.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "janus_gpu.h"

namespace jg {
class WorkerPool;
}

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

// SafeCRDTManager.safeUpdateTracker (SafeCRDTManager.cs:33, a ConcurrentDictionary<NetworkProtocol,
// (Connection, uint)>): message identity (NetworkProtocol.seq, >= 1) -> client origin, held by the library
// on the device (jg_tracker); the apply loop removes a wave's completed entries there.
class SafeUpdateTracker {
  public:
    explicit SafeUpdateTracker(jg_ctx* ctx);
    ~SafeUpdateTracker();
    SafeUpdateTracker(const SafeUpdateTracker&) = delete;
    SafeUpdateTracker& operator=(const SafeUpdateTracker&) = delete;
    void add(uint64_t seq, uint64_t origin);  // TryAdd (SafeCRDT.cs:55-56)
    void add_many(size_t n, const uint64_t* seq, const uint64_t* origin);  // n TryAdds in one call
    bool contains(uint64_t seq) const;         // ContainsKey
    size_t size() const;
    jg_tracker* handle() const { return t_; }

  private:
    jg_tracker* t_ = nullptr;
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

    // HandleAfterConsensusUpdates (SafeCRDTManager.cs:109-160): the committed wave flattened in commit
    // order into the jg_commit arrays (uid, syncMsgType, identity, payload pointer + length) and applied by
    // ONE jg_apply_committed: unknown uids, ManagerMsg_Create and Guid.Empty skipped (:133-136), every state
    // decoded and merged, the safe updates that completed reported in commit order with their tracker
    // entries removed (:141-142).  A rejected payload throws ApplyError after the prefix was applied.
    std::vector<uint64_t> ApplyCommitted(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker = nullptr);

    // The same apply for a wave a transport received into page-locked memory: PackCommitted
    // lays the wave out as such a receive path would (payloads back to back in jg_host_alloc memory + offsets),
    // ApplyPacked applies it with ONE jg_apply_committed that uploads the payloads in place (the library's
    // `direct` path: no gather into its staging).  Same results as ApplyCommitted on the same wave.
    // nontemporal = false: plain cached copies (what a C# caller's parallel Span.CopyTo does, INTEGRATION.md §3;
    // the upload then snoops the dirty lines)
    void PackCommitted(const std::vector<std::vector<UpdateMessage>>& updates, bool nontemporal = true);
    std::vector<uint64_t> ApplyPacked(SafeUpdateTracker* tracker = nullptr);
    // The same with the completions written into the caller's buffer (grown to the wave's size, reused across
    // calls): returns how many of its first entries this wave completed.
    size_t ApplyPackedInto(SafeUpdateTracker* tracker, std::vector<uint64_t>& done);
    size_t ApplyCommittedInto(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker, std::vector<uint64_t>& done);
    // What a C# caller without page-locked receive buffers does with the streamed apply (jg_apply_stream_*): copy
    // the wave's byte[]s into a jg_host_alloc arena part by part (~part_msgs messages of whole UpdateMessages),
    // handing each part to the library as soon as it is copied, so the copy of the next part overlaps the upload
    // of this one.  Same results as ApplyCommitted.
    // nontemporal: the copy with non-temporal line stores (C#: Avx.StoreAlignedNonTemporal over the byte[]s, INTEGRATION.md
    // §3), so the upload reading part k finds no dirty lines of it in the CPU caches to snoop; false: plain cached copies.
    std::vector<uint64_t> ApplyArenaStreamed(const std::vector<std::vector<UpdateMessage>>& updates, SafeUpdateTracker* tracker = nullptr,
                                             size_t part_msgs = 65536, bool nontemporal = true);

    // ConnectionManager.ReceivedBlock -> ReplicationManager.ReceivedUpdateSyncMsg (BFT-CRDT/Network/
    // DAGConnectionManager.cs:40-50, MergeSharp/MergeSharp/ReplicationManager.cs:290-344): the
    // PROSPECTIVE merge of one received block, one jg_apply_block call.  Creation
    // messages (RM:300-302) and the key-space set (Guid.Empty) are not CRDT states of this store and
    // are skipped; a CRDT state of an unknown uid throws ApplyError(JG_EINVAL) after merging the
    // states before it (KeyNotFoundException at RM:329); a rejected payload throws like ApplyCommitted.
    void ReceivedBlock(const std::vector<UpdateMessage>& block);

    // Wrapper Update, batched: ops run in order (PNC increments commute; OR-Set ops keep their order
    // per set).  Returns each op's bool result.  An unknown op id throws EngineError(JG_EINVAL) (the
    // wrappers' InvalidOperationException) before anything is applied.  A PNC op writes this copy's
    // own replica column (column 0, registered by CreateSafeCRDT).
    // add_lim / rem_lim (optional): per op, the ord limits of its OR-Set's snapshot right after it (jg_orset_apply_ops_ords)
    std::vector<uint8_t> ApplyOps(const std::vector<ClientOp>& ops, std::vector<uint64_t>* add_lim = nullptr, std::vector<uint64_t>* rem_lim = nullptr)
    {
        std::vector<const ClientOp*> p(ops.size());
        for (size_t i = 0; i < ops.size(); ++i) p[i] = &ops[i];
        return ApplyOps(p, add_lim, rem_lim, nullptr);
    }

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
    // ORSet GetLastSynchronizedUpdate().Encode() of OR-Set keys, encoded on the device (jg_orset_encode_json),
    // byte for byte the reference's: Dictionary and HashSet enumeration orders come from the records'
    // arrival ordinals (addSet elements in ascending interned id).  add_lim / rem_lim: each state as of those ord
    // limits (a snapshot before a batch's later ops, ApplyOps' limits).
    std::vector<std::string> EncodeORSetStates(const std::vector<Guid>& uids, const std::vector<uint64_t>* add_lim = nullptr,
                                               const std::vector<uint64_t>* rem_lim = nullptr,
                                               std::vector<std::array<uint8_t, 32>>* sha = nullptr);
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
    // The same as each row stood before its last dp[i] / dn[i] of own-column Increment / Decrement amounts
    // (jg_pnc_encode_json_before): the snapshots of a batch of ops applied at once.
    std::vector<std::string> EncodePNCStatesBefore(const std::vector<Guid>& uids, const std::vector<int64_t>& dp, const std::vector<int64_t>& dn);
    // ORSetWrapper's enumeration / ORSet.LookupAll (ORSet.cs:204-227) in the reference's order.
    std::vector<std::optional<std::string>> QueryStableLookupAll(const Guid& uid);

    // Key-space sharding over `world` GPUs: the shard owning `uid` (jg_shard_of).
    // Every rank registers only the keys it owns and applies the same committed waves: states of keys
    // it does not own are skipped exactly like the reference skips unknown uids (SafeCRDTManager.cs:136),
    // so no state crosses GPUs and the data path needs no collective.
    static uint32_t ShardOf(const Guid& uid, uint32_t world);
    // Declare this store the shard `rank` of `world` (jg_node_set_shard): the library's gather then leaves
    // another shard's states out from the uid alone.
    void SetShard(uint32_t rank, uint32_t world);

    jg_ctx* ctx() const { return ctx_; }
    jg_pnc* pnc() const { return pnc_; }
    uint32_t pnc_row(const Guid& uid) const { return ref(uid, CrdtType::PNCounter).idx; }
    // The library's figures for the last ApplyCommitted / ReceivedBlock (jg_node_last_stats), plus the
    // host mirror's own flatten of the wave into the jg_commit arrays.
    const jg_apply_stats& last_apply_stats() const { return stats_; }
    double last_flatten_s() const { return flatten_s_; }
    uint64_t last_apply_msgs() const { return last_msgs_; }

  private:
    struct KeyRef { CrdtType type; uint32_t idx; };  // idx = PNC row or OR-Set set id (queries, ops)
    // ApplyOps in two halves (SubmitClientUpdates prepares a round's ops while the previous round's snapshots encode)
    struct PreparedOps {
        size_t n = 0;
        std::vector<uint32_t> pkey, pcol;
        std::vector<int64_t> pdelta;
        std::vector<uint8_t> pisn;
        std::vector<uint32_t> oset, oelem;
        std::vector<uint8_t> oop;
        std::vector<uint64_t> olo, ohi;
        std::vector<size_t> oidx;
        double prep_ms = 0;
    };
    PreparedOps PrepareOps(const std::vector<const ClientOp*>& ops, const KeyRef* const* refs, bool materialize);
    std::vector<uint8_t> RunOps(PreparedOps& p, std::vector<uint64_t>* add_lim, std::vector<uint64_t>* rem_lim);
    // ApplyOps over ops held elsewhere (no copies), with the ops' keys already resolved and validated (refs[i] for
    // *ops[i]; NULL: look them up)
    std::vector<uint8_t> ApplyOps(const std::vector<const ClientOp*>& ops, std::vector<uint64_t>* add_lim, std::vector<uint64_t>* rem_lim,
                                  const KeyRef* const* refs);
    // PN-Counter snapshots of rows rewound by (dp, dn) into out[at[i]] (jg_pnc_encode_json_before, one call into
    // page-locked memory, the strings built by the workers)
    // sha (optional): SHA-256 of snapshot i into (*sha)[at[i]], (*has)[at[i]] = 1, hashed from the encoder's page-locked
    // output (jg_sha256_batch) — ComputeDigest's first level without a second copy of the payloads
    void EncodePNCRowsBefore(const std::vector<uint32_t>& rows, const std::vector<int64_t>& dp, const std::vector<int64_t>& dn,
                             const std::vector<size_t>& at, std::vector<std::string>& out,
                             std::vector<std::array<uint8_t, 32>>* sha = nullptr, std::vector<uint8_t>* has = nullptr);
    // the encode alone: states in op order in the returned page-locked buffer at off[i] .. off[i + 1], hashes in *sha
    const uint8_t* EncodePNCRowsRaw(const std::vector<uint32_t>& rows, const std::vector<int64_t>& dp, const std::vector<int64_t>& dn,
                                    std::vector<uint64_t>& off, std::vector<uint8_t>* sha);
    void DigestsPinned(std::vector<UpdateMessage>& msgs, size_t first);  // ComputeDigests through page-locked staging
    // ComputeDigests from per-payload SHA-256s (sha[i]: payload i of msgs[first..] in order; has[i] = 0: hash it here)
    void DigestsOf(std::vector<UpdateMessage>& msgs, size_t first, std::vector<std::array<uint8_t, 32>>& sha, const std::vector<uint8_t>& has);
    uint8_t* pinned_buf(size_t bytes);  // a page-locked buffer of at least `bytes`, kept across calls
    uint8_t* pinned_aux(size_t bytes);  // a second one (offsets, hashes beside pinned_buf's bytes)
    void EncodeORSetSets(const std::vector<uint32_t>& sets, const std::vector<uint64_t>* add_lim, const std::vector<uint64_t>* rem_lim,
                         const std::vector<size_t>& at, std::vector<std::string>& out, std::vector<std::array<uint8_t, 32>>* sha,
                         std::vector<uint8_t>* has);
    // its two halves: the library call (names flushed before it; no workers) and the strings (the workers)
    struct OrEnc {
        std::vector<uint64_t> off;
        std::vector<uint8_t> h;
        const uint8_t* buf = nullptr;
        double ms = 0;
    };
    void EncodeORSetSetsDevice(const std::vector<uint32_t>& sets, const std::vector<uint64_t>* add_lim, const std::vector<uint64_t>* rem_lim,
                               bool sha, OrEnc& e);
    void EncodeORSetSetsPlace(const OrEnc& e, const std::vector<size_t>& at, std::vector<std::string>& out,
                              std::vector<std::array<uint8_t, 32>>* sha, std::vector<uint8_t>* has);
    void ApplyEncodePNC(const uint32_t* rows, const int64_t* delta, const uint8_t* isn, const std::vector<size_t>& start,
                        const uint64_t*& off, const uint8_t*& sha, std::vector<const uint8_t*>& cbuf,
                        const std::function<bool(size_t)>& before, const std::function<void(size_t)>& on_chunk);
    std::vector<uint8_t*> pin_more_;  // ApplyEncodePNC's extra page-locked blocks (states past pinned_buf's guess)
    uint8_t* pin_buf_ = nullptr;
    size_t pin_cap_ = 0;
    uint8_t* pin_aux_ = nullptr;
    size_t pin_aux_cap_ = 0;
    double last_pnc_bytes_ = 400;
    std::unordered_map<Guid, KeyRef, GuidHash> uids_;
    // A flat open-addressing copy of uids_ for the producer path's per-op lookups (one 32-byte slot per probe,
    // prefetched a few ops ahead; the node map costs two dependent cache misses per lookup: 12-20 ms per 1M ops
    // on the GPU box's 16 workers).  Rebuilt when uids_ has grown (uids_ only grows; its values never move).
    struct UidSlot { uint64_t lo, hi; const KeyRef* kr; uint64_t pad; };
    std::vector<UidSlot> uidx_;
    uint64_t uidx_mask_ = 0;
    size_t uidx_n_ = SIZE_MAX;
    void ensure_uid_index();
    uint64_t uid_slot0(const Guid& g) const { return GuidHash{}(g) & uidx_mask_; }
    const KeyRef* find_uid(const Guid& g) const {
        for (uint64_t h = uid_slot0(g);; h = (h + 1) & uidx_mask_) {
            const UidSlot& s = uidx_[h];
            if (!s.kr) return nullptr;
            if (s.lo == g.lo && s.hi == g.hi) return s.kr;
        }
    }
    struct SetKey {
        std::unordered_map<std::string, uint32_t> elems;  // live interning (reset by Clear), indexed lazily:
        uint32_t indexed = 0;                              // names[indexed..] are live but not in elems yet
        std::vector<std::string> names;                   // id -> element, every id ever issued
    };
    uint32_t elem_id(uint32_t set, const std::optional<std::string>& e, bool create);
    struct PendingNames;
    uint32_t elem_id_in(SetKey& s, PendingNames* pn, const std::string& e, bool create);
    // Interning changes made here (ORSet.Add of a new element, Clear) that the engine's element table
    // (the wave path, jg_orset_names_sync) has not seen yet, per set: cleared since the last sync, and
    // the ids issued since then (or since the Clear).
    struct PendingNames { bool cleared = false; std::vector<uint32_t> ids; };
    std::unordered_map<uint32_t, PendingNames> pending_names_;
    void flush_names();
    // Ids the OR-Set waves issued join the SetKey tables on first use by anything that reads names
    // (interning for ops, encode, LookupAll, the name sync): pulled then from the engine's names log
    // (jg_orset_names_since, every wave since the last pull at once) — nothing on the apply path.
    // names_seen_ = the log length these tables cover (the names this mirror synced itself included).
    uint64_t names_seen_ = 0;
    void materialize_names();
    const KeyRef& ref(const Guid& uid, CrdtType want) const;
    void check(int rc) const;
    void flush_registrations();  // pending CreateSafeCRDT registrations -> jg_node_register + jg_pnc_intern
    // ApplyCommitted / ReceivedBlock: flatten the messages into the jg_commit arrays, one library call.
    std::vector<uint64_t> apply(const std::vector<const UpdateMessage*>& blocks, SafeUpdateTracker* tracker, bool block_mode);
    size_t index_blocks(const std::vector<const UpdateMessage*>& blocks);  // block_off_ + the flattened arrays' room
    std::vector<uint64_t> run_wave(const jg_commit& wave, SafeUpdateTracker* tracker, bool block_mode);
    size_t run_wave_into(const jg_commit& wave, SafeUpdateTracker* tracker, std::vector<uint64_t>& out);
    jg_commit gather_wave(const std::vector<const UpdateMessage*>& blocks);
    jg::WorkerPool& pool();  // persistent host workers for the flatten

    jg_ctx* ctx_ = nullptr;
    jg_pnc* pnc_ = nullptr;
    jg_orset* orset_ = nullptr;
    jg_node* node_ = nullptr;
    uint32_t max_keys_, R_, eb_;
    uint32_t next_row_ = 0, next_set_ = 0;
    std::vector<uint32_t> reg_rows_;  // CreateSafeCRDT registrations not yet sent: PNC stable replica Guids
    std::vector<jg_guid> reg_guids_;
    std::vector<jg_guid> reg_uid_;    // ... and the node's uid table entries
    std::vector<uint8_t> reg_type_;
    std::vector<uint32_t> reg_idx_;
    // the flattened wave (kept across waves: a fresh 40 MB per 1M-message wave cost its page faults)
    std::vector<size_t> block_off_;
    std::vector<jg_guid> w_uid_;
    std::vector<uint8_t> w_type_;
    std::vector<uint64_t> w_seq_;
    std::vector<const uint8_t*> w_ptr_;
    std::vector<uint32_t> w_len_;
    std::vector<uint64_t> w_done_;  // the library's completions
    std::vector<uint64_t> p_off_;   // PackCommitted: payload offsets into p_bytes_ (page-locked, jg_host_alloc)
    uint8_t* p_bytes_ = nullptr;
    size_t p_cap_ = 0;
    uint64_t p_n_ = 0;
    jg_apply_stats stats_{};
    double flatten_s_ = 0;
    uint64_t last_msgs_ = 0;
    std::unique_ptr<jg::WorkerPool> pool_;
    std::vector<SetKey> sets_;
    std::vector<std::pair<NetworkProtocol, bool>> batch_queue_;  // clientUpdateBuffer (SafeCRDTManager.cs:167): message, tracked
    double last_submit_ms_ = 0;                 // lastSumittedTime
    uint64_t next_seq_ = 1;                     // message identity for the safe-update tracker
};

}  // namespace janus
