/* janus_gpu.h — C ABI of the MI355X (gfx950) CRDT state-merge engine.
 *
 * Drop-in boundary for the Janus state-merge hot path.  The C#/.NET host binds
 * these with [DllImport("janusgpu")]; tests bind them with ctypes.  Rules:
 *   - extern "C", cdecl, blittable types only (uint8_t instead of bool, no structs with references);
 *   - every pointer argument is caller-owned HOST memory, read or written only during the call;
 *     device memory is library-owned and freed by the matching *_destroy;
 *   - every call returns JG_OK or an error code; the message is in jg_last_error (thread-local);
 *     no exception or abort crosses the ABI;
 *   - calls are synchronous (return after the work is complete) unless they take `async` != 0,
 *     in which case jg_fence(ctx) waits for them;
 *   - thread-safe per context: every call holds its context's lock for its duration (the context's
 *     scratch buffers and HIP stream are shared by all of its handles), so concurrent callers — the
 *     reference's receiver threads merging prospective copies under lock(crdt), readers querying —
 *     are serialised per context; use one context per thread for parallel device work.  Each context
 *     owns one HIP stream (plus a copy stream for wave uploads) on one device.
 *
 * Reference interfaces each entry point replaces are cited per function (paths relative to the
 * reference root, MSRG/Janus-CRDT @ 2025-03-10).
 */
#ifndef JANUS_GPU_H
#define JANUS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JG_ABI_VERSION 10

/* Error codes.  The C# layer maps them to the exceptions the reference throws (B1 "Errors"). */
#define JG_OK        0
#define JG_EINVAL    1  /* bad argument (ArgumentException / KeyNotFoundException)            */
#define JG_ENOMEM    2  /* device or host allocation failed (OutOfMemoryException)           */
#define JG_EOVERFLOW 3  /* PNCounter.Get checked Sum overflowed (OverflowException)          */
#define JG_ETYPE     4  /* message of the wrong CRDT type (NotSupportedException, ORSet.cs:290) */
#define JG_EHIP      5  /* HIP runtime error                                                  */
#define JG_ESTATE    6  /* precondition broken: unsorted / duplicate records, capacity, timeout */

/* elem id of the C# null element of an ORSet<string?> (ORSet.cs:136-140, nullAddGuid/nullRemoveGuid). */
#define JG_NULL_ELEM 0xFFFFFFFFu

typedef struct jg_ctx jg_ctx;     /* one device + one HIP stream                               */
typedef struct jg_pnc jg_pnc;     /* PN-Counter store: P and N, [n_keys x n_replicas] row-major */
typedef struct jg_rows jg_rows;   /* device-resident batch of received PN-Counter rows          */
typedef struct jg_orset jg_orset; /* OR-Set store: sorted add and tombstone tag records         */

/* One OR-Set tag record: key = (uint64_t)set << 32 | elem, tag = 16 opaque bytes (a C# Guid:
 * tag_lo = bytes 0..7, tag_hi = bytes 8..15, little-endian).  Streams are sorted strictly
 * increasing by (key, tag_lo, tag_hi), unsigned.
 * ord = the record's ARRIVAL ORDINAL, which carries the reference's enumeration order: a HashSet<Guid>
 * enumerates in first-insertion order (ORSet.cs:138-149 Add, :165/178/259/272/281 UnionWith, :182/263/276
 * the copy constructor; nothing removes a single tag), so the tags of one (set, elem) in one stream
 * enumerate in ascending (ord, tag_lo, tag_hi), and a removeSet Dictionary enumerates its elements in
 * ascending (min ord of the element's tombstones, elem) — the element's first insertion.  The addSet
 * Dictionary enumerates in ascending elem id (ids are interned at first insertion).  Only the relative
 * order of ords within one stream of one set is meaningful: the engine renumbers them (order kept) and
 * returns its own values; input ords must be < 2^32.  32 bytes, 8-byte aligned. */
typedef struct jg_tagrec {
    uint64_t key;
    uint64_t tag_lo;
    uint64_t tag_hi;
    uint64_t ord;
} jg_tagrec;

/* ---------------------------------------------------------------------------------------------
 * Context
 * ------------------------------------------------------------------------------------------- */
int jg_abi_version(void);
/* Open device `device` (HIP ordinal) with a private non-blocking stream. */
int jg_open(int device, jg_ctx** out);
int jg_close(jg_ctx* ctx);
/* Copy the calling thread's last error message (NUL-terminated, truncated to n). */
int jg_last_error(char* buf, size_t n);
/* Wait for every async call issued on ctx. */
int jg_fence(jg_ctx* ctx);
/* The context's hipStream_t (for host-side event timing). */
int jg_stream(jg_ctx* ctx, void** hip_stream);

/* ---------------------------------------------------------------------------------------------
 * PN-Counter store — replaces PNCounter's Dictionary<Guid,int> P/N vectors
 * (MergeSharp/MergeSharp/CRDTs/PNCounters.cs:56-153) for a whole keyspace at once.
 * Row = key (host-interned key Guid -> key_idx), column = replica (per-key replica Guid -> column,
 * assigned in first-insertion order so column order = the Dictionary's enumeration order).
 * elem_bytes 4 = the reference's int; 8 = the long variant of BASELINE.json.
 * In RECEIVED rows the most negative value of the width (INT32_MIN / INT64_MIN) means "replica
 * absent from the message": Merge only visits entries the message holds (PNCounters.cs:133-143).
 * ------------------------------------------------------------------------------------------- */
int jg_pnc_create(jg_ctx* ctx, uint64_t n_keys, uint32_t n_replicas, uint32_t elem_bytes, jg_pnc** out);
int jg_pnc_destroy(jg_pnc* pnc);
/* Overwrite rows (key_idx NULL = rows 0..n_rows-1).  Initial load / restore. */
int jg_pnc_write_rows(jg_pnc* pnc, const uint32_t* key_idx, uint64_t n_rows, const void* P, const void* N);
/* Snapshot rows to the host: GetLastSynchronizedUpdate (PNCounters.cs:115-118). */
int jg_pnc_read_rows(jg_pnc* pnc, const uint32_t* key_idx, uint64_t n_rows, void* P, void* N);
/* Merge received states: for each row m and column c whose value is not ABSENT,
 * A[key_idx[m]][c] = max(A[key_idx[m]][c], B[m][c]) for P and N — PNCounter.Merge
 * (PNCounters.cs:131-144) reached through ApplySynchronizedUpdate (:121-125), SafeCRDT.ApplyUpdateStable
 * (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83) and the committed-batch loop
 * (BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:122-146).  key_idx may repeat (the result is the same
 * in any order: max is associative, commutative, idempotent).  key_idx NULL = identity. */
int jg_pnc_merge_rows(jg_pnc* pnc, const uint32_t* key_idx, uint64_t n_rows, const void* P, const void* N);
/* Increment / Decrement (PNCounters.cs:97-112, unchecked '+='): cell (key[i], col[i]) of P
 * (is_n[i] == 0) or N (is_n[i] != 0) += delta[i], wrapping at the store's width. */
int jg_pnc_apply_ops(jg_pnc* pnc, uint64_t n_ops, const uint32_t* key, const uint32_t* col,
                     const int64_t* delta, const uint8_t* is_n);
/* PNCounter.Get (PNCounters.cs:87-90) per key: checked Sum(P) - checked Sum(N), the sums taken in
 * column order, the subtraction wrapping at the store's width.  overflow[i] = 1 (and out[i] = 0)
 * where a checked Sum throws; the call still returns JG_OK.  key_idx NULL = keys 0..n-1. */
int jg_pnc_values(jg_pnc* pnc, const uint32_t* key_idx, uint64_t n, int64_t* out, uint8_t* overflow);

/* Device-resident received batch (the committed state messages of a wave, decoded to rows).
 * key_idx NULL at upload = identity rows (requires n_rows == the store's n_keys at merge time). */
int jg_rows_create(jg_ctx* ctx, uint64_t n_rows, uint32_t n_replicas, uint32_t elem_bytes, jg_rows** out);
int jg_rows_destroy(jg_rows* rows);
int jg_rows_upload(jg_rows* rows, const uint32_t* key_idx, const void* P, const void* N);
int jg_pnc_merge_batch(jg_pnc* pnc, const jg_rows* rows, int async);

/* ---------------------------------------------------------------------------------------------
 * PN-Counter replica table + wire-format apply (csrc/json.hip).  The store keeps, per key, the
 * replica Guids of its columns in first-insertion order (= the stable PNCounter's Dictionary
 * enumeration order, PNCounters.cs:19-25,73-81,131-144); allocated on first use, at most 256
 * replicas per key.  Guids are C# Guid bytes (lo = bytes 0..7, hi = bytes 8..15, little-endian).
 * ------------------------------------------------------------------------------------------- */
typedef struct jg_guid { uint64_t lo, hi; } jg_guid;
typedef struct jg_wave jg_wave;   /* device-resident wave of encoded state messages            */

/* Register replica[i] in row key_idx[i], in order (append if absent); col_out[i] = its column.
 * The PNCounter() constructor's {self: 0} (PNCounters.cs:73-81): CreateSafeCRDT registers the
 * stable instance's own Guid first.  JG_ESTATE (nothing registered) if a row would overflow. */
int jg_pnc_intern(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, const jg_guid* replica, uint32_t* col_out);
/* Column tables of rows key_idx[0..n): replicas[i*R + c] for c < ncols[i]. */
int jg_pnc_columns(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, jg_guid* replicas, uint32_t* ncols);
/* Apply a committed wave of PNCounterMsg wire payloads (System.Text.Json UTF-8, PNCounters.cs:38-49):
 * message i = bytes[off[i], off[i+1]) (off[0] = 0) is decoded and merged into row key_idx[i]
 * exactly as SafeCRDT.ApplyUpdateStable (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83) -> Decode -> Merge
 * would, message after message (SafeCRDTManager.cs:122-146); new replicas get columns in commit
 * order.  All or nothing: a message outside the accepted JSON form (oracle/json.hpp) returns
 * JG_EINVAL, a key running out of columns JG_ESTATE, nothing is applied, and *bad_msg (if not NULL)
 * = the first such message (UINT64_MAX on success).  The caller re-submits the prefix
 * [0, *bad_msg) to reproduce the reference, whose loop applies the messages before the throwing one. */
int jg_pnc_merge_json(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes, uint64_t* bad_msg);
/* The same call streamed in chunks, so the caller's gathering of chunk k+1 overlaps the upload and the
 * decode/validation pass of chunk k: begin (capacity hints; exceeded capacity grows), append chunks
 * in commit order (chunk offsets relative to the chunk: off[0] = 0; returns once the upload and pass A
 * are queued — the chunk's host buffers must stay untouched until commit or abort returns), then
 * commit (= jg_pnc_merge_json over the concatenation: all or nothing, *bad_msg indexes the whole
 * wave) or abort (nothing applied).  One open wave per store. */
int jg_pnc_wave_begin(jg_pnc* pnc, uint64_t cap_msgs, uint64_t cap_bytes);
int jg_pnc_wave_append(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes);
int jg_pnc_wave_commit(jg_pnc* pnc, uint64_t* bad_msg);
int jg_pnc_wave_abort(jg_pnc* pnc);
/* The same with the wave already in device memory (upload once, merge many: the bench). */
int jg_wave_create(jg_ctx* ctx, uint64_t cap_msgs, uint64_t cap_bytes, jg_wave** out);
int jg_wave_destroy(jg_wave* wave);
int jg_wave_upload(jg_wave* wave, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes);
int jg_pnc_merge_wave(jg_pnc* pnc, const jg_wave* wave, uint64_t* bad_msg);

/* GetLastSynchronizedUpdate().Encode() (PNCounters.cs:115-118, 46-49) of rows key_idx[0..n): state i
 * = out[off[i], off[i+1]) (off has n+1 entries, always filled), System.Text.Json's compact form over
 * the row's replica table in column order — what SafeCRDT.Update ships (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:49).
 * out NULL = size query; JG_ESTATE if off[n] > cap (out untouched). */
int jg_pnc_encode_json(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, uint64_t* off, uint8_t* out, uint64_t cap);
/* The same for the row as it stood before its last dp[i] / dn[i] of Increment / Decrement amounts to column col
 * (the cell type's wrapping arithmetic): the snapshot SafeCRDT.Update shipped right after an earlier op of a
 * batch whose later ops on the same key are already applied (SafeCRDT.cs:39-62; PNCounters.cs:97-112).  Lets a
 * batch of client ops be applied in ONE jg_pnc_apply_ops and every snapshot encoded in ONE call. */
int jg_pnc_encode_json_before(jg_pnc* pnc, uint64_t n, const uint32_t* key_idx, uint32_t col, const int64_t* dp, const int64_t* dn,
                              uint64_t* off, uint8_t* out, uint64_t cap, uint8_t* sha);
/* A round of SafeCRDT.Update's PN-Counter client ops at once (SafeCRDT.cs:39-62; PNCounterWrapper.Update ->
 * Increment / Decrement, PNCounters.cs:96-112, on this copy's own column col): every op applied (as jg_pnc_apply_ops),
 * and for each op with need[i] != 0, in op order, dp / dn = the Increment / Decrement amounts the batch's LATER ops
 * on the same key added (wrapping at the store's width) — the rewind jg_pnc_encode_json_before takes to encode the
 * snapshot that op shipped.  Computed on the device (a sort of the ops by key, newest first, and a segmented sum).
 * dp / dn hold count(need) entries.  ABI v9. */
int jg_pnc_apply_ops_rewind(jg_pnc* pnc, uint64_t n_ops, const uint32_t* key, uint32_t col, const int64_t* delta, const uint8_t* is_n,
                            const uint8_t* need, int64_t* dp, int64_t* dn);
/* The whole PN-Counter round in one call (SafeCRDT.cs:39-62 per op: Increment / Decrement on column col, then
 * GetLastSynchronizedUpdate().Encode()): op i's snapshot — the key's row right after op i, i.e. the row before the
 * batch plus the key's ops 0..i — into out[off[i], off[i+1]) (and its SHA-256 into sha + 32 i when sha is not
 * NULL), then every op applied.  The prefixes are a sort + segmented sum on the device; nothing crosses the host
 * link but the ops, the offsets and the bytes.  JG_ESTATE if off[n] > cap: off filled, NOTHING applied (call
 * again with a larger out).  ABI v10. */
int jg_pnc_apply_ops_encode(jg_pnc* pnc, uint64_t n_ops, const uint32_t* key, uint32_t col, const int64_t* delta, const uint8_t* is_n,
                            uint64_t* off, uint8_t* out, uint64_t cap, uint8_t* sha);
/* (sha, here and in jg_orset_encode_json: NULL, or n * 32 bytes receiving each encoded state's SHA256 — the hash
 * UpdateMessage.ComputeDigest takes of it, DAGUpdateMessage.cs:43 — computed on the device from the bytes just
 * written; filled only when out is.  The producer path feeds them to jg_update_digests_of.) */

/* Page-locked host memory for staging waves (PCIe DMA at full rate); free with jg_host_free. */
int jg_host_alloc(jg_ctx* ctx, uint64_t bytes, void** out);
int jg_host_free(void* p);

/* ---------------------------------------------------------------------------------------------
 * OR-Set store — replaces ORSet<string>'s Dictionary<T,HashSet<Guid>> add/remove maps and null
 * tag sets (MergeSharp/MergeSharp/CRDTs/ORSet.cs:78-327) for a whole keyspace of sets.
 * ------------------------------------------------------------------------------------------- */
int jg_orset_create(jg_ctx* ctx, uint64_t cap_add, uint64_t cap_rem, jg_orset** out);
int jg_orset_destroy(jg_orset* s);
/* Replace the state with the given sorted streams (validated: JG_ESTATE if not strictly increasing). */
int jg_orset_load(jg_orset* s, const jg_tagrec* add, uint64_t n_add, const jg_tagrec* rem, uint64_t n_rem);
int jg_orset_size(jg_orset* s, uint64_t* n_add, uint64_t* n_rem);
/* Canonical snapshot (GetLastSynchronizedUpdate, ORSet.cs:305-308). */
int jg_orset_read(jg_orset* s, jg_tagrec* add, uint64_t cap_add, jg_tagrec* rem, uint64_t cap_rem);
/* ORSet.Merge (ORSet.cs:253-283): per element UnionWith of the add and tombstone tag sets (null
 * element included), from host records (sorted, strictly increasing). */
int jg_orset_merge(jg_orset* s, const jg_tagrec* add, uint64_t n_add, const jg_tagrec* rem, uint64_t n_rem);
/* dst = dst ∪ src for two device-resident stores. */
int jg_orset_merge_store(jg_orset* dst, const jg_orset* src, int async);
/* out = a ∪ b (out must have capacity for a+b; it may not alias a or b). */
int jg_orset_union(const jg_orset* a, const jg_orset* b, jg_orset* out, int async);
/* ORSet.Add / Remove / Clear (ORSet.cs:134-198), the OR-Set ApplyOp, applied in op order per set
 * (ORSetWrapper.Update op ids, BFT-CRDT/SafeCRDTs/ORSetWrapper.cs:30-46): op[i] = 1 Add(elem[i]) with
 * the fresh tag (tag_lo[i], tag_hi[i]) the caller drew (Guid.NewGuid()); 2 Remove(elem[i]) — tombstones
 * every tag of the element's add set if Contains(elem) at that point; 3 Clear() of set[i].
 * result[i] = the op's bool result (Remove: 0 when the element was absent).  Any other op id is
 * JG_EINVAL before anything changes (the wrapper's InvalidOperationException). */
int jg_orset_apply_ops(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op,
                       const uint64_t* tag_lo, const uint64_t* tag_hi, uint8_t* result);
/* The same, and per op i the ord limits of a snapshot of its set taken right after it (SafeCRDT.Update's
 * GetLastSynchronizedUpdate() after each op, SafeCRDT.cs:39-62): jg_orset_encode_json with add_lim[i] / rem_lim[i]
 * encodes the set as it stood then — valid while no later op of the batch Clears that set (a Clear drops the
 * records such a snapshot holds). */
int jg_orset_apply_ops_ords(jg_orset* s, uint64_t n_ops, const uint32_t* set, const uint32_t* elem, const uint8_t* op, const uint64_t* tag_lo,
                            const uint64_t* tag_hi, uint8_t* result, uint64_t* add_lim, uint64_t* rem_lim);
/* ORSet.Contains (ORSet.cs:204-237) for (set[i], elem[i]): elem present iff its add set exists
 * and (it has no tombstone set or the two tag sets differ: !SetEquals); the null element is
 * present iff !SetEquals(nullRemove, nullAdd).  out[i] = 0/1. */
int jg_orset_contains(jg_orset* s, const uint32_t* set, const uint32_t* elem, uint64_t n, uint8_t* out);
/* The records of whole sets set[0..n) (every element and null): set i's adds are
 * add[add_off[i], add_off[i+1]), its tombstones rem[rem_off[i], rem_off[i+1]), sorted; the offsets
 * (n+1 entries each) are always filled.  add and rem NULL = size query; JG_ESTATE if a buffer is
 * short.  The per-set GetLastSynchronizedUpdate (ORSet.cs:305-308) that SafeCRDT.Update encodes. */
int jg_orset_read_sets(jg_orset* s, uint64_t n, const uint32_t* set, uint64_t* add_off, jg_tagrec* add, uint64_t cap_add, uint64_t* rem_off,
                       jg_tagrec* rem, uint64_t cap_rem);
/* ORSetMsg.Encode() (MergeSharp/MergeSharp/CRDTs/ORSet.cs:56-69, 305-308) of sets set[0..n) from the device store,
 * byte for byte the reference's System.Text.Json output: addSet elements in ascending element id (= the add
 * Dictionary's insertion order), removeSet elements by their first tombstone's arrival ordinal (ties by id),
 * tags by (ord, tag) (HashSet<Guid> insertion order), the null element's tags in nullAddGuid / nullRemoveGuid;
 * element strings from the store's element table (names issued by waves or synced with jg_orset_names_sync —
 * JG_ESTATE if a record's id has none).  add_lim / rem_lim (both or neither; NULL = everything): state i keeps
 * only its set's add records with ord < add_lim[i] and tombstones with ord < rem_lim[i] — a snapshot taken
 * before a batch's later ops (jg_orset_apply_ops_ords).  State i = out[off[i], off[i+1]); out NULL = size
 * query; JG_ESTATE if off[n] > cap (off filled, out untouched). */
int jg_orset_encode_json(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* add_lim, const uint64_t* rem_lim, uint64_t* off,
                         uint8_t* out, uint64_t cap, uint8_t* sha);
/* ORSet.LookupAll (ORSet.cs:204-227) of sets set[0..n): members of set[i] are elems[off[i], off[i+1])
 * (off has n+1 entries, always filled), in the reference's order: elements with no tombstone set,
 * then elements whose tag sets differ (each group in ascending elem id = the add Dictionary's
 * insertion order when elem ids are interned at first insertion), then JG_NULL_ELEM if null is
 * present.  elems NULL = size query; JG_ESTATE if off[n] > cap (nothing written to elems). */
int jg_orset_lookup_all(jg_orset* s, uint64_t n, const uint32_t* set, uint64_t* off, uint32_t* elems, uint64_t cap);

/* ---------------------------------------------------------------------------------------------
 * OR-Set wire-format apply (csrc/orset_wire.hip; SURVEY.md §8f F1 + A7/A13).  ORSetMsg<string>
 * payloads (System.Text.Json UTF-8, ORSet.cs:56-69) decoded, their element strings interned and the
 * states merged on the device, as SafeCRDT.ApplyUpdateStable (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83)
 * -> ORSet.DecodePropagationMessage -> Merge (ORSet.cs:253-283) would, message after message.
 * Element table: per set, element string -> 32-bit element id, ids issued in first-insertion order
 * (the add/remove Dictionaries' order; addSet entries before removeSet within a state, Merge's walk)
 * and never reused; Clear drops a set's live strings (later adds take new ids).  The device table
 * is the wave path's copy of the caller's interning: the caller registers the names it issues itself
 * (ORSet.Add ops) and the Clears it applies with jg_orset_names_sync before the next wave, and reads
 * back the ids a wave issued with jg_orset_wave_names.
 * ------------------------------------------------------------------------------------------- */
/* Register caller-side interning changes, applied in this order: for each i < n_sets, set[i]'s live
 * strings are dropped if cleared[i] and its next id becomes next_id[i]; then name i < n_names
 * (bytes[off[i], off[i+1]), off[0] = 0) is live in set name_set[i] with id name_id[i] (the caller
 * guarantees it is not live already). */
int jg_orset_names_sync(jg_orset* s, uint64_t n_sets, const uint32_t* set, const uint32_t* next_id, const uint8_t* cleared,
                        uint64_t n_names, const uint32_t* name_set, const uint32_t* name_id, const uint64_t* off, const uint8_t* bytes);
/* A committed wave of ORSetMsg payloads, streamed like jg_pnc_wave_*: message i of the wave (chunks in
 * commit order, chunk-relative offsets, off[0] = 0) is the state of set[i].  append uploads a chunk and
 * queues its validation pass (host buffers untouched until commit / abort returns).  check ends the
 * validation (element names repeated inside one map need the whole wave): JG_OK, or the code of the
 * first message the reference's Decode/Merge would throw on — JG_EINVAL (JsonException: not an
 * ORSetMsg in the accepted form of oracle/json.hpp, a null member or tag set, an element repeated in
 * one map) or JG_ESTATE (an element whose add or tombstone tag set is empty: Add always inserts a tag and
 * Remove copies a non-empty add set, so no reference state holds one, and the record layout has no
 * record to carry the Dictionary key it would add) — with *bad_msg = its
 * wave index (UINT64_MAX if none).  commit merges messages [0, limit) (limit <= *bad_msg): interns
 * their new element strings in commit order and unions their tag records into the store; the wave
 * closes.  abort closes the wave with nothing applied. */
int jg_orset_wave_begin(jg_orset* s, uint64_t cap_msgs, uint64_t cap_bytes);
int jg_orset_wave_append(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* off, const uint8_t* bytes);
int jg_orset_wave_check(jg_orset* s, uint64_t* bad_msg);
int jg_orset_wave_commit(jg_orset* s, uint64_t limit);
int jg_orset_wave_abort(jg_orset* s);
/* The element ids the last commit issued, sorted by (set, id): name i = bytes[off[i], off[i+1]) got id
 * id[i] in set set[i].  set / id / off / bytes NULL = size query (*n_names, *n_bytes). */
int jg_orset_wave_names(jg_orset* s, uint64_t* n_names, uint64_t* n_bytes, uint32_t* set, uint32_t* id, uint64_t* off, uint8_t* bytes);
/* The store's names log: every name the element table took, in the order it took them (commits and
 * jg_orset_names_sync alike; never reordered, cleared names stay in it).  Names [from, *to) with *to = the
 * log's length now: name i - from = bytes[off[i], off[i+1]) with id id[i] in set set[i] (the caller skips
 * the ones it synced itself).  set / id / off / bytes NULL = size query (*to, *n_bytes).  A caller that only
 * needs the ids when it next interns or reads a name pulls them then, several waves at once, instead of
 * after every wave (jg_orset_wave_names) — the ORSetWorkload wave's ~0.7 ms of host copying leaves the
 * apply loop (replaces nothing in the reference: its names live in the C# Dictionaries, ORSet.cs:83-88). */
int jg_orset_names_since(jg_orset* s, uint64_t from, uint64_t* to, uint64_t* n_bytes, uint32_t* set, uint32_t* id, uint64_t* off, uint8_t* bytes);
/* One-shot: begin + append(all) + check, then commit(n) if every message is good; else nothing is
 * applied and the check's code is returned with *bad_msg (the jg_pnc_merge_json contract). */
int jg_orset_merge_json(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* off, const uint8_t* bytes, uint64_t* bad_msg);

/* ---------------------------------------------------------------------------------------------
 * The committed-wave apply loop (csrc/node.hip) — SafeCRDTManager.HandleAfterConsensusUpdates
 * (BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:109-160) as ONE call per committed wave (SURVEY.md §8b B2's
 * jg_apply_batch).  Inside the library: the walk in commit order, the skip of creation and key-space
 * messages (:133-134), the uid lookup safeCRDTsIndexedByuid.TryGetValue (:136) in a device hash table,
 * Decode + Merge of every state (SafeCRDT.ApplyUpdateStable, BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83) on the
 * device, and safeUpdateTracker.TryRemove (:141-142) in a device table.  The library's host workers only
 * gather the payloads into page-locked staging, chunk by chunk, while the device parses the chunk before.
 * ------------------------------------------------------------------------------------------- */
typedef struct jg_node jg_node;        /* one copy (stable or prospective) of a node's keyspace          */
typedef struct jg_tracker jg_tracker;  /* SafeCRDTManager.safeUpdateTracker (SafeCRDTManager.cs:33)     */

/* A node's copy of its keys over a PN-Counter store and an OR-Set store of one context (either NULL if the
 * node holds no key of that type).  The stores stay owned by the caller and must outlive the node. */
int jg_node_create(jg_pnc* pnc, jg_orset* orset, jg_node** out);
int jg_node_destroy(jg_node* node);
/* SafeCRDTManager.CreateSafeCRDT (SafeCRDTManager.cs:61-101) -> safeCRDTsIndexedByuid[uid] = sc (:73, :98):
 * key uid[i] is a PNCounter (type 0) at row idx[i] of the node's store, or an ORSet (type 1) at set id
 * idx[i].  All or nothing: JG_EINVAL for Guid.Empty, a uid registered twice, a row >= the store's n_keys,
 * a set id >= 2^31 - 16, or a type whose store the node lacks.  (The PNCounter constructor's own replica
 * column is jg_pnc_intern's, as before.) */
int jg_node_register(jg_node* node, uint64_t n, const jg_guid* uid, const uint8_t* type, const uint32_t* idx);
/* Key-space sharding over the GPUs of a node: the owner rank of a key is
 * jg_shard_of(uid, world) (a hash of the 16 uid bytes).  A node declared shard `rank` of `world` leaves
 * another shard's states out of its gather from the uid alone — no upload, no lookup; the uid table would
 * skip them the same way (:136), since such a node registers only its own keys.  Registering a uid of
 * another shard turns the shortcut off (the table decides every state again); each jg_node_set_shard
 * rescans the registered uids.  world 1 = no sharding. */
int jg_node_set_shard(jg_node* node, uint32_t rank, uint32_t world);
int jg_shard_of(const jg_guid* uid, uint32_t world, uint32_t* rank);

int jg_tracker_create(jg_ctx* ctx, jg_tracker** out);
int jg_tracker_destroy(jg_tracker* t);
/* ConcurrentDictionary.TryAdd of SafeCRDT.Update (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:55-56: a safe update with a
 * client origin): seq[i] (>= 1, < UINT64_MAX) identifies the NetworkProtocol object, origin[i] (!= 0) the
 * (Connection, id) to notify.  Thread-safe without the context lock (the reference's client threads add
 * while the apply task runs) and cheap: buffered, the device table takes the adds at the next call that
 * reads the tracker.  An identity already tracked keeps its entry. */
int jg_tracker_add(jg_tracker* t, uint64_t n, const uint64_t* seq, const uint64_t* origin);
int jg_tracker_size(jg_tracker* t, uint64_t* n);
/* ContainsKey: out[i] = 1 while seq[i] is tracked. */
int jg_tracker_contains(jg_tracker* t, uint64_t n, const uint64_t* seq, uint8_t* out);

/* A committed wave in commit order (Consensus.Commit's List<List<UpdateMessage>>, Consensus.cs:123-134,
 * flattened: list, block, update): message i is NetworkProtocol{uid[i], syncMsgType type[i]
 * (0 ManagerMsg_Create, 1 CRDTMsg), message} (MergeSharp/MergeSharp/proto/SyncProtocol.cs:12-62) with
 * identity seq[i] (0 = never tracked; seq NULL = all 0).  Payloads either contiguous (off[n + 1], off[0] = 0,
 * bytes) or scattered (off NULL: message i = ptr[i][0 .. len[i])).  Contiguous payloads in page-locked
 * memory (jg_host_alloc) are uploaded from there without a host copy. */
typedef struct jg_commit {
    uint64_t n;
    const jg_guid* uid;
    const uint8_t* type;
    const uint64_t* seq;
    const uint64_t* off;
    const uint8_t* bytes;
    const uint8_t* const* ptr;
    const uint32_t* len;
} jg_commit;

/* HandleAfterConsensusUpdates over one committed wave.  completed[0 .. *n_completed) = the origins of the
 * safe updates the wave completed (their tracker entries removed), in commit order — the
 * safeUpdateCompleteClientNotifier calls; completed needs room for n entries (NULL: count only); tracker
 * may be NULL.  A state its key's Decode / Merge rejects stops the loop there, as the reference's apply
 * Task faults at it: every message before *stopped_at was applied and its completions reported, nothing
 * from it on, and the call returns the rejection's code (JG_EINVAL: JsonException; JG_ESTATE: an OR-Set
 * element with an empty tag set, or a key out of replica columns) — the one entry point that applies a
 * prefix on error.  JG_OK with *stopped_at = UINT64_MAX otherwise.  An internal failure of the wave's OR-Set
 * commit (its device error flag) is returned AFTER the completions: completed / *n_completed are valid,
 * *stopped_at = UINT64_MAX, and the OR-Set store must be reloaded (its union did not finish). */
int jg_apply_committed(jg_node* node, jg_tracker* tracker, const jg_commit* wave, uint64_t* completed, uint64_t* n_completed,
                       uint64_t* stopped_at);
/* ConnectionManager.ReceivedBlock -> ReplicationManager.ReceivedUpdateSyncMsg (BFT-CRDT/Network/DAGConnectionManager.cs:40-50,
 * MergeSharp/MergeSharp/ReplicationManager.cs:290-344) on a node's PROSPECTIVE copy: the same without a
 * tracker; a CRDT state of an uid the node never registered stops the block there with JG_EINVAL
 * (KeyNotFoundException, RM:329).  The shard shortcut does not apply. */
int jg_apply_block(jg_node* node, const jg_commit* wave, uint64_t* stopped_at);
/* jg_apply_committed handed over part by part, so the caller's own copy of the committed byte[]s into page-locked
 * memory overlaps the uploads and parses of the parts before (SafeCRDTManager.cs:109-160 over
 * a wave that arrives block by block).  begin: at most n_max messages and bytes_max payload bytes; append: the next
 * part (commit indices continue from the previous part; a part whose payloads are page-locked and contiguous is
 * uploaded in place, else gathered) — its chunks' uploads and parses are queued before it returns; end: the cut,
 * both commits and the completions, exactly as jg_apply_committed over the concatenated parts.  A part that breaks
 * the wave's rules (decreasing offsets, past the begin's bounds) rejects the whole wave: nothing of it is applied
 * and the stream is closed.  No shard shortcut (every part is uploaded whole).  One streamed wave per node.  A
 * page-locked part's payload bytes are read by the device after append returns: they must stay unchanged until
 * end returns (a gathered part's arrays and every part's uid / type / identity arrays are copied by append). */
int jg_apply_stream_begin(jg_node* node, jg_tracker* tracker, uint64_t n_max, uint64_t bytes_max);
int jg_apply_stream_append(jg_node* node, const jg_commit* part);
int jg_apply_stream_end(jg_node* node, uint64_t* completed, uint64_t* n_completed, uint64_t* stopped_at);
/* Figures of the node's last apply call.  Host: seconds gathering payloads into staging, waiting for the
 * device after the last chunk was queued, the whole call.  Device: kernel time of the wave (hipEvents
 * around each chunk's kernels and around the final phase, on the context's stream) = chunk_busy_s (the
 * per-chunk classify + parse kernels: the payload decode) + tail_busy_s (after the last chunk).  Messages
 * and payload bytes uploaded, messages applied (registered CRDT states before the cut), chunks.  Host
 * phases (ABI v5, appended): setup_s (registrations and tracker adds to the device, buffers sized, the
 * previous call's kernels drained) and loop_s (the chunk loop: gathers + queueing the uploads and kernels);
 * total_s = setup_s + loop_s + device_wait_s + argument checks. */
typedef struct jg_apply_stats {
    double gather_s, device_wait_s, total_s, device_busy_s;
    uint64_t msgs_uploaded, bytes_uploaded, msgs_applied, chunks;
    double chunk_busy_s, tail_busy_s;
    double setup_s, loop_s;
} jg_apply_stats;
int jg_node_last_stats(jg_node* node, jg_apply_stats* out);

/* ---------------------------------------------------------------------------------------------
 * Cross-shard exchange (csrc/route.hip).  The keyspace of a node is sharded over
 * its GPUs: global key k (PN-Counter row / OR-Set set id) belongs to rank k % world, where it is
 * local key k / world.  The reference has one process per node and no sharding: these entry points
 * serve the sharded deployment of the same stores (one process per GPU) when a received batch
 * lands on a rank that does not own all of its keys — the received states still reach
 * PNCounter.Merge (PNCounters.cs:131-144) / ORSet.Merge (ORSet.cs:253-283) on the owner.
 * EXCEPTION to the host-pointer rule above: the d_* arguments are caller-owned DEVICE memory of the
 * context's device (the collective's send / receive buffers, e.g. RCCL all-to-all over xGMI); the
 * library checks that they are device memory of that device and large enough, and returns after
 * its stream is idle.
 * ------------------------------------------------------------------------------------------- */
/* Stable partition of a device batch by owner rank: d_keys[n_rows] (local keys), d_P/d_N[n_rows x R]
 * receive the rows grouped by destination rank in batch order; counts[world] (host) = rows per
 * destination.  world in [1, 64]; cap_rows >= the batch's rows. */
int jg_rows_route(const jg_rows* rows, uint32_t world, uint64_t* counts, void* d_keys, void* d_P, void* d_N, uint64_t cap_rows);
/* jg_pnc_merge_rows from device memory: rows (d_keys[i], d_P[i], d_N[i]), ABSENT cells skipped, keys
 * may repeat; all or nothing (JG_EINVAL if any key >= n_keys, nothing merged). */
int jg_pnc_merge_device(jg_pnc* pnc, uint64_t n_rows, const void* d_keys, const void* d_P, const void* d_N);
/* Stable partition of both record streams of a store by owner rank (set id % world; set ids
 * rewritten to set / world): keys (8 B), tags (16 B, jg_tagrec order) and ords (uint32_t) per stream. */
int jg_orset_route(jg_orset* s, uint32_t world, uint64_t* add_counts, uint64_t* rem_counts, void* d_add_key, void* d_add_tag,
                   void* d_add_ord, uint64_t cap_add, void* d_rem_key, void* d_rem_tag, void* d_rem_ord, uint64_t cap_rem);
/* ORSet.Merge of n_runs received runs (run r = add_counts[r] adds and rem_counts[r] tombstones,
 * stored run after run; each sorted strictly increasing, JG_ESTATE otherwise) into the store, in run
 * order: run r is the r-th state merged (its ords order its own records, jg_tagrec.ord). */
int jg_orset_merge_device(jg_orset* s, uint32_t n_runs, const uint64_t* add_counts, const uint64_t* rem_counts, const void* d_add_key,
                          const void* d_add_tag, const void* d_add_ord, const void* d_rem_key, const void* d_rem_tag, const void* d_rem_ord);

/* The exchange itself, inside the library over RCCL (csrc/comm.hip): one communicator per process (one
 * rank per GPU of the node), then one call per received batch does route -> all-gather of the counts ->
 * grouped ncclSend/ncclRecv of every run over the xGMI peer links (this rank's own run by a device copy)
 * -> merge of the received runs in source-rank order.  Collective: every rank of the communicator makes
 * the same exchange call (a rank with nothing received passes an empty batch / store). */
typedef struct jg_comm jg_comm;
/* ncclGetUniqueId into id[128]: made by one rank and handed to the others over the caller's own channel. */
int jg_comm_unique_id(uint8_t* id);
/* A non-blocking RCCL communicator (ncclCommInitRankConfig, blocking = 0) on ctx's device: returns once all
 * `world` ranks have joined with the same id, or JG_EHIP after JANUS_COMM_TIMEOUT_S seconds (default 120)
 * with the half-made communicator aborted.  Every exchange on it polls against the same deadline: a rank that
 * never posts its half, or an RCCL async error, aborts the communicator and returns JG_EHIP (every later
 * call on it then fails at once) instead of hanging. */
int jg_comm_init(jg_ctx* ctx, uint32_t rank, uint32_t world, const uint8_t* id, jg_comm** out);
/* The host transport: the same exchange with the counts and the runs moved by the caller's all-to-all-v over
 * host memory — send holds the runs for peers 0..world-1 back to back (send_bytes[p] each), recv receives
 * the peers' runs back to back (recv_bytes[p] each, known in advance); returns 0 on success.  For ranks that
 * RCCL cannot serve (several ranks on one GPU, or shards moved over the caller's own links). */
typedef int (*jg_alltoallv_fn)(void* user, const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes);
int jg_comm_init_host(jg_ctx* ctx, uint32_t rank, uint32_t world, jg_alltoallv_fn fn, void* user, jg_comm** out);
int jg_comm_destroy(jg_comm* comm);
/* The exchange's plan (pure host arithmetic, what every exchange call follows): counts[(src * world + dst) * k
 * + j] = records source src routes to destination dst in buffer j (the all-gathered route counts).  For this
 * rank and each peer p, buffer j (index p * k + j): send[send_off .. + send_n) goes to p (the send buffer
 * holds every destination's run in rank order) and recv[recv_off .. + recv_n) comes from p (the peers' runs
 * back to back in source-rank order).  skip_own: the own run is neither sent nor received (the PN-Counter
 * exchange merges it from the send buffer).  world <= 64. */
int jg_exchange_plan(uint32_t rank, uint32_t world, uint32_t k, const uint64_t* counts, uint8_t skip_own, uint64_t* send_off, uint64_t* send_n,
                     uint64_t* recv_off, uint64_t* recv_n);
/* The one owner rule (SafeCRDTManager.cs:136's routing, sharded): a key registered by the rank
 * jg_shard_of(uid, world) names as its owner, with that rank's local index `local`, has the global key
 * local * world + owner — the id the exchange routes by (owner = global % world, local = global / world). */
int jg_global_key(const jg_guid* uid, uint32_t world, uint32_t local, uint32_t* global);
/* PNCounter.Merge (PNCounters.cs:131-144) of a received batch on the owners of its keys: rows is this
 * rank's batch in GLOBAL keys (row key k goes to rank k % world as local key k / world), store this
 * rank's shard (rows NULL: this rank sends nothing).  sent[world] / received[world] (optional): rows per
 * destination / per source. */
int jg_pnc_exchange(jg_comm* comm, jg_pnc* store, const jg_rows* rows, uint64_t* sent, uint64_t* received);
/* ORSet.Merge (ORSet.cs:253-283) of a received state (global set ids: set s goes to rank s % world as
 * s / world) on the owners: the runs merged into store in source-rank order (jg_orset_merge_device).
 * Per-destination / per-source record counts of both streams (optional, world entries each). */
int jg_orset_exchange(jg_comm* comm, jg_orset* store, jg_orset* received, uint64_t* sent_add, uint64_t* sent_rem, uint64_t* recv_add,
                      uint64_t* recv_rem);
/* Figures of the communicator's last exchange: device seconds of route, counts + runs, merge (hipEvents on
 * the context's stream); bytes that left / reached this rank over the links; records merged. */
typedef struct jg_exchange_stats {
    double route_s, exchange_s, merge_s;
    uint64_t bytes_sent, bytes_received, records_received;
} jg_exchange_stats;
int jg_comm_last_stats(jg_comm* comm, jg_exchange_stats* out);

/* ---------------------------------------------------------------------------------------------
 * UpdateMessage digests (csrc/digest.hip) — replaces UpdateMessage.ComputeDigest
 * (BFT-CRDT/DAGConsensus/DAGUpdateMessage.cs:32-55), run by `new UpdateMessage(list)` (:25-30) for
 * every batch the client batcher submits (SafeCRDTManager.ActualPropagateSyncMsg, SafeCRDTManager.cs:165-198).
 * ------------------------------------------------------------------------------------------- */
/* n NetworkProtocol.message payloads: payload i = bytes[off[i], off[i+1]) (off[0] = 0), a C# null when
 * is_null != NULL && is_null[i] (hashed as 32 zero bytes, :41-42).  n_updates UpdateMessages: update u
 * holds payloads [first[u], first[u+1]) (first[0] = 0, first[n_updates] = n).  digest[32u..32u+32) =
 * SHA256(SHA256(payload) for each payload of u ‖ zeros up to ArrayPool<byte>.Shared.Rent(32 * count)
 * .Length) — the .NET 6 bucket length (oracle/digest.hpp).  msg_digest (optional, n * 32 bytes) receives
 * each payload's SHA256 (zeros for null).  Synchronous; JG_EINVAL on malformed offsets. */
int jg_update_digests(jg_ctx* ctx, uint64_t n, const uint64_t* off, const uint8_t* bytes, const uint8_t* is_null, uint64_t n_updates,
                      const uint64_t* first, uint8_t* msg_digest, uint8_t* digest);
/* SHA256.HashData of n payloads (payload i = bytes[off[i], off[i+1]), off[0] = 0) into out (n * 32 bytes): the
 * per-message hashes ComputeDigest takes (DAGUpdateMessage.cs:43), for a caller that assembles UpdateMessages
 * later from payloads it already holds in one buffer (a page-locked `bytes` uploads in place).  Synchronous. */
int jg_sha256_batch(jg_ctx* ctx, uint64_t n, const uint64_t* off, const uint8_t* bytes, uint8_t* out);
/* ComputeDigest's second level from per-payload hashes the caller already has (jg_sha256_batch, or
 * jg_update_digests' msg_digest): msg_digest[32i..32i+32) = SHA256 of payload i (ignored for a null payload,
 * is_null[i] != 0: hashed as 32 zero bytes), update u = payloads [first[u], first[u+1]) as in jg_update_digests.
 * digest[32u..) = the same bytes jg_update_digests gives.  Synchronous. */
int jg_update_digests_of(jg_ctx* ctx, uint64_t n, const uint8_t* msg_digest, const uint8_t* is_null, uint64_t n_updates, const uint64_t* first,
                         uint8_t* digest);
/* The same over a wave already in device memory (jg_wave_upload; no null payloads): first[n_updates]
 * must equal the wave's message count. */
int jg_wave_update_digests(const jg_wave* wave, uint64_t n_updates, const uint64_t* first, uint8_t* msg_digest, uint8_t* digest);
/* The same for n_waves device-resident waves of one context in ONE call, pipelined: wave k+1's
 * per-payload hashes run while wave k's UpdateMessage chains (the serial second level) run on a second
 * stream.  Wave k: n_updates[k] UpdateMessages over payloads first[k][u].. (rules as above, first[k]
 * [n_updates[k]] = that wave's count), digests into digest[k] (n_updates[k] * 32 bytes).  A wave may
 * appear more than once.  Synchronous; JG_EINVAL (nothing computed) when any wave's arguments are
 * malformed or the waves belong to different contexts.  The batched form of the per-batch
 * ComputeDigest calls the batcher makes (SafeCRDTManager.cs:165-198 → DAGUpdateMessage.cs:25-30). */
int jg_waves_update_digests(const jg_wave* const* waves, uint64_t n_waves, const uint64_t* n_updates, const uint64_t* const* first,
                            uint8_t* const* digest);
/* SHA256.HashData of every payload of a device-resident wave (the per-message hashes ComputeDigest takes,
 * DAGUpdateMessage.cs:43) into DEVICE memory d_out (wave count * 32 bytes, digest bytes), for a consumer
 * on the device; async != 0 returns once queued on the context's stream (jg_fence waits). */
int jg_wave_sha256(const jg_wave* wave, void* d_out, uint8_t async);

/* ---------------------------------------------------------------------------------------------
 * Synthetic workloads (bench / size-independent parity): device-side counter-based generators,
 * defined in DESIGN.md §Synthetic inputs and mirrored on the host by the test oracle.
 * ------------------------------------------------------------------------------------------- */
/* which: 0 = local P, 1 = local N, 2 = received P, 3 = received N.  Local unseen cells are 0;
 * received unseen cells are ABSENT.  jg_synth_pnc_rows fills the values of row i from synthetic key
 * key0 + i and keeps the batch's key indices (identity unless uploaded). */
int jg_synth_pnc_store(jg_pnc* pnc, uint64_t seed);
int jg_synth_pnc_rows(jg_rows* rows, uint64_t seed, uint64_t key0);
/* Fill a store with n_groups (set, elem) groups (group g = set*elems_per_set + elem): adds carry
 * tags u in [add_u0, add_u0+add_per_group), tombstones u in [rem_u0, rem_u0+rem_per_group). */
int jg_synth_orset(jg_orset* s, uint64_t seed, uint64_t n_groups, uint32_t elems_per_set,
                   uint32_t add_per_group, uint32_t add_u0, uint32_t rem_per_group, uint32_t rem_u0);

#ifdef __cplusplus
}
#endif

#endif /* JANUS_GPU_H */
