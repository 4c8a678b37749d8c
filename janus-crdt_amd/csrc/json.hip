// json.hip — committed state messages applied straight from their wire bytes (SURVEY.md §8f F1 + A2/A13).
//
// The reference's stable apply decodes every committed state with System.Text.Json and merges it:
// SafeCRDT.ApplyUpdateStable (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83) -> PNCounter.DecodePropagationMessage
// -> PNCounterMsg.Decode (MergeSharp/MergeSharp/CRDTs/PNCounters.cs:38-43) -> Merge (:131-144), one
// message at a time inside HandleAfterConsensusUpdates (SafeCRDTManager.cs:109-160).  Here a whole
// wave of PNCounterMsg JSON payloads is uploaded once and decoded, interned and merged on the GPU:
//
//   pass A  k_scan      8 lanes per message (json_wave.hpp) prove the payload is the compact form
//                       System.Text.Json writes and check it against the wire contract of
//                       oracle/json.hpp; every Guid is looked up in its row's replica table (read-only);
//                       a Guid repeated among a vector's known replicas sends the message to the serial
//                       parser (System.Text.Json keeps the key's last value at its first place).  Each message
//                       leaves a record: its entries' columns and values (pass B applies it), or, when
//                       it names a replica its row has not seen (DEFERRED, marked per message), the
//                       entries' Guids and values with the columns still open.  Payloads not in the
//                       compact form go to the slow list: k_scan_slow runs the serial parser on them.
//   host     deferral marks compacted (hipcub select, count written beside the status) and one
//            D2H of the status words: first bad message, deferred count.  A bad message = nothing
//            is written.
//   sort     hipcub radix sort of the deferred list -> messages grouped by row in commit order.
//   pass C   k_resolve_rows  one lane per row segment walks the row's deferred records in commit
//                       order and appends the new replica Guids (pVector entries first, then nVector —
//                       Merge's order) to the row's table: first-insertion order = the stable
//                       Dictionary's enumeration order; the columns go back into the records.  A walk
//                       reaching a non-compact message continues serially (k_resolve_resume).  A Guid
//                       repeated in one vector keeps its first place and its last value (the earlier
//                       entries are voided).  A full row rolls the appended columns back and fails the call.
//   pass B  k_apply_emit  one lane per record entry, atomicMax into P / N (messages of one wave may
//                       repeat a key; max is order-free); k_apply_list parses the slow list again.
//
// Fused pass A (round 5, the default; JANUS_JSON_FUSE=0 turns it off): a message whose replicas are all known
// is applied by pass A itself once its checks are done, and its record then holds only the entries that
// raised their cell, each with the cell's old value.  All or nothing still holds: max has no inverse, but a
// cell's smallest recorded old value is its value before the wave whatever order the raises took, so a wave
// that fails later (a bad message, a full row, a node wave cut or aborted) is undone exactly by atomicMin over
// the records (k_undo_applied).  The steady state — every replica known, the common wave — writes no record
// entries at all when its states repeat the cells and runs no pass B: the 64-byte records pass B read back and
// the second touch of every cell's lines (pass A + pass B moved 3.1x the algorithmic bytes) go.
//
// JANUS_JSON_GROUP=1 runs the serial parser (scan_one / resolve_one / apply_one: byte-serial per thread
// through a 16-byte window register) for every message: the reference the group path is tested
// against.  The bound of the end-to-end call is the PCIe upload of the payload.
//
// Replica table (jg_pnc::cols / ncols, allocated on first use): [n_keys x R] Guids + [n_keys] counts.
// P and N share one column per replica: the reference keeps two dictionaries whose key orders coincide
// for every state its nodes produce (constructor inserts self into both, Merge inserts new keys in
// message order), which the shared order reproduces.
#include <cstring>
#include <hipcub/hipcub.hpp>

#include "jg_internal.hpp"
#include "wire_cursor.hpp"

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kMaxJsonReplicas = 256;  // per-vector duplicate masks are 4 x 64 bits

enum : uint32_t { kErrSyntax = 0, kErrFull = 1, kErrInternal = 2 };

struct Guid16 { unsigned long long lo, hi; };

using jgw::Cursor;  // byte cursor with a 16-byte aligned window (wire_cursor.hpp)
using jgw::hexv;
using jgw::wave_sync;  // SWAR / LDS helpers shared with orset_wire.hip
using jgw::zero_bytes;
using jgw::ge_bytes;
using jgw::le_bytes;
using jgw::digit_bytes;
using jgw::bits4;
using jgw::hex4;
using jgw::hex_pairs;
using jgw::hex_be16;
using jgw::hex_le16;
using jgw::lds_words;
using jgw::lds_words_b64;

// 36-char "D" Guid (Guid.ToString() layout: b3b2b1b0-b5b4-b7b6-b8b9-b10..b15) + the closing quote.
__device__ __forceinline__ bool read_guid(Cursor& c, Guid16& g) {
    unsigned long long lo = 0, hi = 0;
    // groups: a (8 hex) -> lo[0:32), b (4) -> lo[32:48), c (4) -> lo[48:64), then 8 bytes of hi in text order
    uint32_t v = 0;
    for (int i = 0; i < 8; ++i) { const int h = hexv(c.get()); if (h < 0) return false; v = v << 4 | (uint32_t)h; }
    lo = v;
    if (c.get() != '-') return false;
    v = 0;
    for (int i = 0; i < 4; ++i) { const int h = hexv(c.get()); if (h < 0) return false; v = v << 4 | (uint32_t)h; }
    lo |= (unsigned long long)v << 32;
    if (c.get() != '-') return false;
    v = 0;
    for (int i = 0; i < 4; ++i) { const int h = hexv(c.get()); if (h < 0) return false; v = v << 4 | (uint32_t)h; }
    lo |= (unsigned long long)v << 48;
    if (c.get() != '-') return false;
    for (int b = 0; b < 8; ++b) {
        if (b == 2 && c.get() != '-') return false;
        const int h = hexv(c.get()), l = hexv(c.get());
        if (h < 0 || l < 0) return false;
        hi |= (unsigned long long)(h << 4 | l) << (8 * b);
    }
    if (c.get() != '"') return false;
    g.lo = lo;
    g.hi = hi;
    return true;
}

// -?(0|[1-9][0-9]*) within the width (Utf8JsonReader.GetInt32 / GetInt64).
template <int EB>
__device__ __forceinline__ bool read_int(Cursor& c, long long& out) {
    c.ws();
    bool neg = false;
    int ch = c.peek();
    if (ch == '-') { neg = true; ++c.p; ch = c.peek(); }
    if (ch < '0' || ch > '9') return false;
    unsigned long long mag = 0;
    if (ch == '0') {
        ++c.p;
        ch = c.peek();
        if (ch >= '0' && ch <= '9') return false;  // leading zero
    } else {
        while (ch >= '0' && ch <= '9') {
            const unsigned d = (unsigned)(ch - '0');
            if (mag > (~0ull - d) / 10) return false;
            mag = mag * 10 + d;
            ++c.p;
            ch = c.peek();
        }
    }
    const unsigned long long lim = EB == 4 ? (neg ? 0x80000000ull : 0x7FFFFFFFull) : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
    if (mag > lim) return false;
    out = neg ? (long long)(0ull - mag) : (long long)mag;
    return true;
}

// ---- the decode contract (oracle/json.hpp, System.Text.Json 6.0's defaults) ------------------------------------
// Property names are matched after unescaping; a member the type does not have is skipped (jgw::skip_value); a
// member given twice takes its last occurrence; a Guid key repeated inside one vector keeps its first place and
// takes its last value (Dictionary's indexer).  The compact form System.Text.Json writes — every state a reference
// node emits — is proven by the group parse (json_wave.hpp); the serial parser below runs only on the rest.

struct PncPropSink {  // "pVector" -> 0, "nVector" -> 1, anything else -> 2 (case-sensitive, unescaped)
    uint32_t len = 0, mask = 3;
    __device__ void esc() {}
    __device__ void put(int b) {
        const char* rest = "Vector";
        if (len == 0) mask &= (b == 'p' ? 1u : 0u) | (b == 'n' ? 2u : 0u);
        else if (len > 6 || rest[len - 1] != (char)b) mask = 0;
        ++len;
    }
    __device__ int which() const { return len == 7 && mask ? (mask & 1 ? 0 : 1) : 2; }
};

// A property name (after its opening quote has been found): 0 / 1 / 2 as PncPropSink, -1 if not a string.
__device__ __forceinline__ int read_prop(Cursor& c) {
    if (!c.expect('"')) return -1;
    PncPropSink ps;
    if (!jgw::read_string(c, ps)) return -1;
    return ps.which();
}

// A Guid key after its opening quote: the raw 36-character form, or (escapes) the unescaped string's.
__device__ __forceinline__ bool read_key(Cursor& c, Guid16& g) {
    Cursor t = c;
    if (read_guid(t, g)) {
        c = t;
        return true;
    }
    jgw::GuidSink gs;
    if (!jgw::read_string(c, gs) || !gs.ok()) return false;
    g.lo = gs.lo();
    g.hi = gs.hi;
    return true;
}

__device__ __forceinline__ bool same_guid(const Guid16& a, const Guid16& b) { return a.lo == b.lo && a.hi == b.hi; }

// Per vector, over the whole message: occurrences of the member, whether the last one is `null`, and whether the
// last one may repeat a key (a 128-bit filter of its keys: no shared bit = no repeat, so the common state skips the
// repeat scans).
struct VecInfo {
    uint32_t occ = 0;
    bool null_last = false, maybe_dup = false;
};

// The whole payload checked (every occurrence of every member, skipped ones included): true iff System.Text.Json
// decodes it and both vectors end non-null (else Merge would throw).  No visits.
template <int EB>
__device__ bool validate_pnc(Cursor& c, VecInfo (&vi)[2]) {
    if (!c.expect('{')) return false;
    c.ws();
    if (c.peek() == '}') return false;  // {}: both vectors missing
    for (;;) {
        const int which = read_prop(c);
        if (which < 0 || !c.expect(':')) return false;
        if (which == 2) {
            if (!jgw::skip_value(c, 1)) return false;
        } else {
            VecInfo& v = vi[which];
            ++v.occ;
            v.maybe_dup = false;
            c.ws();
            v.null_last = c.peek() == 'n';
            if (v.null_last) {
                if (!jgw::take_literal(c, "null")) return false;
            } else {
                if (!c.expect('{')) return false;
                unsigned long long f0 = 0, f1 = 0;
                c.ws();
                if (c.peek() == '}') {
                    ++c.p;
                } else {
                    for (;;) {
                        Guid16 g;
                        long long x;
                        if (!c.expect('"') || !read_key(c, g) || !c.expect(':') || !read_int<EB>(c, x)) return false;
                        const uint32_t h = (uint32_t)((g.lo ^ g.hi) * 0x9E3779B97F4A7C15ull >> 57);  // 7 bits
                        const unsigned long long b = 1ull << (h & 63);
                        const bool hit = (h & 64) ? (f1 & b) != 0 : (f0 & b) != 0;
                        v.maybe_dup |= hit;
                        if (h & 64) f1 |= b;
                        else f0 |= b;
                        c.ws();
                        const int ch = c.get();
                        if (ch == '}') break;
                        if (ch != ',') return false;
                    }
                }
            }
        }
        c.ws();
        const int ch = c.get();
        if (ch == '}') break;
        if (ch != ',') return false;
    }
    c.ws();
    return c.p == c.end && vi[0].occ && vi[1].occ && !vi[0].null_last && !vi[1].null_last;
}

// Parse one PNCounterMsg: vis.entry(which, pos, guid, value) for every entry of the decoded message (the last
// occurrence of each vector; a repeated key once, at its first place, with its last value; pos = its place among
// the vector's distinct keys), returning false to abort.  `only` = -1 visits both vectors, 0 / 1 only pVector /
// nVector; begin_vector(which) opens each visited occurrence either way.  The payload is validated whole first
// (validate_pnc), so a message is visited only if System.Text.Json decodes it.
template <int EB, class V>
__device__ bool parse_pnc(Cursor& c, V& vis, int only = -1) {
    VecInfo vi[2];
    {
        Cursor t = c;
        if (!validate_pnc<EB>(t, vi)) {
            c = t;
            return false;
        }
    }
    uint32_t occ[2] = {0, 0};
    (void)c.expect('{');
    for (;;) {
        const int which = read_prop(c);
        (void)c.expect(':');
        if (which == 2 || ++occ[which] < vi[which].occ) {
            (void)jgw::skip_value(c, 1);  // validated: a skipped member, or an occurrence a later one replaces
        } else {
            vis.begin_vector(which);
            (void)c.expect('{');
            c.ws();
            if (c.peek() == '}') {
                ++c.p;
            } else {
                const Cursor vstart = c;
                const bool dups = vi[which].maybe_dup;
                uint32_t pos = 0;
                for (;;) {
                    c.ws();
                    const uint64_t at = c.p;
                    Guid16 g;
                    long long v;
                    (void)c.expect('"');
                    (void)read_key(c, g);
                    (void)c.expect(':');
                    (void)read_int<EB>(c, v);
                    bool first = true;
                    if (dups) {  // a key met earlier in this vector was visited there; else its LAST value counts
                        Cursor t = vstart;
                        for (;;) {
                            t.ws();
                            if (t.p >= at) break;
                            Guid16 h;
                            long long y;
                            (void)t.expect('"');
                            (void)read_key(t, h);
                            (void)t.expect(':');
                            (void)read_int<EB>(t, y);
                            if (same_guid(h, g)) {
                                first = false;
                                break;
                            }
                            (void)t.expect(',');
                        }
                        if (first) {
                            Cursor t2 = c;
                            for (;;) {
                                t2.ws();
                                if (t2.get() != ',') break;
                                Guid16 h;
                                long long y;
                                (void)t2.expect('"');
                                (void)read_key(t2, h);
                                (void)t2.expect(':');
                                (void)read_int<EB>(t2, y);
                                if (same_guid(h, g)) v = y;
                            }
                        }
                    }
                    if (first) {
                        if ((only < 0 || only == which) && !vis.entry(which, pos, g, v)) return false;
                        ++pos;
                    }
                    c.ws();
                    if (c.get() == '}') break;
                }
            }
        }
        c.ws();
        if (c.get() == '}') break;
    }
    c.ws();
    return true;
}

// ---- replica table helpers -------------------------------------------------------------------------
struct Table {
    Guid16* cols;   // [n_keys x R]
    uint32_t* ncols;
    uint32_t R;
};

__device__ __forceinline__ uint32_t find_col(const Guid16* row, uint32_t n, const Guid16& g, uint32_t hint) {
    if (hint < n) {
        const Guid16 h = row[hint];
        if (h.lo == g.lo && h.hi == g.hi) return hint;
    }
    for (uint32_t j = 0; j < n; ++j) {
        const Guid16 h = row[j];
        if (h.lo == g.lo && h.hi == g.hi) return j;
    }
    return UINT32_MAX;
}

// 256-bit column mask without dynamic register indexing (no scratch spills).
struct Mask256 {
    unsigned long long w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __device__ void clear() { w0 = w1 = w2 = w3 = 0; }
    __device__ bool test_set(uint32_t c) {  // returns the old bit (no address taken: stays in registers)
        const unsigned long long b = 1ull << (c & 63);
        bool old;
        switch (c >> 6) {
            case 0: old = (w0 & b) != 0; w0 |= b; break;
            case 1: old = (w1 & b) != 0; w1 |= b; break;
            case 2: old = (w2 & b) != 0; w2 |= b; break;
            default: old = (w3 & b) != 0; w3 |= b; break;
        }
        return old;
    }
};

// Pass A visitor: unknown Guids mark the message deferred (parse_pnc visits a repeated key once).
struct ScanVis {
    const Guid16* row;
    uint32_t n;
    bool miss = false;
    __device__ void begin_vector(int) {}
    __device__ bool entry(int, uint32_t pos, const Guid16& g, long long) {
        if (find_col(row, n, g, pos) == UINT32_MAX) miss = true;
        return true;
    }
};

// Pass A's per-message output (json_wave.hpp writes it for the payloads it proves compact): a u16
// entry count (kReparse: pass B parses the message again), a u16 code per entry (column | vector << 15),
// then the entries' values at +32.  Entries in token order; at most kEmitMax.
constexpr uint32_t kEmitMax = 14;
constexpr uint16_t kReparse = 0xFFFF;
constexpr uint32_t kNeedsCols = 0x4000;  // count flag: a deferred record whose columns pass C resolves
constexpr uint32_t kVoidCol = 0x7FFF;    // entry code column of a voided entry (a key its vector repeats later)
constexpr uint32_t kApplied = 0x2000;    // count flag: pass A applied the message itself (fused); low bits = the
                                         // entries it raised, recorded as (column code, old value) for the undo
__host__ __device__ constexpr uint64_t emit_stride(uint32_t eb) { return 32 + kEmitMax * eb; }

// deferred[m] (pass A): row << 32 | m for a message naming a replica its row has not seen, else this.
constexpr unsigned long long kNotDeferred = ~0ull;

// Serial pass-A body for one message (one lane): the definitive parse.  A message it accepts is marked
// deferred (a replica its row has not seen) or, given a `slow` list, appended to it (pass B parses it
// again); k_scan_slow passes none: its messages are on the list already.
template <int EB>
__device__ void scan_one(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, const uint32_t* __restrict__ rows, uint64_t m,
                         const Table& t, unsigned long long* __restrict__ status, unsigned long long* __restrict__ deferred,
                         uint8_t* __restrict__ emit, unsigned long long* __restrict__ slow) {
    const uint32_t row = rows[m];
    if (row == jg::kSkipIdx) {  // another kind's message in a node wave (csrc/node.hip): no entries
        *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) = 0;
        deferred[m] = kNotDeferred;
        return;
    }
    *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) = kReparse;
    Cursor c(bytes, off[m], off[m + 1]);
    ScanVis vis{t.cols + (uint64_t)row * t.R, t.ncols[row]};
    if (!parse_pnc<EB>(c, vis)) {
        atomicMin(status, (unsigned long long)m << 2 | kErrSyntax);
        return;
    }
    deferred[m] = vis.miss ? (unsigned long long)row << 32 | m : kNotDeferred;  // counted by select_deferred
    if (vis.miss) status[1] = 1;  // any deferral: the guarded tail of finish_wave stands down
    if (!vis.miss && slow) {
        const unsigned long long at = atomicAdd(status + 3, 1ull);
        slow[at] = m;
    }
}

// Chunk offsets arrive relative to their chunk: add the chunk's byte base.
__global__ void k_rebase(uint64_t* __restrict__ off, uint64_t n, uint64_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) off[i] += base;
}

// Pass C visitor: exclusive owner of the row; appends new Guids.  Merge visits every pVector entry
// before any nVector entry (PNCounters.cs:133-143): one parse covers both when pVector comes first in
// the text (every Encode'd state); an nVector ahead of its pVector is skipped and visited by a second
// parse (`only` = 1) once the pVector is in.
struct ResolveVis {
    Guid16* row;
    uint32_t* ncol;
    uint32_t R;
    uint32_t err = UINT32_MAX;
    bool p_seen = false, n_skipped = false;
    __device__ void begin_vector(int which) {
        if (which == 0) p_seen = true;
    }
    __device__ bool entry(int which, uint32_t pos, const Guid16& g, long long) {
        if (which == 1 && !p_seen) { n_skipped = true; return true; }
        uint32_t c = find_col(row, *ncol, g, pos);
        if (c == UINT32_MAX) {
            if (*ncol >= R) { err = kErrFull; return false; }
            c = (*ncol)++;
            row[c] = g;
        }
        return true;
    }
};

// One message of a row's walk (serial): new Guids appended to the row; returns an error code or UINT32_MAX.
template <int EB>
__device__ uint32_t resolve_msg(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t m, Guid16* row, uint32_t* ncol,
                                uint32_t R) {
    ResolveVis vis{row, ncol, R};
    Cursor c(bytes, off[m], off[m + 1]);
    bool ok = parse_pnc<EB>(c, vis);
    if (ok && vis.n_skipped) {
        Cursor c2(bytes, off[m], off[m + 1]);
        ok = parse_pnc<EB>(c2, vis, 1);
    }
    return ok ? UINT32_MAX : vis.err == UINT32_MAX ? kErrInternal : vis.err;
}

// Serial pass C for sorted deferred entry i: a segment head (first entry of a row) walks its row's
// messages in commit order.  saved[i] = the head's ncols before the walk (for roll-back).
template <int EB>
__device__ void resolve_one(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, const unsigned long long* __restrict__ keys,
                            uint64_t nd, uint64_t i, const Table& t, uint32_t* __restrict__ saved, unsigned long long* __restrict__ status) {
    const uint32_t row = (uint32_t)(keys[i] >> 32);
    if (i > 0 && (uint32_t)(keys[i - 1] >> 32) == row) return;
    uint32_t* ncol = t.ncols + row;
    saved[i] = *ncol;
    for (uint64_t j = i; j < nd && (uint32_t)(keys[j] >> 32) == row; ++j) {
        const uint64_t m = (uint32_t)keys[j];
        const uint32_t err = resolve_msg<EB>(bytes, off, m, t.cols + (uint64_t)row * t.R, ncol, t.R);
        if (err != UINT32_MAX) {
            atomicMin(status + 2, (unsigned long long)m << 2 | err);
            return;
        }
    }
}

// The row's count back to its value before the walk, and every slot past it zeroed: a failed walk may have
// written columns it never counted (k_resolve_rows keeps its count in a register until the row is done),
// and pass A reads a row's columns as its leading non-zero slots (json_wave.hpp row_cache).
__global__ __launch_bounds__(kBlock) void k_rollback(const unsigned long long* __restrict__ keys, uint64_t nd, Table t,
                                                     const uint32_t* __restrict__ saved) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nd) return;
    const uint32_t row = (uint32_t)(keys[i] >> 32);
    if (i > 0 && (uint32_t)(keys[i - 1] >> 32) == row) return;
    t.ncols[row] = saved[i];
    for (uint32_t c = saved[i]; c < t.R; ++c) t.cols[(uint64_t)row * t.R + c] = Guid16{0, 0};
}

// Pass B visitor: max into the cells.
template <int EB>
struct ApplyVis {
    using T = typename std::conditional<EB == 4, int, long long>::type;
    T* P;
    T* N;
    const Guid16* row;
    uint32_t n;
    bool bad = false;
    __device__ void begin_vector(int) {}
    __device__ bool entry(int which, uint32_t pos, const Guid16& g, long long v) {
        const uint32_t c = find_col(row, n, g, pos);
        if (c == UINT32_MAX) { bad = true; return false; }
        atomicMax((which ? N : P) + c, (T)v);
        return true;
    }
};

template <int EB>
__device__ void apply_one(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, const uint32_t* __restrict__ rows, uint64_t m,
                          const Table& t, void* P, void* N, unsigned long long* __restrict__ status) {
    using T = typename ApplyVis<EB>::T;
    const uint32_t row = rows[m];
    const uint64_t base = (uint64_t)row * t.R;
    Cursor c(bytes, off[m], off[m + 1]);
    ApplyVis<EB> vis{static_cast<T*>(P) + base, static_cast<T*>(N) + base, t.cols + base, t.ncols[row]};
    if (!parse_pnc<EB>(c, vis)) atomicMin(status + 2, (unsigned long long)m << 2 | kErrInternal);
}

#include "json_wave.hpp"

// jg_pnc_intern: entries (row, guid) in order; keys = row << 32 | i sorted; segment heads walk.
__global__ __launch_bounds__(kBlock) void k_intern(const unsigned long long* __restrict__ keys, uint64_t n, const Guid16* __restrict__ g,
                                                   Table t, uint32_t* __restrict__ col_out, uint32_t* __restrict__ saved,
                                                   unsigned long long* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = (uint32_t)(keys[i] >> 32);
    if (i > 0 && (uint32_t)(keys[i - 1] >> 32) == row) return;
    uint32_t* ncol = t.ncols + row;
    Guid16* cols = t.cols + (uint64_t)row * t.R;
    saved[i] = *ncol;
    for (uint64_t j = i; j < n && (uint32_t)(keys[j] >> 32) == row; ++j) {
        const uint32_t e = (uint32_t)keys[j];
        uint32_t c = find_col(cols, *ncol, g[e], UINT32_MAX);
        if (c == UINT32_MAX) {
            if (*ncol >= t.R) {
                atomicMin(status + 2, (unsigned long long)e << 2 | kErrFull);
                return;
            }
            c = (*ncol)++;
            cols[c] = g[e];
        }
        col_out[e] = c;
    }
}

// Increment / Decrement of one column (PNCounters.cs:97-112, unchecked '+='): wrapping atomic adds.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_ops_col(void* P, void* N, const uint32_t* __restrict__ key, uint32_t col,
                                                          const long long* __restrict__ delta, const uint8_t* __restrict__ is_n, uint64_t n,
                                                          uint32_t R) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t at = (uint64_t)key[i] * R + col;
    if constexpr (EB == 4) atomicAdd(static_cast<unsigned int*>(is_n[i] ? N : P) + at, (unsigned int)delta[i]);
    else atomicAdd(static_cast<unsigned long long*>(is_n[i] ? N : P) + at, (unsigned long long)delta[i]);
}

__global__ void k_make_keys(const uint32_t* __restrict__ rows, uint64_t n, unsigned long long* __restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) keys[i] = (unsigned long long)rows[i] << 32 | i;
}

__global__ void k_gather_cols(const Guid16* __restrict__ cols, const uint32_t* __restrict__ ncols, const uint32_t* __restrict__ rows,
                              uint64_t n, uint32_t R, Guid16* __restrict__ out, uint32_t* __restrict__ nout) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n * R) return;
    const uint64_t q = i / R, c = i - q * R;
    const uint32_t row = rows[q];
    out[i] = cols[(uint64_t)row * R + c];
    if (c == 0) nout[q] = ncols[row];
}

unsigned blocks_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// ---- GetLastSynchronizedUpdate().Encode() on the device ----------------------
// PNCounterMsg.Encode (PNCounters.cs:46-49) of a row: {"pVector":{"<guid D>":P,...},"nVector":{...}}
// over the row's columns in table order (= the Dictionaries' enumeration order), System.Text.Json's
// compact form (the oracle's json::EncodePNC is the checker).  Pass 0: byte length per row; scan;
// pass 1: each thread writes its row's bytes.
__device__ __forceinline__ uint32_t dec_len(long long v) {
    unsigned long long u = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
    uint32_t n = v < 0 ? 2 : 1;
    while (u >= 10) { u /= 10; ++n; }
    return n;
}

template <int EB>
__device__ __forceinline__ long long cell(const void* base, uint64_t i) {
    if constexpr (EB == 4) return static_cast<const int*>(base)[i];
    else return static_cast<const long long*>(base)[i];
}

struct Out {
    uint8_t* p;
    __device__ void put(char c) { *p++ = (uint8_t)c; }
    template <int L>
    __device__ void str(const char (&s)[L]) {  // literals only: unrolled into immediate stores
#pragma unroll
        for (int k = 0; k + 1 < L; ++k) put(s[k]);
    }
    __device__ static char hexc(uint32_t v) {  // arithmetic, not a table: an indexed table is a memory load per digit
        v &= 15;
        return (char)(v < 10 ? '0' + v : 'a' - 10 + v);
    }
    __device__ void hex2(uint32_t b) {
        put(hexc(b >> 4));
        put(hexc(b));
    }
    __device__ void guid(const Guid16& g) {  // Guid.ToString("D"): b3b2b1b0-b5b4-b7b6-b8b9-b10..b15
        for (int k = 3; k >= 0; --k) hex2((uint32_t)(g.lo >> (8 * k)));
        put('-');
        hex2((uint32_t)(g.lo >> 40)); hex2((uint32_t)(g.lo >> 32));
        put('-');
        hex2((uint32_t)(g.lo >> 56)); hex2((uint32_t)(g.lo >> 48));
        put('-');
        hex2((uint32_t)g.hi); hex2((uint32_t)(g.hi >> 8));
        put('-');
        for (int k = 2; k < 8; ++k) hex2((uint32_t)(g.hi >> (8 * k)));
    }
    __device__ void dec(long long v) {
        char d[20];
        int n = 0;
        unsigned long long u = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
        do { d[n++] = (char)('0' + u % 10); u /= 10; } while (u);
        if (v < 0) put('-');
        while (n) put(d[--n]);
    }
};

// Rewind: the row as it stood before its last dp[i] / dn[i] of increments to column `col` (jg_pnc_encode_json_before;
// the cell type's wrapping arithmetic, as Increment's); NULL dp: the row as it is.
template <int EB>
__device__ __forceinline__ long long cell_at(const void* base, uint64_t i, bool rewind, long long d) {
    if constexpr (EB == 4) return rewind ? (long long)(int)((unsigned)cell<4>(base, i) - (unsigned)d) : cell<4>(base, i);
    else return rewind ? (long long)((unsigned long long)cell<8>(base, i) - (unsigned long long)d) : cell<8>(base, i);
}

template <int EB>
__device__ __forceinline__ void encode_row(Out o, Table t, const void* P, const void* N, uint32_t row, uint32_t col, bool rewind,
                                           long long rp, long long rn) {
    const uint32_t nc = t.ncols[row];
    const uint64_t base = (uint64_t)row * t.R;
    for (int which = 0; which < 2; ++which) {
        if (which) o.str("},\"nVector\":{");
        else o.str("{\"pVector\":{");
        const void* V = which ? N : P;
        for (uint32_t c = 0; c < nc; ++c) {
            if (c) o.put(',');
            o.put('"');
            o.guid(t.cols[base + c]);
            o.str("\":");
            o.dec(cell_at<EB>(V, base + c, rewind && c == col, which ? rn : rp));
        }
    }
    o.str("}}");
}

// The write pass stages each wave's rows in LDS.  A wave's rows are consecutive, so their states are one contiguous
// span of the output (the offsets are an exclusive scan), and the span goes out in aligned 16-byte stores of whole
// lines instead of every lane storing its own row a byte at a time ~370 bytes from its neighbours (64 partial lines
// per store instruction, which the memory side then merges line by line).  The span is placed in LDS at the output
// address's offset within 16 bytes, so LDS chunk k is output chunk k.  A span past kEncStage (rows with many replica
// columns) is written directly.  One wave per workgroup: 64 C5 rows (4 replicas) are ~23.5 KB.
constexpr uint32_t kEncStage = 32768;
constexpr int kEncLanes = 64;

template <int EB, int PASS>
__global__ __launch_bounds__(kBlock) void k_encode(const uint32_t* __restrict__ rows, uint64_t n, Table t, const void* P, const void* N,
                                                   unsigned long long* __restrict__ len_off, uint8_t* __restrict__ out, uint32_t col,
                                                   const long long* __restrict__ dp, const long long* __restrict__ dn) {
    if (PASS == 0) {
        const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (i >= n) return;
        const uint32_t row = rows[i];
        const uint32_t nc = t.ncols[row];
        const uint64_t base = (uint64_t)row * t.R;
        const long long rp = dp ? dp[i] : 0, rn = dp ? dn[i] : 0;
        unsigned long long len = 27 + (nc ? 2ull * (40ull * nc - 1) : 0);
        for (uint32_t c = 0; c < nc; ++c)
            len += dec_len(cell_at<EB>(P, base + c, dp && c == col, rp)) + dec_len(cell_at<EB>(N, base + c, dp && c == col, rn));
        len_off[i] = len;
        return;
    } else {  // launched with kEncLanes threads per workgroup
        __shared__ __attribute__((aligned(16))) uint8_t stage[kEncStage + 16];
        const uint64_t first = (uint64_t)blockIdx.x * kEncLanes, i = first + threadIdx.x;
        const uint64_t last = first + kEncLanes < n ? first + kEncLanes : n;
        const unsigned long long lo = len_off[first], hi = len_off[last];  // (len_off holds n + 1 offsets)
        const bool staged = hi - lo <= kEncStage;  // uniform over the workgroup
        const uint32_t mis = (uint32_t)((uintptr_t)(out + lo) & 15);
        if (i < n) {
            const unsigned long long at = len_off[i];
            const uint32_t row = rows[i];
            const long long rp = dp ? dp[i] : 0, rn = dp ? dn[i] : 0;
            if (staged) encode_row<EB>(Out{stage + mis + (at - lo)}, t, P, N, row, col, dp != nullptr, rp, rn);  // LDS stores
            else encode_row<EB>(Out{out + at}, t, P, N, row, col, dp != nullptr, rp, rn);
        }
        if (!staged) return;
        __syncthreads();
        uint8_t* g = out + lo - mis;  // 16-byte aligned; only bytes [mis, end) of it are written
        const uint32_t end = mis + (uint32_t)(hi - lo), chunks = (end + 15) >> 4;
        for (uint32_t k = threadIdx.x; k < chunks; k += kEncLanes) {
            const uint32_t b0 = 16 * k;
            if (b0 >= mis && b0 + 16 <= end) {
                *reinterpret_cast<uint4*>(g + b0) = *reinterpret_cast<const uint4*>(stage + b0);
            } else {
                for (uint32_t b = b0; b < b0 + 16; ++b)
                    if (b >= mis && b < end) g[b] = stage[b];
            }
        }
    }
}

void ensure_table(jg_pnc* p) {
    if (p->cols.p) return;
    JG_REQUIRE(p->R <= kMaxJsonReplicas, JG_EINVAL, "replica table: at most %u replicas per key (store has %u)", kMaxJsonReplicas, p->R);
    p->cols.alloc((size_t)p->n_keys * p->R * sizeof(Guid16));
    p->ncols.alloc((size_t)p->n_keys * 4);
    JG_HIP(hipMemsetAsync(p->cols.p, 0, p->cols.bytes, p->ctx->stream));  // unused slots are zero (json_wave.hpp row_cache)
    JG_HIP(hipMemsetAsync(p->ncols.p, 0, p->ncols.bytes, p->ctx->stream));
}

Table table_of(jg_pnc* p) { return Table{p->cols.as<Guid16>(), p->ncols.as<uint32_t>(), p->R}; }

struct IsDeferred {
    __host__ __device__ bool operator()(const unsigned long long& k) const { return k != kNotDeferred; }
};

// Pass A's per-message deferral marks (n of them) compacted into a list, its length written to *count
// on the device; then sorted by (row, message) = commit order within each row.  Marks and a compaction
// instead of an appended list or a counter: every wave touching one address serialises the grid at
// that address's L2 channel — a cold wave (every message deferred) measured 1.5 ms for pass A instead
// of 0.33 with one non-returning atomic per wave.
struct DeferredLists {
    unsigned long long* list;    // n slots
    unsigned long long* sorted;  // n slots
    void* tmp;
    size_t tmp_bytes;
    int end_bit;
};

// Radix sorts of the (row << 32 | index) keys on the row bits: Onesweep at every size.  hipcub's default takes a
// block sort plus merge passes below 1M items (the config's merge_sort_limit), ~200 us for a C5 wave's ~0.5M
// deferred entries, whatever the bit range; three 8-bit Onesweep passes cover 1M rows.
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
hipError_t sort_row_keys(void* tmp, size_t& bytes, const unsigned long long* in, unsigned long long* out, uint64_t n, int end_bit,
                         hipStream_t stream) {
    return rocprim::radix_sort_keys<OnesweepSort>(tmp, bytes, in, out, (size_t)n, 32u, (unsigned)end_bit, stream);
}

DeferredLists select_deferred(jg_ctx* ctx, const unsigned long long* marks, uint64_t n, uint64_t n_keys, unsigned long long* count) {
    JG_REQUIRE(n <= 0x7FFFFFFFull, JG_EINVAL, "sort: %llu entries exceed one radix sort", (unsigned long long)n);
    using ull = unsigned long long;
    DeferredLists d{};
    int row_bits = 1;
    while (row_bits < 32 && (1ull << row_bits) < n_keys) ++row_bits;
    d.end_bit = 32 + row_bits;
    size_t tsel = 0, tsort = 0;
    JG_HIP(hipcub::DeviceSelect::If(nullptr, tsel, marks, (ull*)nullptr, (ull*)nullptr, (int)n, IsDeferred(), ctx->stream));
    JG_HIP(sort_row_keys(nullptr, tsort, (const ull*)nullptr, (ull*)nullptr, n, d.end_bit, ctx->stream));
    const size_t a = (n * 8 + 255) & ~255ull;
    d.tmp_bytes = std::max(tsel, tsort);
    char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, 2 * a + d.tmp_bytes + 256));
    d.list = reinterpret_cast<ull*>(s);
    d.sorted = reinterpret_cast<ull*>(s + a);
    d.tmp = s + 2 * a;
    JG_HIP(hipcub::DeviceSelect::If(d.tmp, tsel, marks, d.list, count, (int)n, IsDeferred(), ctx->stream));
    return d;
}

// The list comes out of the (stable) select in message order, so a stable sort on the row bits alone gives the
// order of the whole key (row, then message): 20 bits for 1M keys instead of 52.
unsigned long long* sort_deferred(jg_ctx* ctx, DeferredLists& d, uint64_t nd) {
    size_t t = d.tmp_bytes;
    JG_HIP(sort_row_keys(d.tmp, t, d.list, d.sorted, nd, d.end_bit, ctx->stream));
    return d.sorted;
}

// Sort `n` 64-bit keys (row << 32 | index) in place through ctx scratch.  end_bit covers the row bits; the keys
// arrive in index order (k_make_keys), so a stable sort on the row bits alone orders the whole key.
unsigned long long* sort_keys(jg_ctx* ctx, unsigned long long* keys, uint64_t n, uint64_t n_keys) {
    JG_REQUIRE(n <= 0x7FFFFFFFull, JG_EINVAL, "sort: %llu entries exceed one radix sort", (unsigned long long)n);
    int row_bits = 1;
    while (row_bits < 32 && (1ull << row_bits) < n_keys) ++row_bits;
    const int end_bit = 32 + row_bits;
    size_t temp = 0;
    JG_HIP(sort_row_keys(nullptr, temp, keys, keys, n, end_bit, ctx->stream));
    char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch3, temp + n * 8 + 256));
    unsigned long long* out = reinterpret_cast<unsigned long long*>(s);
    void* tmp = s + ((n * 8 + 255) & ~255ull);
    JG_HIP(sort_row_keys(tmp, temp, keys, out, n, end_bit, ctx->stream));
    return out;
}

struct Status { unsigned long long first_bad, n_deferred, resolve_bad, n_slow, n_resume; };

static_assert(sizeof(Status) <= 256, "status fits the context's page-locked word");

// Into the context's page-locked bytes: a pageable destination is staged by the runtime (a blit plus a host
// copy per read; three reads per wave)
Status read_status(jg_ctx* ctx, const unsigned long long* d) {
    Status s;
    jg::pin_get(ctx, 0, d, sizeof s);
    jg::pin_sync(ctx);
    std::memcpy(&s, jg::pin_at(ctx, 0), sizeof s);
    return s;
}

// kErrInternal (a message pass A accepted that a later pass could not parse or resolve again) is the library's
// own inconsistency, never a verdict on the message: it leaves *bad_msg unset, so a node wave does not take it for
// the reference's cut (pnc_node_finish rethrows, wave_end aborts the wave) and no caller blames the payload.
[[noreturn]] void fail_msg(unsigned long long code, uint64_t* bad_msg, const char* what) {
    const uint64_t m = code >> 2;
    const uint32_t kind = (uint32_t)(code & 3);
    if (bad_msg && kind != kErrInternal) *bad_msg = m;
    if (kind == kErrFull)
        jg::fail(JG_ESTATE, "%s %llu: its key holds more replicas than the store's columns", what, (unsigned long long)m);
    if (kind == kErrInternal) jg::fail(JG_EHIP, "%s %llu: internal replica-table inconsistency", what, (unsigned long long)m);
    jg::fail(JG_EINVAL, "%s %llu is not a PNCounterMsg in the accepted JSON form (JsonException)", what, (unsigned long long)m);
}

// Grow a wave buffer to `need` bytes keeping the first `keep` bytes (stream-ordered copy).
void grow_keep(jg_ctx* ctx, jg::DevBuf& b, size_t need, size_t keep) {
    if (b.bytes >= need) return;
    jg::DevBuf nb;
    nb.alloc(need + need / 2);
    if (keep) JG_HIP(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    std::swap(nb.p, b.p);
    std::swap(nb.bytes, b.bytes);
}

// Wave-level device scratch: status words, pass A's deferred marks and the roll-back slots (n messages),
// pass A's per-message entries and its list of messages for pass B to parse again.
struct WaveScratch {
    unsigned long long* status;
    unsigned long long* deferred;
    uint32_t* saved;
    uint8_t* emit;
    Guid16* eguid;  // [n x kEmitMax] entry Guids of the deferred compact messages
    unsigned long long* slow;
};

// Room for n messages; growing keeps the status words and the first `keep` deferred entries (a
// streamed wave grows between chunks).  The roll-back slots follow the deferred list, so their
// offset depends on the capacity: they are only written at finish time.
WaveScratch wave_scratch(jg_pnc* p, uint64_t n, uint64_t keep = 0) {
    const size_t need = 64 + n * 8 + n * 4 + 256;
    if (p->wstat.bytes < need) grow_keep(p->ctx, p->wstat, need, p->wstat.p ? 64 + keep * 8 : 0);
    grow_keep(p->ctx, p->wemit, n * emit_stride(p->eb) + 256, keep * emit_stride(p->eb));
    grow_keep(p->ctx, p->wslow, n * 8 + 256, keep * 8);
    grow_keep(p->ctx, p->wguid, n * kEmitMax * sizeof(Guid16) + 256, keep * kEmitMax * sizeof(Guid16));
    n = (p->wstat.bytes - 64 - 256) / 12;  // the capacity actually there
    char* s = p->wstat.as<char>();
    return WaveScratch{reinterpret_cast<unsigned long long*>(s), reinterpret_cast<unsigned long long*>(s + 64),
                       reinterpret_cast<uint32_t*>(s + 64 + ((n * 8 + 15) & ~15ull)), p->wemit.as<uint8_t>(), p->wguid.as<Guid16>(),
                       p->wslow.as<unsigned long long>()};
}

__global__ void k_reset_status(unsigned long long* status) {
    const unsigned long long init[5] = {~0ull, 0, ~0ull, 0, 0};  // Status{first_bad, n_deferred, resolve_bad, n_slow, n_resume}
    if (threadIdx.x < 5) status[threadIdx.x] = init[threadIdx.x];
}

// a one-wave kernel instead of a copy from pageable host memory (staged by the runtime: a blit and a host
// round trip in front of every wave's pass A)
void reset_status(jg_ctx* ctx, unsigned long long* status) {
    hipLaunchKernelGGL(k_reset_status, dim3(1), dim3(64), 0, ctx->stream, status);
    JG_HIP(hipGetLastError());
}

// A wave's status words at their initial values: reset on the device unless the last wave left them so (a
// clean wave — nothing bad, deferred, slow or resumed — never writes them: round 6 skips the reset launch).
void begin_status(jg_pnc* p, unsigned long long* status) {
    if (!p->status_clean) reset_status(p->ctx, status);
    p->status_clean = false;
}

// JANUS_JSON_FUSE=0: pass A leaves every message to pass B (read per launch: tests and A/B runs switch it)
// Latched into jg_pnc::fuse when a wave begins (merge_wave_dev, jg_pnc_wave_begin, pnc_node_begin): the chunks'
// pass A and the wave's finish must agree on it, or finish_wave would skip pass B for records pass A left to it
// (ADVICE r05).
bool json_fuse() {
    const char* e = std::getenv("JANUS_JSON_FUSE");
    return !(e && std::strcmp(e, "0") == 0);
}

void launch_scan(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t m0, uint64_t m1,
                 const WaveScratch& w) {
    if (m1 <= m0) return;
    const Table t = table_of(p);
    const int G = json_group();
    const bool fuse = p->fuse;
    if (p->eb == 8) launch_scan_g<8>(G, p->ctx->stream, bytes, off, rows, m0, m1, t, w.status, w.deferred, w.emit, w.eguid, w.slow, p->P.p, p->N.p, fuse);
    else launch_scan_g<4>(G, p->ctx->stream, bytes, off, rows, m0, m1, t, w.status, w.deferred, w.emit, w.eguid, w.slow, p->P.p, p->N.p, fuse);
    JG_HIP(hipGetLastError());
    p->scan_hi = std::max(p->scan_hi, m1);
}

// A fused pass A over messages [0, p->scan_hi) taken back (stream-ordered): the wave failed after it, or a node
// wave was cut or aborted.  Idempotent; a no-op for messages pass A left to pass B.
void undo_applied(jg_pnc* p, const uint32_t* rows) {
    const uint64_t n = p->scan_hi;
    if (n == 0 || !p->wemit.p) return;
    const Table t = table_of(p);
    const unsigned g = (unsigned)((n * kEmitLanes + kBlock - 1) / kBlock);
    if (p->eb == 8) hipLaunchKernelGGL(k_undo_applied<8>, dim3(g), dim3(kBlock), 0, p->ctx->stream, p->wemit.as<uint8_t>(), rows, n, t.R, p->P.p, p->N.p);
    else hipLaunchKernelGGL(k_undo_applied<4>, dim3(g), dim3(kBlock), 0, p->ctx->stream, p->wemit.as<uint8_t>(), rows, n, t.R, p->P.p, p->N.p);
    JG_HIP(hipGetLastError());
}

// After pass A over all n messages: check, resolve new replicas, apply.  All or nothing.
void finish_wave(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, const WaveScratch& w,
                 uint64_t* bad_msg) {
    jg_ctx* ctx = p->ctx;
    const Table t = table_of(p);
    const int G = json_group();
    const unsigned ge = (unsigned)((n * kEmitLanes + kBlock - 1) / kBlock);
    if (G > 1) {
        // The steady state of a fused wave (every payload compact and valid, every replica known): pass A's status
        // alone ends it — one read, no slow-list launches (round 6: k_scan_slow and k_apply_slow cost ~5 µs each
        // even with nothing to do, the next wave's status reset another 5).  Otherwise the launches below.
        if (p->fuse) {
            const Status s0 = read_status(ctx, w.status);
            if (s0.first_bad == ~0ull && s0.n_deferred == 0 && s0.resolve_bad == ~0ull && s0.n_slow == 0 && s0.n_resume == 0) {
                p->status_clean = true;
                return;
            }
        }
        // the payloads the group parse left to the serial parser (count read on the device)
        if (p->eb == 8) hipLaunchKernelGGL(k_scan_slow<8>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, rows, t, w.status, w.deferred, w.emit, w.slow);
        else hipLaunchKernelGGL(k_scan_slow<4>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, rows, t, w.status, w.deferred, w.emit, w.slow);
        JG_HIP(hipGetLastError());
        // The steady state (every payload valid, every replica known): pass B right away, guarded on the
        // device by pass A's status, so the wave costs one status read.  If pass A failed or deferred a
        // message both launches are no-ops and the full path below runs (all or nothing).  A fused pass A
        // (json_fuse) applied every record pass B would read here (a deferral sends the wave to the full path,
        // whose pass B runs unguarded): only the slow list's launch is left.
        const bool fused = p->fuse;
        if (p->eb == 8) {
            if (!fused) hipLaunchKernelGGL(k_apply_emit<8>, dim3(ge), dim3(kBlock), 0, ctx->stream, w.emit, rows, n, t.R, p->P.p, p->N.p, w.status);
            hipLaunchKernelGGL(k_apply_slow<8>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, rows, w.slow, t, p->P.p, p->N.p, w.status);
        } else {
            if (!fused) hipLaunchKernelGGL(k_apply_emit<4>, dim3(ge), dim3(kBlock), 0, ctx->stream, w.emit, rows, n, t.R, p->P.p, p->N.p, w.status);
            hipLaunchKernelGGL(k_apply_slow<4>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, rows, w.slow, t, p->P.p, p->N.p, w.status);
        }
        JG_HIP(hipGetLastError());
        const Status st = read_status(ctx, w.status);
        if (st.first_bad != ~0ull) undo_applied(p, rows), fail_msg(st.first_bad, bad_msg, "state message");
        if (!st.n_deferred) {
            // only k_apply_slow can have set it here (no walk ran): kErrInternal, a JG_EHIP without a cut; the
            // fused applies are taken back, the slow list's raises (no undo records) stay — an internal failure
            if (st.resolve_bad != ~0ull) undo_applied(p, rows), fail_msg(st.resolve_bad, bad_msg, "state message");
            return;
        }
    }
    DeferredLists dl = select_deferred(ctx, w.deferred, n, p->n_keys, w.status + 1);
    Status st = read_status(ctx, w.status);
    if (st.first_bad != ~0ull) undo_applied(p, rows), fail_msg(st.first_bad, bad_msg, "state message");
    unsigned long long* sorted_deferred = nullptr;
    if (st.n_deferred) {
        const uint64_t nd = st.n_deferred;
        unsigned long long* sorted = sort_deferred(ctx, dl, nd);
        sorted_deferred = sorted;
        const unsigned gd = blocks_for(nd);
        // the resume list reuses pass A's deferral marks (dead once compacted)
        if (p->eb == 8) launch_resolve_g<8>(G, ctx->stream, bytes, off, sorted, nd, t, w.emit, w.eguid, w.saved, w.status, w.deferred);
        else launch_resolve_g<4>(G, ctx->stream, bytes, off, sorted, nd, t, w.emit, w.eguid, w.saved, w.status, w.deferred);
        JG_HIP(hipGetLastError());
        st = read_status(ctx, w.status);
        if (st.n_resume && st.resolve_bad == ~0ull) {  // walks the group parse handed to the serial parser
            if (p->eb == 8)
                hipLaunchKernelGGL(k_resolve_resume<8>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, sorted, nd, t, w.status, w.deferred, w.emit, w.eguid);
            else
                hipLaunchKernelGGL(k_resolve_resume<4>, dim3(64), dim3(kBlock), 0, ctx->stream, bytes, off, sorted, nd, t, w.status, w.deferred, w.emit, w.eguid);
            JG_HIP(hipGetLastError());
            st = read_status(ctx, w.status);
        }
        if (st.resolve_bad != ~0ull) {
            hipLaunchKernelGGL(k_rollback, dim3(gd), dim3(kBlock), 0, ctx->stream, sorted, nd, t, w.saved);
            JG_HIP(hipGetLastError());
            undo_applied(p, rows);
            JG_HIP(hipStreamSynchronize(ctx->stream));
            fail_msg(st.resolve_bad, bad_msg, "state message");
        }
    }
    // pass B: pass A's records (resolved by pass C where deferred), then the messages left to the serial
    // parser (slow: not in the compact form; with JANUS_JSON_GROUP=1 also the deferred ones).  max is
    // order-free.
    if (p->eb == 8) hipLaunchKernelGGL(k_apply_emit<8>, dim3(ge), dim3(kBlock), 0, ctx->stream, w.emit, rows, n, t.R, p->P.p, p->N.p, nullptr);
    else hipLaunchKernelGGL(k_apply_emit<4>, dim3(ge), dim3(kBlock), 0, ctx->stream, w.emit, rows, n, t.R, p->P.p, p->N.p, nullptr);
    JG_HIP(hipGetLastError());
    const unsigned long long* lists[2] = {st.n_deferred ? sorted_deferred : nullptr, w.slow};
    const uint64_t counts[2] = {st.n_deferred, st.n_slow};
    for (int l = G > 1 ? 1 : 0; l < 2; ++l) {
        if (!counts[l]) continue;
        const unsigned gl = blocks_for(counts[l]);
        if (p->eb == 8) hipLaunchKernelGGL(k_apply_list<8>, dim3(gl), dim3(kBlock), 0, ctx->stream, bytes, off, rows, lists[l], counts[l], t, p->P.p, p->N.p, w.status);
        else hipLaunchKernelGGL(k_apply_list<4>, dim3(gl), dim3(kBlock), 0, ctx->stream, bytes, off, rows, lists[l], counts[l], t, p->P.p, p->N.p, w.status);
        JG_HIP(hipGetLastError());
    }
    st = read_status(ctx, w.status);
    // Past pass C every message has been judged, so only k_apply_list's re-parse (apply_one: kErrInternal) can set
    // it now: the library's own inconsistency, raised as JG_EHIP without naming a message (fail_msg), so it is never
    // taken for a cut whose prefix re-run would leave pass B's raises (no undo records) in the store.
    if (st.resolve_bad != ~0ull) {
        JG_REQUIRE((st.resolve_bad & 3) == kErrInternal, JG_EHIP, "pass B: status %llx after every message was judged", st.resolve_bad);
        undo_applied(p, rows);
        fail_msg(st.resolve_bad, bad_msg, "state message");
    }
}

// The whole device side of a wave already in device memory.
void merge_wave_dev(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, uint64_t* bad_msg) {
    ensure_table(p);
    const WaveScratch w = wave_scratch(p, n);
    begin_status(p, w.status);
    p->scan_hi = 0;
    p->fuse = json_fuse();
    launch_scan(p, bytes, off, rows, 0, n, w);
    finish_wave(p, bytes, off, rows, n, w, bad_msg);
}

void check_wave_host(const jg_pnc* p, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const char* fn) {
    JG_REQUIRE(n < 0xFFFFFFFFull, JG_EINVAL, "%s: at most 2^32-2 messages per wave", fn);
    JG_REQUIRE(off[0] == 0, JG_EINVAL, "%s: off[0] must be 0", fn);
    for (uint64_t i = 0; i < n; ++i) {
        JG_REQUIRE(off[i + 1] >= off[i], JG_EINVAL, "%s: offsets decrease at message %llu", fn, (unsigned long long)i);
        JG_REQUIRE(key_idx[i] < p->n_keys, JG_EINVAL, "%s: key_idx[%llu] = %u out of range (n_keys %llu)", fn, (unsigned long long)i,
                   key_idx[i], (unsigned long long)p->n_keys);
    }
}

}  // namespace

// ---- node waves (csrc/node.hip) ------------------------------------------------------------------
// The node uploads every kind's messages of a committed wave once, classifies them on the device and
// drives this path over its own buffers: rows[m] = the message's row, or kSkipIdx for another kind's.
namespace jg {

void pnc_node_begin(jg_pnc* p, uint64_t n) {
    ensure_table(p);
    begin_status(p, wave_scratch(p, n).status);
    p->scan_hi = 0;
    p->fuse = json_fuse();
    p->wn = n;  // the node wave's capacity (jg_pnc_wave_* calls are refused while it is open: node_open)
}

void pnc_node_scan(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t m0, uint64_t m1) {
    launch_scan(p, bytes, off, rows, m0, m1, wave_scratch(p, p->wn));
}

// The rest of the wave over messages [0, n) (pass A ran on all of them), all or nothing: JG_OK, or the
// code of the first rejected message (*bad, why) with nothing applied.  Other failures throw.
int pnc_node_finish(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, uint64_t* bad, std::string* why) {
    *bad = UINT64_MAX;
    if (n == 0) return JG_OK;
    try {
        finish_wave(p, bytes, off, rows, n, wave_scratch(p, p->wn), bad);
        p->scan_hi = 0;  // committed: a later abort of the node wave (an OR-Set commit failing) must not undo it
        return JG_OK;
    } catch (const Error& e) {
        if (*bad == UINT64_MAX) throw;
        *why = e.msg;
        return e.code;
    }
}

// Pass A again over [0, n) only, then the rest: the prefix of a wave cut at n (the reference's loop
// applied the messages before the one that threw).
int pnc_node_prefix(jg_pnc* p, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t n, uint64_t* bad, std::string* why) {
    *bad = UINT64_MAX;
    undo_applied(p, rows);  // the chunks' fused pass A applied messages past the cut too: back to the state before the wave
    p->scan_hi = 0;
    if (n == 0) return JG_OK;  // a cut at message 0: nothing applied (the undo used to come after this return)
    const WaveScratch w = wave_scratch(p, p->wn);
    begin_status(p, w.status);
    p->scan_hi = 0;
    launch_scan(p, bytes, off, rows, 0, n, w);
    return pnc_node_finish(p, bytes, off, rows, n, bad, why);
}

// A node wave abandoned after its chunks' pass A (an internal failure): the fused applies taken back.
void pnc_node_undo(jg_pnc* p, const uint32_t* rows) {
    undo_applied(p, rows);
    p->scan_hi = 0;
}

}  // namespace jg

// Device-resident wave of encoded state messages (bench / pre-staged waves).
extern "C" {

int jg_pnc_intern(jg_pnc* p, uint64_t n, const uint32_t* key_idx, const jg_guid* replica, uint32_t* col_out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_intern");
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_intern: store is NULL");
        if (n == 0) return;
        JG_REQUIRE(key_idx && replica && col_out, JG_EINVAL, "jg_pnc_intern: NULL argument");
        JG_REQUIRE(n < 0xFFFFFFFFull, JG_EINVAL, "jg_pnc_intern: at most 2^32-2 entries per call");
        for (uint64_t i = 0; i < n; ++i)
            JG_REQUIRE(key_idx[i] < p->n_keys, JG_EINVAL, "jg_pnc_intern: key_idx[%llu] = %u out of range", (unsigned long long)i, key_idx[i]);
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        ensure_table(p);
        const Table t = table_of(p);
        char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch, 64 + n * (4 + 16 + 8 + 4 + 4) + 256));
        auto* status = reinterpret_cast<unsigned long long*>(s);
        auto* keys = reinterpret_cast<unsigned long long*>(s + 64);
        auto* g = reinterpret_cast<Guid16*>(s + 64 + n * 8);
        auto* rows = reinterpret_cast<uint32_t*>(s + 64 + n * 24);
        auto* cols = rows + n;
        auto* saved = cols + n;
        const Status init{~0ull, 0, ~0ull, 0};
        JG_HIP(hipMemcpyAsync(status, &init, sizeof init, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(rows, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(g, replica, n * 16, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_make_keys, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, rows, n, keys);
        unsigned long long* sorted = sort_keys(ctx, keys, n, p->n_keys);
        hipLaunchKernelGGL(k_intern, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, sorted, n, g, t, cols, saved, status);
        JG_HIP(hipGetLastError());
        const Status st = read_status(ctx, status);
        if (st.resolve_bad != ~0ull) {
            hipLaunchKernelGGL(k_rollback, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, sorted, n, t, saved);
            JG_HIP(hipStreamSynchronize(ctx->stream));
            jg::fail(JG_ESTATE, "jg_pnc_intern: entry %llu: its key holds more replicas than the store's columns",
                     (unsigned long long)(st.resolve_bad >> 2));
        }
        JG_HIP(hipMemcpyAsync(col_out, cols, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_columns(jg_pnc* p, uint64_t n, const uint32_t* key_idx, jg_guid* replicas, uint32_t* ncols) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_columns: store is NULL");
        if (n == 0) return;
        JG_REQUIRE(key_idx && replicas && ncols, JG_EINVAL, "jg_pnc_columns: NULL argument");
        for (uint64_t i = 0; i < n; ++i)
            JG_REQUIRE(key_idx[i] < p->n_keys, JG_EINVAL, "jg_pnc_columns: key_idx[%llu] = %u out of range", (unsigned long long)i, key_idx[i]);
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        ensure_table(p);
        char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * (4 + 4 + 16ull * p->R) + 256));
        auto* rows = reinterpret_cast<uint32_t*>(s);
        auto* nout = rows + n;
        auto* out = reinterpret_cast<Guid16*>(s + ((n * 8 + 15) & ~15ull));
        JG_HIP(hipMemcpyAsync(rows, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_gather_cols, dim3(blocks_for(n * p->R)), dim3(kBlock), 0, ctx->stream, p->cols.as<Guid16>(), p->ncols.as<uint32_t>(),
                           rows, n, p->R, out, nout);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(replicas, out, n * 16ull * p->R, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(ncols, nout, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_wave_create(jg_ctx* ctx, uint64_t cap_msgs, uint64_t cap_bytes, jg_wave** out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_wave_create: NULL argument");
        JG_REQUIRE(cap_msgs < 0xFFFFFFFFull, JG_EINVAL, "jg_wave_create: at most 2^32-2 messages per wave");
        jg::ensure_device(ctx);
        auto* w = new jg_wave();
        w->ctx = ctx;
        w->cap_msgs = cap_msgs;
        w->cap_bytes = cap_bytes;
        try {
            w->bytes.alloc(((cap_bytes + 15) & ~15ull) + 16);  // the parser reads aligned 16-byte windows
            w->off.alloc((cap_msgs + 1) * 8);
            w->keys.alloc(cap_msgs * 4 + 4);
        } catch (...) {
            delete w;
            throw;
        }
        *out = w;
    });
}

int jg_wave_destroy(jg_wave* w) {
    return jg::guard([&] {
        auto lk_ = jg::lock(w);  // calls on one context are serialised (shared scratch, stream)
        if (!w) return;
        jg::ensure_device(w->ctx);
        JG_HIP(hipStreamSynchronize(w->ctx->stream));
        delete w;
    });
}

int jg_wave_upload(jg_wave* w, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(w);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(w && key_idx && off && (bytes || n == 0), JG_EINVAL, "jg_wave_upload: NULL argument");
        JG_REQUIRE(n <= w->cap_msgs && off[n] <= w->cap_bytes, JG_EINVAL, "jg_wave_upload: wave exceeds the capacity");
        JG_REQUIRE(off[0] == 0, JG_EINVAL, "jg_wave_upload: off[0] must be 0");
        uint32_t mx = 0;
        for (uint64_t i = 0; i < n; ++i) {
            JG_REQUIRE(off[i + 1] >= off[i], JG_EINVAL, "jg_wave_upload: offsets decrease at message %llu", (unsigned long long)i);
            mx = key_idx[i] > mx ? key_idx[i] : mx;
        }
        jg_ctx* ctx = w->ctx;
        jg::ensure_device(ctx);
        if (off[n]) JG_HIP(hipMemcpyAsync(w->bytes.p, bytes, off[n], hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(w->off.p, off, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        if (n) JG_HIP(hipMemcpyAsync(w->keys.p, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        w->n = n;
        w->n_bytes = off[n];
        w->max_key = mx;
    });
}

int jg_pnc_merge_wave(jg_pnc* p, const jg_wave* w, uint64_t* bad_msg) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_merge_wave");
        if (bad_msg) *bad_msg = UINT64_MAX;
        JG_REQUIRE(p && w, JG_EINVAL, "jg_pnc_merge_wave: NULL argument");
        JG_REQUIRE(p->ctx == w->ctx, JG_EINVAL, "jg_pnc_merge_wave: wave and store belong to different contexts");
        if (w->n == 0) return;
        JG_REQUIRE(w->max_key < p->n_keys, JG_EINVAL, "jg_pnc_merge_wave: wave addresses key %u >= n_keys %llu", w->max_key,
                   (unsigned long long)p->n_keys);
        jg::ensure_device(p->ctx);
        merge_wave_dev(p, w->bytes.as<uint8_t>(), w->off.as<uint64_t>(), w->keys.as<uint32_t>(), w->n, bad_msg);
    });
}

int jg_pnc_wave_begin(jg_pnc* p, uint64_t cap_msgs, uint64_t cap_bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_wave_begin");
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_wave_begin: store is NULL");
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        ensure_table(p);
        grow_keep(ctx, p->wbytes, ((cap_bytes + 15) & ~15ull) + 16, 0);
        grow_keep(ctx, p->woff, (cap_msgs + 1) * 8, 0);
        grow_keep(ctx, p->wrows, cap_msgs * 4 + 4, 0);
        const WaveScratch w = wave_scratch(p, cap_msgs);
        begin_status(p, w.status);
        p->scan_hi = 0;
        p->fuse = json_fuse();
        JG_HIP(hipMemsetAsync(p->woff.p, 0, 8, ctx->stream));  // off[0] = 0
        p->wn = 0;
        p->wnb = 0;
        p->wopen = true;
    });
}

int jg_pnc_wave_append(jg_pnc* p, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_wave_append");
        JG_REQUIRE(p && p->wopen, JG_EINVAL, "jg_pnc_wave_append: no open wave (jg_pnc_wave_begin)");
        if (n == 0) return;
        JG_REQUIRE(key_idx && off && bytes, JG_EINVAL, "jg_pnc_wave_append: NULL argument");
        check_wave_host(p, n, key_idx, off, "jg_pnc_wave_append");
        JG_REQUIRE(p->wn + n < 0xFFFFFFFFull, JG_EINVAL, "jg_pnc_wave_append: at most 2^32-2 messages per wave");
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        const uint64_t m0 = p->wn, b0 = p->wnb, nb = off[n];
        // grow (rare: the caller's capacity hint was short); earlier chunks are kept
        if (p->wbytes.bytes < ((b0 + nb + 15) & ~15ull) + 16 || p->woff.bytes < (m0 + n + 1) * 8 || p->wrows.bytes < (m0 + n) * 4 + 4) {
            const uint64_t need_m = 2 * (m0 + n), need_b = 2 * (b0 + nb);
            grow_keep(ctx, p->wbytes, ((need_b + 15) & ~15ull) + 16, b0);
            grow_keep(ctx, p->woff, (need_m + 1) * 8, (m0 + 1) * 8);
            grow_keep(ctx, p->wrows, need_m * 4 + 4, m0 * 4);
        }
        const WaveScratch w = wave_scratch(p, m0 + n, m0);  // keeps the entries earlier chunks deferred
        if (nb) JG_HIP(hipMemcpyAsync(p->wbytes.as<uint8_t>() + b0, bytes, nb, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(p->woff.as<uint64_t>() + m0 + 1, off + 1, n * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(p->wrows.as<uint32_t>() + m0, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
        if (b0) hipLaunchKernelGGL(k_rebase, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, p->woff.as<uint64_t>() + m0 + 1, n, b0);
        launch_scan(p, p->wbytes.as<uint8_t>(), p->woff.as<uint64_t>(), p->wrows.as<uint32_t>(), m0, m0 + n, w);
        p->wn = m0 + n;
        p->wnb = b0 + nb;
    });
}

int jg_pnc_wave_commit(jg_pnc* p, uint64_t* bad_msg) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_wave_commit");
        if (bad_msg) *bad_msg = UINT64_MAX;
        JG_REQUIRE(p && p->wopen, JG_EINVAL, "jg_pnc_wave_commit: no open wave (jg_pnc_wave_begin)");
        jg::ensure_device(p->ctx);
        p->wopen = false;
        if (p->wn == 0) return;
        finish_wave(p, p->wbytes.as<uint8_t>(), p->woff.as<uint64_t>(), p->wrows.as<uint32_t>(), p->wn, wave_scratch(p, p->wn), bad_msg);
    });
}

int jg_pnc_wave_abort(jg_pnc* p) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_wave_abort");
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_wave_abort: store is NULL");
        jg::ensure_device(p->ctx);
        if (p->wopen) undo_applied(p, p->wrows.as<uint32_t>());  // the appended chunks' fused pass A
        p->scan_hi = 0;
        JG_HIP(hipStreamSynchronize(p->ctx->stream));
        p->wopen = false;
    });
}

int jg_pnc_merge_json(jg_pnc* p, uint64_t n, const uint32_t* key_idx, const uint64_t* off, const uint8_t* bytes, uint64_t* bad_msg) {
    auto lk_ = jg::lock(p);  // the whole begin/append/commit sequence under the context lock
    if (bad_msg) *bad_msg = UINT64_MAX;
    if (p && n && off) {
        int rc = jg_pnc_wave_begin(p, n, off[n]);
        if (rc == JG_OK) rc = jg_pnc_wave_append(p, n, key_idx, off, bytes);
        if (rc != JG_OK) {
            char keep[1024];
            jg_last_error(keep, sizeof keep);
            jg_pnc_wave_abort(p);
            return jg::guard([&] { jg::fail(rc, "%s", keep); });
        }
        return jg_pnc_wave_commit(p, bad_msg);
    }
    return jg::guard([&] {
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_merge_json: store is NULL");
        JG_REQUIRE(n == 0, JG_EINVAL, "jg_pnc_merge_json: NULL argument");
    });
}

int jg_host_alloc(jg_ctx* ctx, uint64_t bytes, void** out) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && out, JG_EINVAL, "jg_host_alloc: NULL argument");
        jg::ensure_device(ctx);
        *out = nullptr;
        if (bytes == 0) return;
        JG_HIP(hipHostMalloc(out, bytes, hipHostMallocDefault));
    });
}

int jg_host_free(void* p) {
    return jg::guard([&] {
        if (p) JG_HIP(hipHostFree(p));
    });
}

namespace {
// ---- SafeCRDT.Update's rewinds on the device (jg_pnc_apply_ops_rewind) -------------------------------------------
// A batch of own-column client ops applied at once (PNCounters.cs:96-112), and for every op whose snapshot ships
// (SafeCRDT.cs:39-62), the amounts the batch's LATER ops on the same key added to P (Increment) and N (Decrement):
// jg_pnc_encode_json_before rewinds the row by them.  Keys are made in reverse op order and sorted stably on the row
// bits, so each key's ops sit together newest first, and an exclusive segmented sum over that order is exactly the
// later ops' amounts (wrapping, as the host's walk of round 5 summed them: 13-18 ms of host time per 1M C5 ops).
struct PN2 { unsigned long long p, n; };
struct PN2Add {
    __host__ __device__ PN2 operator()(const PN2& a, const PN2& b) const { return PN2{a.p + b.p, a.n + b.n}; }
};

__global__ void k_make_keys_rev(const uint32_t* __restrict__ rows, uint64_t n, unsigned long long* __restrict__ keys) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < n) {
        const uint64_t i = n - 1 - j;
        keys[j] = (unsigned long long)rows[i] << 32 | i;
    }
}

// sorted position s: the op's amount on its vector (the store's width first, as the cells wrap), its key's row
__global__ void k_rewind_vals(const unsigned long long* __restrict__ sorted, uint64_t n, const long long* __restrict__ delta,
                              const uint8_t* __restrict__ is_n, uint32_t eb, PN2* __restrict__ vals, uint32_t* __restrict__ seg) {
    const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const uint32_t i = (uint32_t)sorted[s];
    const unsigned long long a = (unsigned long long)(eb == 4 ? (long long)(int)delta[i] : delta[i]);
    vals[s] = is_n[i] ? PN2{0, a} : PN2{a, 0};
    seg[s] = (uint32_t)(sorted[s] >> 32);
}

__global__ void k_flags_u32(const uint8_t* __restrict__ f, uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) out[i] = f[i] ? 1u : 0u;
}

// the needed ops' rewinds into need order (need_pos = exclusive count of needed ops before op i)
__global__ void k_rewind_scatter(const unsigned long long* __restrict__ sorted, uint64_t n, const PN2* __restrict__ later,
                                 const uint8_t* __restrict__ need, const uint32_t* __restrict__ need_pos, long long* __restrict__ dp,
                                 long long* __restrict__ dn) {
    const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const uint32_t i = (uint32_t)sorted[s];
    if (!need[i]) return;
    dp[need_pos[i]] = (long long)later[s].p;
    dn[need_pos[i]] = (long long)later[s].n;
}

// op i's snapshot from the row as it stands BEFORE the batch (jg_pnc_apply_ops_encode): the key's ops up to and
// including i added to it, i.e. minus the rewind k_encode subtracts.  `excl` is the exclusive segmented sum over the
// stably sorted (forward) order, `vals` each op's own amount.
__global__ void k_prefix_scatter(const unsigned long long* __restrict__ sorted, uint64_t n, const PN2* __restrict__ vals,
                                 const PN2* __restrict__ excl, long long* __restrict__ dp, long long* __restrict__ dn) {
    const uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const uint32_t i = (uint32_t)sorted[s];
    dp[i] = (long long)(0ull - (excl[s].p + vals[s].p));
    dn[i] = (long long)(0ull - (excl[s].n + vals[s].n));
}

// jg_pnc_encode_json(_before): length pass, scan, offsets to the host; with `out`, the write pass and its bytes.
void encode_rows(jg_pnc* p, uint64_t n, const uint32_t* key_idx, uint32_t col, const int64_t* dp, const int64_t* dn, uint64_t* off, uint8_t* out,
                 uint64_t cap, const char* fn, uint8_t* sha = nullptr) {
    JG_REQUIRE(p && off, JG_EINVAL, "%s: NULL argument", fn);
    off[0] = 0;
    if (n == 0) return;
    JG_REQUIRE(key_idx, JG_EINVAL, "%s: NULL key_idx", fn);
    JG_REQUIRE(n <= 0x7FFFFFFFull, JG_EINVAL, "%s: at most 2^31-1 rows per call", fn);
    for (uint64_t i = 0; i < n; ++i)
        JG_REQUIRE(key_idx[i] < p->n_keys, JG_EINVAL, "%s: key_idx[%llu] = %u out of range", fn, (unsigned long long)i, key_idx[i]);
    jg_ctx* ctx = p->ctx;
    jg::ensure_device(ctx);
    ensure_table(p);
    const Table t = table_of(p);
    char* s = static_cast<char*>(jg::scratch(ctx, ctx->scratch, n * 4 + (n + 1) * 16 + (dp ? n * 16 : 0) + 768));
    auto* rows = reinterpret_cast<uint32_t*>(s);
    auto* len = reinterpret_cast<unsigned long long*>(s + ((n * 4 + 255) & ~255ull));
    auto* doff = len + n + 1;
    long long* ddp = nullptr;
    long long* ddn = nullptr;
    JG_HIP(hipMemcpyAsync(rows, key_idx, n * 4, hipMemcpyHostToDevice, ctx->stream));
    if (dp) {
        ddp = reinterpret_cast<long long*>(doff + n + 1);
        ddn = ddp + n;
        JG_HIP(hipMemcpyAsync(ddp, dp, n * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(ddn, dn, n * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    const unsigned g = blocks_for(n);
    if (p->eb == 8) hipLaunchKernelGGL((k_encode<8, 0>), dim3(g), dim3(kBlock), 0, ctx->stream, rows, n, t, p->P.p, p->N.p, len, nullptr, col, ddp, ddn);
    else hipLaunchKernelGGL((k_encode<4, 0>), dim3(g), dim3(kBlock), 0, ctx->stream, rows, n, t, p->P.p, p->N.p, len, nullptr, col, ddp, ddn);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemsetAsync(len + n, 0, 8, ctx->stream));
    size_t temp = 0;
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, len, doff, (int)(n + 1), ctx->stream));
    void* tmp = jg::scratch(ctx, ctx->scratch3, temp + 256);
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, temp, len, doff, (int)(n + 1), ctx->stream));
    JG_HIP(hipMemcpyAsync(off, doff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    if (!out) return;  // size query
    JG_REQUIRE(off[n] <= cap, JG_ESTATE, "%s: %llu bytes exceed cap %llu", fn, (unsigned long long)off[n], (unsigned long long)cap);
    auto* dout = static_cast<uint8_t*>(jg::scratch(ctx, ctx->scratch2, off[n] + 64));
    const unsigned g1 = (unsigned)((n + kEncLanes - 1) / kEncLanes);  // the write pass: one wave per workgroup
    if (p->eb == 8) hipLaunchKernelGGL((k_encode<8, 1>), dim3(g1), dim3(kEncLanes), 0, ctx->stream, rows, n, t, p->P.p, p->N.p, doff, dout, col, ddp, ddn);
    else hipLaunchKernelGGL((k_encode<4, 1>), dim3(g1), dim3(kEncLanes), 0, ctx->stream, rows, n, t, p->P.p, p->N.p, doff, dout, col, ddp, ddn);
    JG_HIP(hipGetLastError());
    if (sha) jg::sha256_device(ctx, dout, reinterpret_cast<const uint64_t*>(doff), n, sha);  // each state's SHA-256 (ComputeDigest's first level)
    JG_HIP(hipMemcpyAsync(out, dout, off[n], hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
}
}  // namespace

int jg_pnc_apply_ops_rewind(jg_pnc* p, uint64_t n_ops, const uint32_t* key, uint32_t col, const int64_t* delta, const uint8_t* is_n,
                            const uint8_t* need, int64_t* dp, int64_t* dn) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(p, "jg_pnc_apply_ops_rewind");
        JG_REQUIRE(p, JG_EINVAL, "jg_pnc_apply_ops_rewind: store is NULL");
        if (n_ops == 0) return;
        JG_REQUIRE(key && delta && is_n && need && dp && dn, JG_EINVAL, "jg_pnc_apply_ops_rewind: NULL argument");
        JG_REQUIRE(col < p->R, JG_EINVAL, "jg_pnc_apply_ops_rewind: column %u past the store's %u replicas", col, p->R);
        JG_REQUIRE(n_ops <= 0x7FFFFFFFull, JG_EINVAL, "jg_pnc_apply_ops_rewind: at most 2^31-1 ops per call");
        uint64_t n_need = 0;
        for (uint64_t i = 0; i < n_ops; ++i) {
            JG_REQUIRE(key[i] < p->n_keys, JG_EINVAL, "jg_pnc_apply_ops_rewind: op %llu addresses key %u outside the store", (unsigned long long)i,
                       key[i]);
            n_need += need[i] != 0;
        }
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        using ull = unsigned long long;
        const uint64_t n = n_ops;
        auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
        // the ops (scratch2): key, delta, is_n, need, then the need positions
        const uint64_t o_del = al(n * 4), o_isn = o_del + al(n * 8), o_need = o_isn + al(n), o_pos = o_need + al(n), o_end = o_pos + al(n * 4);
        char* a = static_cast<char*>(jg::scratch(ctx, ctx->scratch2, o_end + 256));
        auto* dkey = reinterpret_cast<uint32_t*>(a);
        auto* ddel = reinterpret_cast<long long*>(a + o_del);
        auto* disn = reinterpret_cast<uint8_t*>(a + o_isn);
        auto* dneed = reinterpret_cast<uint8_t*>(a + o_need);
        auto* dpos = reinterpret_cast<uint32_t*>(a + o_pos);
        JG_HIP(hipMemcpyAsync(dkey, key, n * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(ddel, delta, n * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(disn, is_n, n, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(dneed, need, n, hipMemcpyHostToDevice, ctx->stream));
        // Increment / Decrement (k_apply_ops with every op on column col)
        const unsigned g = blocks_for(n);
        if (p->eb == 8) hipLaunchKernelGGL(k_apply_ops_col<8>, dim3(g), dim3(kBlock), 0, ctx->stream, p->P.p, p->N.p, dkey, col, ddel, disn, n, p->R);
        else hipLaunchKernelGGL(k_apply_ops_col<4>, dim3(g), dim3(kBlock), 0, ctx->stream, p->P.p, p->N.p, dkey, col, ddel, disn, n, p->R);
        JG_HIP(hipGetLastError());
        if (n_need == 0) {
            JG_HIP(hipStreamSynchronize(ctx->stream));
            return;
        }
        // the rewinds (scratch: keys, values, sums, segments, the scans' temp; sort_keys uses scratch3)
        const uint64_t o_val = al(n * 8), o_sum = o_val + al(n * 16), o_seg = o_sum + al(n * 16), o_dp = o_seg + al(n * 4),
                       o_tmp = o_dp + al(n_need * 16);
        size_t t_scan = 0, t_pos = 0;
        JG_HIP(hipcub::DeviceScan::ExclusiveScanByKey(nullptr, t_scan, (const uint32_t*)nullptr, (const PN2*)nullptr, (PN2*)nullptr, PN2Add(),
                                                      PN2{0, 0}, (int)n, hipcub::Equality(), ctx->stream));
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t_pos, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, ctx->stream));
        char* b = static_cast<char*>(jg::scratch(ctx, ctx->scratch, o_tmp + std::max(t_scan, t_pos) + 256));
        auto* keys = reinterpret_cast<ull*>(b);
        auto* vals = reinterpret_cast<PN2*>(b + o_val);
        auto* later = reinterpret_cast<PN2*>(b + o_sum);
        auto* seg = reinterpret_cast<uint32_t*>(b + o_seg);
        auto* ddp = reinterpret_cast<long long*>(b + o_dp);
        auto* ddn = ddp + n_need;
        void* tmp = b + o_tmp;
        // need positions first (the flags as u32 in `seg`: a scan of u8 would sum in u8), then the keys
        hipLaunchKernelGGL(k_flags_u32, dim3(g), dim3(kBlock), 0, ctx->stream, dneed, n, seg);
        size_t t = t_pos;
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, t, seg, dpos, (int)n, ctx->stream));
        hipLaunchKernelGGL(k_make_keys_rev, dim3(g), dim3(kBlock), 0, ctx->stream, dkey, n, keys);
        JG_HIP(hipGetLastError());
        const ull* sorted = sort_keys(ctx, keys, n, p->n_keys);
        hipLaunchKernelGGL(k_rewind_vals, dim3(g), dim3(kBlock), 0, ctx->stream, sorted, n, ddel, disn, p->eb, vals, seg);
        JG_HIP(hipGetLastError());
        t = t_scan;
        JG_HIP(hipcub::DeviceScan::ExclusiveScanByKey(tmp, t, seg, vals, later, PN2Add(), PN2{0, 0}, (int)n, hipcub::Equality(), ctx->stream));
        hipLaunchKernelGGL(k_rewind_scatter, dim3(g), dim3(kBlock), 0, ctx->stream, sorted, n, later, dneed, dpos, ddp, ddn);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemcpyAsync(dp, ddp, n_need * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(dn, ddn, n_need * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_apply_ops_encode(jg_pnc* p, uint64_t n_ops, const uint32_t* key, uint32_t col, const int64_t* delta, const uint8_t* is_n,
                            uint64_t* off, uint8_t* out, uint64_t cap, uint8_t* sha) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(p && off, JG_EINVAL, "jg_pnc_apply_ops_encode: NULL argument");
        jg::require_writable(p, "jg_pnc_apply_ops_encode");
        off[0] = 0;
        if (n_ops == 0) return;
        JG_REQUIRE(key && delta && is_n && out, JG_EINVAL, "jg_pnc_apply_ops_encode: NULL argument");
        JG_REQUIRE(col < p->R, JG_EINVAL, "jg_pnc_apply_ops_encode: column %u past the store's %u replicas", col, p->R);
        JG_REQUIRE(n_ops <= 0x7FFFFFFFull, JG_EINVAL, "jg_pnc_apply_ops_encode: at most 2^31-1 ops per call");
        for (uint64_t i = 0; i < n_ops; ++i)
            JG_REQUIRE(key[i] < p->n_keys, JG_EINVAL, "jg_pnc_apply_ops_encode: op %llu addresses key %u outside the store",
                       (unsigned long long)i, key[i]);
        jg_ctx* ctx = p->ctx;
        jg::ensure_device(ctx);
        ensure_table(p);
        const Table t = table_of(p);
        using ull = unsigned long long;
        const uint64_t n = n_ops;
        auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
        // everything but the sort (scratch3) and the bytes (scratch2) in ctx->scratch, sized once
        const uint64_t o_del = al(n * 4), o_isn = o_del + al(n * 8), o_k64 = o_isn + al(n), o_val = o_k64 + al(n * 8),
                       o_exc = o_val + al(n * 16), o_seg = o_exc + al(n * 16), o_dp = o_seg + al(n * 4), o_dn = o_dp + al(n * 8),
                       o_len = o_dn + al(n * 8), o_off = o_len + al((n + 1) * 8), o_tmp = o_off + al((n + 1) * 8);
        size_t t_scan = 0, t_sum = 0;
        JG_HIP(hipcub::DeviceScan::ExclusiveScanByKey(nullptr, t_scan, (const uint32_t*)nullptr, (const PN2*)nullptr, (PN2*)nullptr, PN2Add(),
                                                      PN2{0, 0}, (int)n, hipcub::Equality(), ctx->stream));
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t_sum, (const ull*)nullptr, (ull*)nullptr, (int)(n + 1), ctx->stream));
        char* a = static_cast<char*>(jg::scratch(ctx, ctx->scratch, o_tmp + std::max(t_scan, t_sum) + 256));
        auto* dkey = reinterpret_cast<uint32_t*>(a);
        auto* ddel = reinterpret_cast<long long*>(a + o_del);
        auto* disn = reinterpret_cast<uint8_t*>(a + o_isn);
        auto* keys = reinterpret_cast<ull*>(a + o_k64);
        auto* vals = reinterpret_cast<PN2*>(a + o_val);
        auto* excl = reinterpret_cast<PN2*>(a + o_exc);
        auto* seg = reinterpret_cast<uint32_t*>(a + o_seg);
        auto* ddp = reinterpret_cast<long long*>(a + o_dp);
        auto* ddn = reinterpret_cast<long long*>(a + o_dn);
        auto* len = reinterpret_cast<ull*>(a + o_len);
        auto* doff = reinterpret_cast<ull*>(a + o_off);
        void* tmp = a + o_tmp;
        JG_HIP(hipMemcpyAsync(dkey, key, n * 4, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(ddel, delta, n * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipMemcpyAsync(disn, is_n, n, hipMemcpyHostToDevice, ctx->stream));
        // each op's amounts up to and including it, per key (forward keys: a stable sort keeps op order per key)
        const unsigned g = blocks_for(n);
        hipLaunchKernelGGL(k_make_keys, dim3(g), dim3(kBlock), 0, ctx->stream, dkey, n, keys);
        JG_HIP(hipGetLastError());
        const ull* sorted = sort_keys(ctx, keys, n, p->n_keys);
        hipLaunchKernelGGL(k_rewind_vals, dim3(g), dim3(kBlock), 0, ctx->stream, sorted, n, ddel, disn, p->eb, vals, seg);
        JG_HIP(hipGetLastError());
        size_t tt = t_scan;
        JG_HIP(hipcub::DeviceScan::ExclusiveScanByKey(tmp, tt, seg, vals, excl, PN2Add(), PN2{0, 0}, (int)n, hipcub::Equality(), ctx->stream));
        hipLaunchKernelGGL(k_prefix_scatter, dim3(g), dim3(kBlock), 0, ctx->stream, sorted, n, vals, excl, ddp, ddn);
        JG_HIP(hipGetLastError());
        // the snapshots' lengths from the rows as they stand (nothing applied yet), their offsets to the host
        if (p->eb == 8) hipLaunchKernelGGL((k_encode<8, 0>), dim3(g), dim3(kBlock), 0, ctx->stream, dkey, n, t, p->P.p, p->N.p, len, nullptr, col, ddp, ddn);
        else hipLaunchKernelGGL((k_encode<4, 0>), dim3(g), dim3(kBlock), 0, ctx->stream, dkey, n, t, p->P.p, p->N.p, len, nullptr, col, ddp, ddn);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemsetAsync(len + n, 0, 8, ctx->stream));
        tt = t_sum;
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tt, len, doff, (int)(n + 1), ctx->stream));
        JG_HIP(hipMemcpyAsync(off, doff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        JG_REQUIRE(off[n] <= cap, JG_ESTATE, "jg_pnc_apply_ops_encode: %llu bytes exceed cap %llu (nothing applied)", (unsigned long long)off[n],
                   (unsigned long long)cap);
        // the bytes, then the ops (stream order: the write pass reads the rows before the adds land), the hashes
        auto* dout = static_cast<uint8_t*>(jg::scratch(ctx, ctx->scratch2, off[n] + 64));
        const unsigned g1 = (unsigned)((n + kEncLanes - 1) / kEncLanes);  // the write pass: one wave per workgroup
        if (p->eb == 8) {
            hipLaunchKernelGGL((k_encode<8, 1>), dim3(g1), dim3(kEncLanes), 0, ctx->stream, dkey, n, t, p->P.p, p->N.p, doff, dout, col, ddp, ddn);
            hipLaunchKernelGGL(k_apply_ops_col<8>, dim3(g), dim3(kBlock), 0, ctx->stream, p->P.p, p->N.p, dkey, col, ddel, disn, n, p->R);
        } else {
            hipLaunchKernelGGL((k_encode<4, 1>), dim3(g1), dim3(kEncLanes), 0, ctx->stream, dkey, n, t, p->P.p, p->N.p, doff, dout, col, ddp, ddn);
            hipLaunchKernelGGL(k_apply_ops_col<4>, dim3(g), dim3(kBlock), 0, ctx->stream, p->P.p, p->N.p, dkey, col, ddel, disn, n, p->R);
        }
        JG_HIP(hipGetLastError());
        if (sha) jg::sha256_device(ctx, dout, reinterpret_cast<const uint64_t*>(doff), n, sha);
        JG_HIP(hipMemcpyAsync(out, dout, off[n], hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_pnc_encode_json(jg_pnc* p, uint64_t n, const uint32_t* key_idx, uint64_t* off, uint8_t* out, uint64_t cap) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);  // calls on one context are serialised (shared scratch, stream)
        encode_rows(p, n, key_idx, 0, nullptr, nullptr, off, out, cap, "jg_pnc_encode_json");
    });
}

int jg_pnc_encode_json_before(jg_pnc* p, uint64_t n, const uint32_t* key_idx, uint32_t col, const int64_t* dp, const int64_t* dn, uint64_t* off,
                              uint8_t* out, uint64_t cap, uint8_t* sha) {
    return jg::guard([&] {
        auto lk_ = jg::lock(p);
        JG_REQUIRE(p && (n == 0 || (dp && dn)), JG_EINVAL, "jg_pnc_encode_json_before: NULL argument");
        JG_REQUIRE(col < p->R, JG_EINVAL, "jg_pnc_encode_json_before: column %u past the store's %u replicas", col, p->R);
        encode_rows(p, n, key_idx, col, dp, dn, off, out, cap, "jg_pnc_encode_json_before", out ? sha : nullptr);
    });
}

}  // extern "C"
