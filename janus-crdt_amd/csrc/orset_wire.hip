// orset_wire.hip — committed OR-Set states applied straight from their wire bytes (SURVEY.md §8f F1 + A7/A13).
//
// The reference's stable apply decodes every committed OR-Set state with System.Text.Json and merges it:
// SafeCRDT.ApplyUpdateStable (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:80-83) -> ORSet.DecodePropagationMessage
// (MergeSharp/MergeSharp/CRDTs/ORSet.cs:297-302) -> ORSetMsg.Decode (:56-69) -> ORSet.Merge (:253-283), one
// state at a time inside HandleAfterConsensusUpdates (SafeCRDTManager.cs:109-160).  The store's records are
// (set << 32 | element id, 16-byte tag), so element STRINGS must become ids first.  A wave is:
//
//   pass 1  k_ow_parse   one thread per message, launched per uploaded chunk: full parse + validation (the
//                        accepted form of oracle/json.hpp, which host/wire.cpp's reader also follows); the
//                        byte position of the first error: a syntax error (JG_EINVAL) or an element with an
//                        empty add or tombstone tag set (JG_ESTATE: no ORSet op produces one, and the
//                        record layout cannot hold the Dictionary key it would add); one entry per
//                        (message, map, element) with a 64-bit hash of its unescaped string (escaped
//                        strings unescaped in place) and one record per tag, into regions addressed by
//                        the message's byte offset (no wave-wide prefix needed yet).
//   compact scan of the per-message counts (hipcub), then k_ow_compact: entries numbered in commit order
//                        with addSet entries before removeSet ones (Merge walks addSet first,
//                        ORSet.cs:255-279).
//   sort    entries by the low 32 bits of their (set, string) hash, stable (hipcub radix sort): commit
//                        order within a hash.
//   group   k_ow_link / k_ow_label label every entry with the first entry of its string in the set,
//                        strings compared byte for byte (a hash collision only takes a slower path).  The
//                        same string twice in one map of one message is Decode's duplicate-key error
//                        (JG_EINVAL at the second name).  First bad message = min over messages.
//   commit(limit)   strings whose first entry precedes the limit are looked up in the set's element
//                   table; new ones are ordered by (set, first entry) and take the set's next ids in that
//                   order = first insertion into the reference's Dictionaries.  Tag records get their keys,
//                   lose their repeats through a hash table (a full-state message repeats most of its
//                   set's records), are radix-sorted by (key, tag) and unioned into the store (orset.hip).
//
// Element table (per store, first use): open addressing over 64-bit words (hash high half << 32 | name
// index + 1; 0 = empty), names as (set, id, Clear generation, length, pool offset, hash), bytes in a pool.
// A name is live while its generation equals its set's (a Clear bumps the set's generation).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "jg_internal.hpp"
#include "wire_cursor.hpp"

namespace {

using jgw::Cursor;
using jgw::hexv;
using jgw::GuidSink;
using jgw::read_string;
using jgw::put_utf8;

constexpr int kBlock = 256;
constexpr unsigned long long kNone = ~0ull;
constexpr unsigned long long kKindState = 1, kKindInval = 2;  // error word = position << 2 | kind
constexpr uint32_t kDead = 0xFFFFFFFFu;                        // id of an entry at or beyond the limit
constexpr uint32_t kNoName = 0xFFFFFFFFu;

struct Tag16 { unsigned long long lo, hi; };

unsigned blocks_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, (n + kBlock - 1) / kBlock); }

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull, kFnvPrime = 0x100000001b3ull;
// (set, string) key of an element name: the string's FNV-1a mixed with its set and the store's random salt
// (drawn at the store's first wave), so a peer cannot aim names at one value of the sort's low 32 bits
__device__ __forceinline__ uint64_t name_key(uint32_t set, uint64_t fnv, uint64_t salt) {
    return mix64(fnv ^ mix64((uint64_t)set + salt));
}

// ---- string sinks: read_string feeds each unescaped UTF-8 byte to put(), esc() at a backslash -------
__constant__ char kProp[4][16] = {"addSet", "removeSet", "nullAddGuid", "nullRemoveGuid"};
__constant__ uint32_t kPropLen[4] = {6, 9, 11, 14};

struct PropSink {  // which of the four ORSetMsg members (after unescaping, as System.Text.Json matches)
    uint32_t len = 0, mask = 15;
    __device__ void esc() {}
    __device__ void put(int b) {
        for (int k = 0; k < 4; ++k)
            if ((mask >> k & 1) && (len >= kPropLen[k] || kProp[k][len] != (char)b)) mask &= ~(1u << k);
        ++len;
    }
    __device__ int which() const {
        for (int k = 0; k < 4; ++k)
            if ((mask >> k & 1) && kPropLen[k] == len) return k;
        return -1;
    }
};

struct NameSink {  // FNV-1a of the unescaped bytes and the first 8 of them; with w set, the bytes after the
                   // first escape are written back at the string's start (unescaping never lengthens a string)
    unsigned long long h = kFnvBasis, pf = 0;
    uint32_t len = 0;
    uint8_t* w = nullptr;
    bool shifted = false;
    __device__ void esc() { shifted = w != nullptr; }
    __device__ void put(int b) {
        h = (h ^ (uint32_t)b) * kFnvPrime;
        if (len < 8) pf |= (unsigned long long)(uint8_t)b << (8 * len);
        if (shifted) w[len] = (uint8_t)b;
        ++len;
    }
};

// The common case of a tag string, decoded without the byte loop: [p, p + 37) holds exactly the
// 36-character "D" form with hex digits and the closing quote.  Eleven independent dword loads cover it
// (the payload buffer's 16-byte tail pad keeps them in bounds), v_alignbyte shifts them to p, and every
// digit is checked and decoded at a fixed position.  Anything else (an escape, a bad digit, a string
// running past the payload) returns false before the cursor moves, and the byte-wise GuidSink path
// then reads the same bytes and reports the same error position.
__device__ __forceinline__ bool guid_fast(const uint8_t* __restrict__ base, uint64_t p, uint64_t end, Tag16& t) {
    if (p + 37 > end) return false;
    const uint64_t a = p & ~3ull;
    const uint32_t s = (uint32_t)(p - a);
    const uint32_t* d = reinterpret_cast<const uint32_t*>(base + a);
    uint32_t raw[11];
#pragma unroll
    for (int i = 0; i < 11; ++i) raw[i] = d[i];
    uint32_t w[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) w[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], s);
    uint32_t bad = 0;
    auto byte = [&](int k) -> uint32_t { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; };
    auto hx = [&](int k) -> uint32_t {
        const uint32_t b = byte(k), dg = b - '0', lt = (b | 0x20u) - 'a';
        const bool isd = dg < 10u;
        bad |= (uint32_t)(!isd && lt >= 6u);
        return isd ? dg : lt + 10u;
    };
    bad |= (byte(8) ^ '-') | (byte(13) ^ '-') | (byte(18) ^ '-') | (byte(23) ^ '-') | (byte(36) ^ '"');
    uint32_t va = 0, vb = 0, vc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) va = va << 4 | hx(k);
#pragma unroll
    for (int k = 9; k < 13; ++k) vb = vb << 4 | hx(k);
#pragma unroll
    for (int k = 14; k < 18; ++k) vc = vc << 4 | hx(k);
    unsigned long long hi = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {  // GuidSink's order: byte j/2 of hi, high nibble first
        const int k = j < 4 ? 19 + j : 20 + j;
        hi |= (unsigned long long)hx(k) << (8 * (j >> 1) + ((j & 1) ? 0 : 4));
    }
    t = Tag16{(unsigned long long)va | (unsigned long long)vb << 32 | (unsigned long long)vc << 48, hi};
    return bad == 0;
}

// A tag array after its '['.  Null tag sets (nullAddGuid / nullRemoveGuid) report is_null.
template <class V> __device__ __forceinline__ bool read_tags(Cursor& c, V& v, int side, bool is_null, uint32_t& nt) {
    nt = 0;
    c.ws();
    if (c.peek() == ']') { ++c.p; return true; }
    for (;;) {
        if (!c.expect('"')) return false;
        Tag16 g;
        if (guid_fast(c.base, c.p, c.end, g)) {
            c.p += 37;
            v.tag(side, is_null, g);
            ++nt;
            c.ws();
            const int ch = c.get();
            if (ch == ']') return true;
            if (ch != ',') return false;
            continue;
        }
        GuidSink gs;
        if (!read_string(c, gs) || !gs.ok()) return false;
        v.tag(side, is_null, Tag16{gs.lo(), gs.hi});
        ++nt;
        c.ws();
        const int ch = c.get();
        if (ch == ']') return true;
        if (ch != ',') return false;
    }
}

// ---- the decode contract (oracle/json.hpp, System.Text.Json 6.0's defaults) ---------------------------------------
// Members in any order; a name that is not a member is skipped (jgw::skip_value); a member given twice takes its
// last occurrence; an element named twice in one map keeps its first place and takes its last tag set (Dictionary's
// indexer); a `null` last occurrence of a member or an element is rejected (Merge would throw).

// Per member over the whole message: occurrences, the last one `null`, and (maps) whether its last occurrence may
// name an element twice (a 128-bit filter of the names' hashes: no shared bit, no repeat, no scans).
struct MemInfo {
    uint32_t occ = 0;
    bool null_last = false, maybe_dup = false;
};

struct NoTags {  // read_tags' visitor for a validation pass
    __device__ __forceinline__ void tag(int, bool, const Tag16&) {}
};

// The whole payload checked, every occurrence of every member (skipped ones included): true iff System.Text.Json
// decodes it and no member ends `null`.  Writes nothing.
__device__ bool validate_orset(Cursor& c, MemInfo (&mi)[4]) {
    if (!c.expect('{')) return false;
    c.ws();
    if (c.peek() == '}') return false;  // {}: every member missing
    NoTags nv;
    for (;;) {
        if (!c.expect('"')) return false;
        PropSink ps;
        if (!read_string(c, ps) || !c.expect(':')) return false;
        const int which = ps.which();
        if (which < 0) {
            if (!jgw::skip_value(c, 1)) return false;
        } else {
            MemInfo& v = mi[which];
            ++v.occ;
            v.maybe_dup = false;
            c.ws();
            v.null_last = c.peek() == 'n';
            uint32_t nt;
            if (v.null_last) {
                if (!jgw::take_literal(c, "null")) return false;
            } else if (which >= 2) {
                if (!c.expect('[') || !read_tags(c, nv, 0, true, nt)) return false;
            } else {
                if (!c.expect('{')) return false;
                unsigned long long f0 = 0, f1 = 0;
                c.ws();
                if (c.peek() == '}') {
                    ++c.p;
                } else {
                    for (;;) {
                        NameSink ns;
                        if (!c.expect('"') || !read_string(c, ns) || !c.expect(':')) return false;
                        c.ws();
                        if (c.peek() == 'n') {  // a null tag set: valid JSON, judged by the visiting pass if it is the last
                            if (!jgw::take_literal(c, "null")) return false;
                        } else if (!c.expect('[') || !read_tags(c, nv, 0, false, nt)) {
                            return false;
                        }
                        const uint32_t h = (uint32_t)(ns.h * 0x9E3779B97F4A7C15ull >> 57);  // 7 bits
                        const unsigned long long b = 1ull << (h & 63);
                        v.maybe_dup |= (h & 64) ? (f1 & b) != 0 : (f0 & b) != 0;
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
    if (c.p != c.end) return false;
    for (int k = 0; k < 4; ++k)
        if (!mi[k].occ || mi[k].null_last) return false;
    return true;
}

// A name's unescaped bytes compared with `want` (len bytes) as they are decoded.
struct CmpSink {
    const uint8_t* want;
    uint32_t len, k = 0;
    bool eq = true;
    __device__ void esc() {}
    __device__ void put(int b) {
        eq &= k < len && want[k] == (uint8_t)b;
        ++k;
    }
    __device__ bool same() const { return eq && k == len; }
};

// One ORSetMsg<string> as System.Text.Json decodes it: the last occurrence of each member visited (v.map / v.entry /
// v.tag / v.entry_end), an element named twice in one map visited once, at its first place, with the tags of its
// last occurrence — so entry and tag slots come in ORSet.Merge's walk order.  The payload is validated whole first;
// the visiting pass can still fail on an element whose last tag set is `null`.  W: unescape element strings in
// place (pass 2).
template <bool W, class V> __device__ __forceinline__ bool parse_orset(Cursor& c, uint8_t* wbase, V& v) {
    MemInfo mi[4];
    {
        Cursor t = c;
        if (!validate_orset(t, mi)) {
            c = t;
            return false;
        }
    }
    uint32_t occ[4] = {0, 0, 0, 0};
    (void)c.expect('{');
    for (;;) {
        (void)c.expect('"');
        PropSink ps;
        (void)read_string(c, ps);
        (void)c.expect(':');
        const int which = ps.which();
        if (which < 0 || ++occ[which] < mi[which].occ) {
            (void)jgw::skip_value(c, 1);  // validated: a skipped member, or an occurrence a later one replaces
        } else if (which >= 2) {
            uint32_t nt;
            (void)c.expect('[');
            (void)read_tags(c, v, which - 2, true, nt);
        } else {
            (void)c.expect('{');
            v.map(which);
            c.ws();
            if (c.peek() == '}') {
                ++c.p;
            } else {
                const bool dups = mi[which].maybe_dup;
                const uint32_t e0 = v.entries();  // this map's first entry (a repeat looks among e0 ..)
                for (;;) {
                    c.ws();
                    const uint64_t npos = c.p;
                    ++c.p;  // the opening quote
                    const uint64_t noff = c.p;
                    NameSink ns;
                    if (W) ns.w = wbase + noff;
                    (void)read_string(c, ns);
                    (void)c.expect(':');
                    Cursor val = c;  // the tag set this entry takes (the element's last occurrence's)
                    bool first = true;
                    if (dups) {
                        first = !v.named_before(e0, ns, c.base, noff);
                        if (first) {
                            Cursor t = c;
                            (void)jgw::skip_value(t, 2);
                            for (;;) {
                                t.ws();
                                if (t.get() != ',') break;
                                CmpSink cs{c.base + noff, ns.len};
                                (void)t.expect('"');
                                (void)read_string(t, cs);
                                (void)t.expect(':');
                                if (cs.same()) val = t;
                                (void)jgw::skip_value(t, 2);
                            }
                        }
                    }
                    if (first) {
                        val.ws();
                        if (val.peek() != '[') {  // the element's last tag set is null: UnionWith(null) throws
                            c = val;
                            return false;
                        }
                        ++val.p;
                        v.entry(which, npos, noff, ns.len, ns.h, ns.pf);
                        uint32_t nt;
                        (void)read_tags(val, v, which, false, nt);
                        v.entry_end(which, val.p, nt);
                    }
                    (void)jgw::skip_value(c, 2);  // this occurrence's value
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

// Pass 1 writes each message's entries and tags into SPARSE regions addressed by its byte offset, so
// no prefix over the wave is needed before parsing: an entry needs >= 5 payload bytes after an 11-byte
// `{"addSet":{` prefix and a tag >= 38 bytes, so message m's entries fit in slots [ceil(off/4),
// ceil(off_next/4)) and its tags in [ceil(off/32), ceil(off_next/32)) whatever the payload holds.
// check() compacts them in commit order (k_ow_compact).
constexpr uint64_t kEntryDiv = 4, kTagDiv = 32;

struct Sparse {  // entry slots: sort key, string offset, length | side << 31, error position, the string's
                 // first 8 bytes (zero past its end); tag slots
    unsigned long long* key;
    unsigned long long* noff;
    unsigned long long* pfx;
    uint32_t* meta;
    uint32_t* pos;
    uint32_t* set;             // the message's set
    uint32_t* sid;             // the string's slot in the wave's string table (k_ow_strings)
    unsigned long long* tref;  // null << 63 | side << 62 | the entry's parse-order ordinal in its message
    Tag16* tval;
    unsigned long long* trk;   // the record's identity without its tag (k_ow_rkeys): sid << 1 | side, or
                               // 1 << 63 | set << 1 | side for a null tag set
};

struct ParseVis {
    Sparse S;
    uint64_t base, es, ts, kmask, salt;  // message byte offset; first entry / tag slot
    uint32_t set, n_add = 0, n_rem = 0, nt = 0, cur = 0;
    bool rem_first = false, add_seen = false;
    unsigned long long estate = kNone;
    __device__ __forceinline__ void map(int which) {
        if (which == 0) add_seen = true;
        else if (!add_seen) rem_first = true;
    }
    __device__ __forceinline__ void entry(int side, uint64_t npos, uint64_t noff, uint32_t len, uint64_t h, uint64_t pf) {
        cur = n_add + n_rem;
        const uint64_t e = es + cur;
        S.key[e] = name_key(set, h, salt) & kmask;
        S.noff[e] = noff;
        S.pfx[e] = pf;
        S.meta[e] = len | (uint32_t)side << 31;
        S.pos[e] = (uint32_t)(npos - base);
        S.set[e] = set;
        n_add += side == 0;
        n_rem += side != 0;
    }
    __device__ __forceinline__ void tag(int side, bool is_null, const Tag16& g) {
        S.tref[ts + nt] = (unsigned long long)is_null << 63 | (unsigned long long)side << 62 | cur;
        S.tval[ts + nt] = g;
        ++nt;
    }
    __device__ __forceinline__ void entry_end(int side, uint64_t pos, uint32_t ntags) {
        if (ntags == 0 && estate == kNone) estate = (unsigned long long)(pos - base) << 2 | kKindState;  // add or tombstone
    }
    __device__ __forceinline__ uint32_t entries() const { return n_add + n_rem; }
    // an entry of this map (entries e0 ..) already names the string ns decoded at payload offset noff (both unescaped
    // in place: parse_orset<true>)
    __device__ bool named_before(uint32_t e0, const NameSink& ns, const uint8_t* base, uint64_t noff) const {
        const unsigned long long key = name_key(set, ns.h, salt) & kmask;
        for (uint32_t q = e0; q < n_add + n_rem; ++q) {
            const uint64_t e = es + q;
            if (S.key[e] != key || (S.meta[e] & 0x7FFFFFFFu) != ns.len || S.pfx[e] != ns.pf) continue;
            bool same = true;
            for (uint32_t i = 8; i < ns.len && same; ++i) same = base[S.noff[e] + i] == base[noff + i];
            if (same) return true;
        }
        return false;
    }
};

// One thread per message: parse + validate (first error position: syntax or empty tag set), element
// strings hashed (escaped ones unescaped in place), entries and tags into the sparse regions.  The
// entries before a syntax error are kept: a repeated name before it is reported first.
__global__ __launch_bounds__(kBlock) void k_ow_parse(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, const uint32_t* __restrict__ mset,
                                                     uint64_t m0, uint64_t m1, Sparse S, uint64_t kmask, uint64_t salt, unsigned long long* __restrict__ ne,
                                                     unsigned long long* __restrict__ nt, uint32_t* __restrict__ na,
                                                     unsigned long long* __restrict__ err, const uint8_t* __restrict__ slow) {
    const uint64_t m = m0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (m >= m1 || (slow && !slow[m])) return;  // slow: the messages k_ow_group left to the serial parse
    if (mset[m] == jg::kSkipIdx) {  // another kind's message in a node wave (csrc/node.hip)
        ne[m] = nt[m] = 0;
        na[m] = 0;
        err[m] = kNone;
        return;
    }
    const uint64_t b = off[m];
    ParseVis v{S, b, (b + kEntryDiv - 1) / kEntryDiv, (b + kTagDiv - 1) / kTagDiv, kmask, salt, mset[m]};
    Cursor c(bytes, b, off[m + 1]);
    unsigned long long e = kNone;
    if (!parse_orset<true>(c, bytes, v)) e = (unsigned long long)(c.p - b) << 2 | kKindInval;
    if (v.estate < e) e = v.estate;
    ne[m] = v.n_add + v.n_rem;
    nt[m] = v.nt;
    na[m] = v.n_add | (v.rem_first ? 0x80000000u : 0u);
    err[m] = e;
}

#include "orset_group.hpp"

__global__ void k_ow_rebase(uint64_t* __restrict__ off, uint64_t n, uint64_t base) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) off[i] += base;
}

struct Entries {  // entry e: sort key, string (offset into the payload, length | side << 31), message, error position
    unsigned long long* key;
    uint32_t* val;
    unsigned long long* noff;
    uint32_t* msg;
    uint32_t* meta;
    uint32_t* pos;
    unsigned long long* pfx;  // the string's first 8 bytes (zero past its end): k_ow_link compares short strings here
    uint32_t* set;            // the message's set
};

// Sparse -> dense in commit order: entry ordinal = addSet entries first, then removeSet (Merge's walk),
// whatever the member order of the payload.  One wave per message, lanes over its entries and tags (a
// message's slots are contiguous on both sides: coalesced copies).
constexpr int kCompactMsgs = kBlock / 64;
__global__ __launch_bounds__(kBlock) void k_ow_compact(const uint64_t* __restrict__ off, uint64_t n, const unsigned long long* __restrict__ ne,
                                                       const unsigned long long* __restrict__ nt, const uint32_t* __restrict__ na,
                                                       const unsigned long long* __restrict__ eoff, const unsigned long long* __restrict__ toff,
                                                       const uint32_t* __restrict__ mset, const uint8_t* __restrict__ bytes, Sparse S, Entries E,
                                                       unsigned long long* __restrict__ tref, Tag16* __restrict__ tval) {
    const uint64_t m = (uint64_t)blockIdx.x * kCompactMsgs + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (m >= n) return;
    const uint64_t b = off[m], es = (b + kEntryDiv - 1) / kEntryDiv, ts = (b + kTagDiv - 1) / kTagDiv;
    const uint32_t cnt = (uint32_t)ne[m], n_add = na[m] & 0x7FFFFFFFu, n_rem = cnt - n_add;
    const bool rem_first = (na[m] >> 31) != 0;
    const uint64_t e0 = eoff[m], t0 = toff[m];
    auto canon = [&](uint32_t q) -> uint32_t { return !rem_first ? q : (q < n_rem ? n_add + q : q - n_rem); };
    const uint32_t set = mset[m];
    for (uint32_t q = lane; q < cnt; q += 64) {
        const uint64_t e = e0 + canon(q);
        const unsigned long long no = S.noff[es + q];
        const uint32_t meta = S.meta[es + q];
        E.key[e] = S.key[es + q];
        E.val[e] = (uint32_t)e;
        E.noff[e] = no;
        E.msg[e] = (uint32_t)m;
        E.meta[e] = meta;
        E.pos[e] = S.pos[es + q];
        E.pfx[e] = S.pfx[es + q];
        E.set[e] = set;
    }
    const uint32_t k = (uint32_t)nt[m];
    for (uint32_t q = lane; q < k; q += 64) {
        const unsigned long long r = S.tref[ts + q];
        tref[t0 + q] = (r >> 63) ? (r & (3ull << 62)) | m : e0 + canon((uint32_t)r);
        tval[t0 + q] = S.tval[ts + q];
    }
}

__device__ __forceinline__ bool same_bytes(const uint8_t* a, const uint8_t* b, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

__device__ __forceinline__ bool same_name(const Entries& E, const uint32_t* mset, const uint8_t* bytes, uint32_t a, uint32_t b) {
    const uint32_t la = E.meta[a] & 0x7FFFFFFFu, lb = E.meta[b] & 0x7FFFFFFFu;
    if (la != lb || E.set[a] != E.set[b] || E.pfx[a] != E.pfx[b]) return false;
    return la <= 8 || same_bytes(bytes + E.noff[a] + 8, bytes + E.noff[b] + 8, la - 8);
}

// Entries are sorted on the low sort_bits (32) of their 64-bit (set, string) key (half the radix passes
// of the full key); a run is one value of those bits, so two strings whose keys differ only above them
// share a run, which k_ow_link marks impure like any other collision.  Each entry keeps its full key for
// the element table.
__global__ void k_ow_head(const unsigned long long* __restrict__ skey, uint64_t n, unsigned long long run_mask, uint32_t* __restrict__ hs) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) hs[i] = (i == 0 || ((skey[i] ^ skey[i - 1]) & run_mask) != 0) ? (uint32_t)i : 0u;
}

// A run of equal hashes holding two different strings (a collision) is marked impure.
__global__ void k_ow_link(Entries E, const uint32_t* __restrict__ mset, const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ sval,
                          const uint32_t* __restrict__ seg, uint64_t n, uint8_t* __restrict__ impure) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || seg[i] == i) return;
    if (!same_name(E, mset, bytes, sval[i], sval[i - 1])) impure[seg[i]] = 1;
}

__device__ __forceinline__ void report_dup(const Entries& E, uint32_t e, unsigned long long* err) {
    atomicMin(err + E.msg[e], (unsigned long long)E.pos[e] << 2 | kKindInval);
}

// label[i] = sorted index of the first entry with the same (set, string).  Pure runs: the run's head
// (stable sort = commit order), and a repeat within one map of one message is adjacent to its twin.
// Impure runs (hash collision): a scan of the run before i.
// An impure run is scanned entry by entry (O(L) per entry); past scan_limit entries into such a run the
// kernel raises *long_run instead, and the caller sorts the entries again on their full 64-bit keys (runs
// then mix only strings whose whole keys collide) and labels once more without a limit.
__global__ void k_ow_label(Entries E, const uint32_t* __restrict__ mset, const uint8_t* __restrict__ bytes, const uint32_t* __restrict__ sval,
                           const uint32_t* __restrict__ seg, const uint8_t* __restrict__ impure, uint64_t n, uint32_t* __restrict__ label,
                           unsigned long long* __restrict__ err, uint32_t scan_limit, unsigned long long* __restrict__ long_run) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = seg[i], e = sval[i];
    if (!impure[s]) {
        label[i] = s;
        if (i > s) {
            const uint32_t p = sval[i - 1];
            if (E.msg[p] == E.msg[e] && (E.meta[p] >> 31) == (E.meta[e] >> 31)) report_dup(E, e, err);
        }
        return;
    }
    if (i - s > scan_limit) {
        *long_run = 1;
        return;
    }
    uint32_t lab = (uint32_t)i;
    bool dup = false;
    const unsigned long long ke = E.key[e];
    for (uint32_t j = s; j < i; ++j) {
        const uint32_t q = sval[j];
        if (E.key[q] != ke || !same_name(E, mset, bytes, e, q)) continue;  // whole keys first: bytes only on a full match
        if (lab == i) lab = j;
        dup |= E.msg[q] == E.msg[e] && (E.meta[q] >> 31) == (E.meta[e] >> 31);
    }
    label[i] = lab;
    if (dup) report_dup(E, e, err);
}

constexpr uint32_t kImpureScan = 64;  // entries of an impure run labelled by a scan before the full-key re-sort

__global__ void k_ow_first_bad(const unsigned long long* __restrict__ err, uint64_t n, unsigned long long* __restrict__ status) {
    const uint64_t m = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (m < n && err[m] != kNone) atomicMin(status, (unsigned long long)m);
}

// ---- element table ----------------------------------------------------------------------------------
struct Names {
    unsigned long long* tab;
    uint64_t mask;
    uint32_t *set, *id, *gen, *len;
    unsigned long long *off, *key;
    uint8_t* pool;
    uint32_t* set_gen;
    uint32_t* next_id;
    // (set, id) -> name index, for the encoder (jg_orset_encode_json): every name ever issued, dead ones too
    unsigned long long* ikey;  // (set << 32 | id) + 1; 0 = empty
    uint32_t* ival;            // the name's index g
    uint64_t imask;
};

__device__ __forceinline__ void tab_insert(const Names& N, uint64_t key, uint32_t g) {
    const unsigned long long word = (key >> 32) << 32 | (unsigned long long)(g + 1);
    for (uint64_t s = key & N.mask;; s = (s + 1) & N.mask)
        if (atomicCAS(N.tab + s, 0ull, word) == 0ull) return;
}

__device__ __forceinline__ void itab_insert(const Names& N, uint32_t set, uint32_t id, uint32_t g) {
    const unsigned long long k = ((unsigned long long)set << 32 | id) + 1;
    for (uint64_t s = mix64(k) & N.imask;; s = (s + 1) & N.imask)
        if (atomicCAS(N.ikey + s, 0ull, k) == 0ull) {
            N.ival[s] = g;
            return;
        }
}

// The name index of (set, id), or kNoName (a kernel after the inserting ones: no race).
__device__ __forceinline__ uint32_t itab_find(const Names& N, uint32_t set, uint32_t id) {
    const unsigned long long k = ((unsigned long long)set << 32 | id) + 1;
    for (uint64_t s = mix64(k) & N.imask;; s = (s + 1) & N.imask) {
        const unsigned long long w = N.ikey[s];
        if (w == k) return N.ival[s];
        if (w == 0) return kNoName;
    }
}

__device__ __forceinline__ uint32_t tab_find(const Names& N, uint64_t key, uint32_t set, const uint8_t* name, uint32_t len) {
    const uint32_t tag = (uint32_t)(key >> 32), gen = N.set_gen[set];
    for (uint64_t s = key & N.mask;; s = (s + 1) & N.mask) {
        const unsigned long long w = N.tab[s];
        if (w == 0) return kNoName;
        if ((uint32_t)(w >> 32) != tag) continue;
        const uint32_t g = (uint32_t)w - 1;
        if (N.set[g] != set || N.gen[g] != gen || N.len[g] != len || !same_bytes(N.pool + N.off[g], name, len)) continue;
        return N.id[g];
    }
}

__global__ void k_names_rebuild(Names N, uint64_t n_names) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g < n_names && N.gen[g] == N.set_gen[N.set[g]]) tab_insert(N, N.key[g], (uint32_t)g);
}

__global__ void k_itab_rebuild(Names N, uint64_t n_names) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g < n_names) itab_insert(N, N.set[g], N.id[g], (uint32_t)g);
}

__global__ void k_sets_update(Names N, const uint32_t* __restrict__ set, const uint32_t* __restrict__ next, const uint8_t* __restrict__ cleared, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (cleared[i]) N.set_gen[set[i]] += 1;
    N.next_id[set[i]] = next[i];
}

__global__ void k_names_put(Names N, uint64_t g0, uint64_t pool0, const uint32_t* __restrict__ nset, const uint32_t* __restrict__ nid,
                            const uint64_t* __restrict__ off, uint64_t n, uint64_t kmask, uint64_t salt) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t g = g0 + i;
    const uint32_t set = nset[i], len = (uint32_t)(off[i + 1] - off[i]);
    const uint8_t* b = N.pool + pool0 + off[i];
    uint64_t h = kFnvBasis;
    for (uint32_t k = 0; k < len; ++k) h = (h ^ b[k]) * kFnvPrime;
    const uint64_t key = name_key(set, h, salt) & kmask;
    N.set[g] = set;
    N.id[g] = nid[i];
    N.gen[g] = N.set_gen[set];
    N.len[g] = len;
    N.off[g] = pool0 + off[i];
    N.key[g] = key;
    tab_insert(N, key, (uint32_t)g);
    itab_insert(N, set, nid[i], (uint32_t)g);
}

// commit: each live group head looks its string up; new strings are marked (set << 32 | entry) at their
// sorted index.  Marks, not a wave-aggregated counter: every wave that met a new string took a returning
// atomic on one address, which serialised the grid there.
__global__ void k_ow_resolve(Entries E, const uint32_t* __restrict__ mset, const uint8_t* __restrict__ bytes, const unsigned long long* __restrict__ skey,
                             const uint32_t* __restrict__ sval, const uint32_t* __restrict__ label, uint64_t n, uint64_t limit, Names N,
                             uint32_t* __restrict__ gid, unsigned long long* __restrict__ newk) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool fresh = false;
    uint32_t e = 0, set = 0;
    if (i < n && label[i] == i) {
        e = sval[i];
        const uint32_t m = E.msg[e];
        if (m >= limit) {
            gid[i] = kDead;
        } else {
            set = mset[m];
            const uint32_t id = tab_find(N, skey[i], set, bytes + E.noff[e], E.meta[e] & 0x7FFFFFFFu);
            if (id != kNoName) gid[i] = id;
            else fresh = true;
        }
    }
    // new strings: marked in place (compacted by select_marked; their order is fixed later by the sort)
    if (i < n) newk[i] = fresh ? (unsigned long long)set << 32 | e : kNone;
}

// Keys of the compacted new-string marks (count on the device).
__global__ void k_ow_gather_new(const unsigned long long* __restrict__ newk, const uint32_t* __restrict__ idx,
                                const unsigned long long* __restrict__ count, unsigned long long* __restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j < *count) out[j] = newk[idx[j]];
}

__device__ __forceinline__ uint64_t set_begin(const unsigned long long* snk, uint64_t n, uint32_t set) {
    uint64_t lo = 0, hi = n;
    const unsigned long long x = (unsigned long long)set << 32;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (snk[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// New strings sorted by (set, first entry): the r-th new string of a set takes next_id + r.
__global__ void k_ow_assign(Entries E, const uint8_t* __restrict__ bytes, const unsigned long long* __restrict__ skey,
                            const unsigned long long* __restrict__ snk, const uint32_t* __restrict__ snv, uint64_t nnew, uint64_t g0, Names N,
                            uint32_t* __restrict__ gid, unsigned long long* __restrict__ status) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= nnew) return;
    const uint32_t set = (uint32_t)(snk[k] >> 32);
    const uint64_t r = k - set_begin(snk, nnew, set);
    const uint64_t id = (uint64_t)N.next_id[set] + r;
    if (id >= JG_NULL_ELEM - 1) atomicOr(status + 3, 1ull);
    const uint32_t i = snv[k], e = (uint32_t)(snk[k] & 0xFFFFFFFFull), len = E.meta[e] & 0x7FFFFFFFu;
    gid[i] = (uint32_t)id;
    const uint64_t g = g0 + k;
    const unsigned long long p = atomicAdd(status + 2, (unsigned long long)len);
    const uint8_t* src = bytes + E.noff[e];
    for (uint32_t q = 0; q < len; ++q) N.pool[p + q] = src[q];
    N.set[g] = set;
    N.id[g] = (uint32_t)id;
    N.gen[g] = N.set_gen[set];
    N.len[g] = len;
    N.off[g] = p;
    N.key[g] = skey[i];
    tab_insert(N, skey[i], (uint32_t)g);
    itab_insert(N, set, (uint32_t)id, (uint32_t)g);
}

__global__ void k_ow_next_ids(const unsigned long long* __restrict__ snk, uint64_t nnew, Names N) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= nnew) return;
    const uint32_t set = (uint32_t)(snk[k] >> 32);
    if (k + 1 < nnew && (uint32_t)(snk[k + 1] >> 32) == set) return;  // not the set's last new string
    N.next_id[set] += (uint32_t)(k + 1 - set_begin(snk, nnew, set));
}

__global__ void k_ow_entry_ids(const uint32_t* __restrict__ sval, const uint32_t* __restrict__ label, const uint32_t* __restrict__ gid, uint64_t n,
                               uint32_t* __restrict__ eid) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) eid[sval[i]] = gid[label[i]];
}

// Record keys of every tag (kNone beyond the limit) and its side (0 add, 1 tombstone).
__global__ void k_ow_rec_keys(Entries E, const uint32_t* __restrict__ mset, const unsigned long long* __restrict__ tref, const uint32_t* __restrict__ eid,
                              uint64_t nt, uint64_t limit, unsigned long long* __restrict__ rkey, uint8_t* __restrict__ rside) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= nt) return;
    const unsigned long long r = tref[t];
    uint32_t m, id, side;
    bool live;
    if (r >> 63) {  // a null tag set: no string to intern (kDead == JG_NULL_ELEM: test the limit only)
        m = (uint32_t)r;
        side = (uint32_t)(r >> 62 & 1);
        id = JG_NULL_ELEM;
        live = m < limit;
    } else {
        const uint32_t e = (uint32_t)r;
        m = E.msg[e];
        side = E.meta[e] >> 31;
        id = eid[e];
        live = m < limit && id != kDead;
    }
    rkey[t] = live ? ((unsigned long long)mset[m] << 32 | id) : kNone;
    rside[t] = (uint8_t)side;
}

__device__ __forceinline__ uint64_t rec_hash(unsigned long long k, const Tag16& g, uint32_t side) {
    return mix64(k ^ mix64(g.lo + side) ^ (g.hi * 0x9E3779B97F4A7C15ull));
}

// Distinct records: insert-if-absent into an open-addressing table of record indices (exact compare on a
// hash match); the copy that wins the slot marks itself with its side (fsel = 1 + side, compacted per
// side afterwards: a wave-aggregated counter per side had every wave wait on one of two addresses) and
// its table slot, and every copy lowers the slot's mint to its tag index: mint = the record's
// FIRST occurrence in commit order = its arrival ordinal (a HashSet keeps a tag where it was first
// inserted; tag indices run message after message, each message in its arrays' order).
__global__ __launch_bounds__(kBlock) void k_ow_dedup(const unsigned long long* __restrict__ rkey, const uint8_t* __restrict__ rside,
                                                     const Tag16* __restrict__ tval, uint64_t nt, unsigned long long* __restrict__ tab, uint64_t mask,
                                                     uint32_t* __restrict__ mint, uint8_t* __restrict__ fsel, uint32_t* __restrict__ fslot) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    bool fresh = false;
    uint32_t side = 0;
    unsigned long long k = kNone;
    Tag16 g{0, 0};
    uint64_t slot = 0;
    if (t < nt) {
        k = rkey[t];
        side = rside[t];
        g = tval[t];
    }
    if (k != kNone) {
        const uint64_t h = rec_hash(k, g, side);
        const unsigned long long word = (h >> 32) << 32 | (t + 1);
        for (uint64_t s = h & mask;; s = (s + 1) & mask) {
            // most records repeat one seen earlier in the wave: a plain load settles those without an
            // atomic (a slot never changes once set; a stale 0 only sends us to the CAS)
            unsigned long long w = tab[s];
            if (w == 0) {
                w = atomicCAS(tab + s, 0ull, word);
                if (w == 0) { fresh = true; slot = s; break; }
            }
            if ((w >> 32) != (h >> 32)) continue;
            const uint64_t u = (w & 0xFFFFFFFFull) - 1;
            const Tag16 o = tval[u];
            if (rkey[u] == k && rside[u] == side && o.lo == g.lo && o.hi == g.hi) { slot = s; break; }
        }
        // most copies arrive after the first (lower tag index, earlier block) has set the slot: a plain
        // read settles them without an atomic on what is often a hot address
        if (mint[slot] > (uint32_t)t) atomicMin(mint + slot, (uint32_t)t);
    }
    if (t < nt) {
        fsel[t] = fresh ? (uint8_t)(1 + side) : (uint8_t)0;
        fslot[t] = (uint32_t)slot;
    }
}

// The distinct records of one side, compacted (select_marked) in tag order: keys, tags, table slots.
__global__ void k_ow_gather_side(const uint32_t* __restrict__ idx, const unsigned long long* __restrict__ count,
                                 const unsigned long long* __restrict__ rkey, const Tag16* __restrict__ tval, const uint32_t* __restrict__ fslot,
                                 unsigned long long* __restrict__ dk, Tag16* __restrict__ dt, uint32_t* __restrict__ ds) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= *count) return;
    const uint32_t t = idx[j];
    dk[j] = rkey[t];
    dt[j] = tval[t];
    ds[j] = fslot[t];
}

struct IsNewAt {
    const unsigned long long* k;
    __host__ __device__ bool operator()(const uint32_t& i) const { return k[i] != kNone; }
};
struct OnSide {
    const uint8_t* fsel;
    uint8_t want;
    __host__ __device__ bool operator()(const uint32_t& t) const { return fsel[t] == want; }
};

__global__ void k_iota(uint32_t* __restrict__ p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}
// which: 0 tag.hi, 1 tag.lo, 2 key — the radix key of pass `which` through the current permutation
__global__ void k_gather_radix(const unsigned long long* __restrict__ dk, const Tag16* __restrict__ dt, const uint32_t* __restrict__ perm, uint64_t n,
                               int which, unsigned long long* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = perm[i];
    out[i] = which == 2 ? dk[p] : which == 1 ? dt[p].lo : dt[p].hi;
}
// Records sorted by key alone: each run of equal keys (one element's new tags, a handful) put in (tag.lo,
// tag.hi) order by its head thread (insertion sort over the permutation); a run longer than kRunFix
// raises *long_run and the caller sorts the whole side by all three words instead.
constexpr uint32_t kRunFix = 64;
__global__ void k_fix_runs(const unsigned long long* __restrict__ skey, const Tag16* __restrict__ dt, uint32_t* __restrict__ perm, uint64_t n,
                           unsigned long long* __restrict__ long_run) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || (i > 0 && skey[i] == skey[i - 1])) return;
    uint64_t j = i + 1;
    while (j < n && skey[j] == skey[i] && j - i <= kRunFix) ++j;
    if (j - i > kRunFix) {
        atomicOr(long_run, 1ull);
        return;
    }
    for (uint64_t a = i + 1; a < j; ++a) {
        const uint32_t x = perm[a];
        const Tag16 tx = dt[x];
        uint64_t b = a;
        while (b > i) {
            const Tag16 ty = dt[perm[b - 1]];
            if (ty.lo < tx.lo || (ty.lo == tx.lo && ty.hi <= tx.hi)) break;
            perm[b] = perm[b - 1];
            --b;
        }
        perm[b] = x;
    }
}

__global__ void k_gather_recs(const unsigned long long* __restrict__ dk, const Tag16* __restrict__ dt, const uint32_t* __restrict__ ds,
                              const uint32_t* __restrict__ mint, uint32_t mstride, const uint32_t* __restrict__ perm, uint64_t n,
                              unsigned long long* __restrict__ ok, Tag16* __restrict__ ot, uint32_t* __restrict__ oo) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = perm[i];
    ok[i] = dk[p];
    ot[i] = dt[p];
    oo[i] = mint[(uint64_t)ds[p] * mstride];  // mstride: 1 (dedup table's array) or 4 (the record table's 16-byte slots)
}

#include "orset_tables.hpp"
#include "orset_commit.hpp"

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

int bits_for(uint64_t x) {
    int b = 1;
    while (b < 32 && (1ull << b) <= x) ++b;
    return b;
}


// ---- ORSetMsg.Encode on the device (jg_orset_encode_json; ORSet.cs:56-69, 305-308) ----------------------------
// {"addSet":{"<e>":[<tags>],...},"removeSet":{...},"nullAddGuid":[<tags>],"nullRemoveGuid":[<tags>]} in
// System.Text.Json's compact form: addSet elements in ascending element id (the add Dictionary's insertion
// order), removeSet elements by their first tombstone's ord (when the element entered the remove Dictionary),
// ties by id, tags by (ord, tag) (HashSet<Guid> insertion order), the null element's tags in the two lists.
// Runs = the kept records of one (query, side, element); sections: 0 addSet, 1 removeSet, 2 nullAddGuid,
// 3 nullRemoveGuid; seg = query * 4 + section.
constexpr uint32_t kEncFixed = 65;                           // the five fixed texts of one ORSetMsg
__constant__ const uint32_t kEncBefore[4] = {11, 26, 43, 63};  // fixed bytes before each section

// JavaScriptEncoder.Default for a UTF-8 element string (host/wire.cpp escape): its escaped length, or its bytes.
template <bool WRITE>
__device__ uint32_t enc_escape(const uint8_t* s, uint32_t len, uint8_t* o) {
    const char* HX = "0123456789ABCDEF";
    uint32_t n = 0;
    auto unit = [&](uint32_t u) {
        if (WRITE) {
            o[n] = '\\', o[n + 1] = 'u', o[n + 2] = HX[u >> 12 & 15], o[n + 3] = HX[u >> 8 & 15], o[n + 4] = HX[u >> 4 & 15], o[n + 5] = HX[u & 15];
        }
        n += 6;
    };
    for (uint32_t i = 0; i < len;) {
        const uint32_t c = s[i];
        if (c >= 0x80) {
            const uint32_t k = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
            uint32_t cp = c & (k == 4 ? 0x07 : k == 3 ? 0x0F : 0x1F);
            for (uint32_t q = 1; q < k && i + q < len; ++q) cp = cp << 6 | (s[i + q] & 0x3F);
            i += k;
            if (cp >= 0x10000) {
                unit(0xD800 | (cp - 0x10000) >> 10);
                unit(0xDC00 | ((cp - 0x10000) & 0x3FF));
            } else {
                unit(cp);
            }
            continue;
        }
        ++i;
        char e = 0;
        if (c == '\\') e = '\\';
        else if (c == '\b') e = 'b';
        else if (c == '\t') e = 't';
        else if (c == '\n') e = 'n';
        else if (c == '\f') e = 'f';
        else if (c == '\r') e = 'r';
        if (e) {
            if (WRITE) o[n] = '\\', o[n + 1] = e;
            n += 2;
        } else if (c < 0x20 || c == 0x7F || c == '"' || c == '&' || c == '\'' || c == '+' || c == '<' || c == '>' || c == '`') {
            unit(c);
        } else {
            if (WRITE) o[n] = (uint8_t)c;
            ++n;
        }
    }
    return n;
}

__device__ __forceinline__ void enc_put(uint8_t* o, const char* s) {
    while (*s) *o++ = (uint8_t)*s++;
}

// "<Guid D>" (38 bytes): b3 b2 b1 b0 - b5 b4 - b7 b6 - b8 b9 - b10..b15, lower-case hex
__device__ __forceinline__ void enc_guid(uint8_t* o, unsigned long long lo, unsigned long long hi) {
    const char* hx = "0123456789abcdef";
    const int order[16] = {3, 2, 1, 0, 5, 4, 7, 6, 8, 9, 10, 11, 12, 13, 14, 15};
    int p = 0;
    o[p++] = '"';
    for (int k = 0; k < 16; ++k) {
        if (k == 4 || k == 6 || k == 8 || k == 10) o[p++] = '-';
        const uint32_t b = (uint32_t)((order[k] < 8 ? lo >> (8 * order[k]) : hi >> (8 * (order[k] - 8))) & 0xFF);
        o[p++] = hx[b >> 4];
        o[p++] = hx[b & 15];
    }
    o[p] = '"';
}

struct EncRec {  // the gathered records (jg::orset_gather_sets)
    const unsigned long long *key, *tlo, *thi;
    const uint32_t *ord, *qs;
};

// run heads over the kept records kidx[0..K) (K on the device); positions >= K are padding
__global__ void k_enc_heads(EncRec G, const uint32_t* __restrict__ kidx, const unsigned long long* __restrict__ K, uint64_t R, uint32_t* __restrict__ hf) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= R) return;
    uint32_t h = 0;
    if (j < *K) {
        const uint32_t r = kidx[j];
        h = j == 0 || G.key[kidx[j - 1]] != G.key[r] || G.qs[kidx[j - 1]] != G.qs[r];
    }
    hf[j] = h;
}

// per run (rid[j] - 1 = the run of kept record j): its first kept record, end, query / side / key; first ord reset
__global__ void k_enc_runs(EncRec G, const uint32_t* __restrict__ kidx, const unsigned long long* __restrict__ K, const uint32_t* __restrict__ rid,
                           uint32_t* __restrict__ rstart, uint32_t* __restrict__ rend, uint32_t* __restrict__ rfirst, unsigned long long* __restrict__ nruns) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t k = *K;
    if (j >= k) return;
    const uint32_t run = rid[j] - 1;
    if (j == 0 || rid[j - 1] != rid[j]) {
        rstart[run] = (uint32_t)j;
        rfirst[run] = 0xFFFFFFFFu;
        if (j > 0) rend[run - 1] = (uint32_t)j;
    }
    if (j + 1 == k) {
        rend[run] = (uint32_t)k;
        *nruns = run + 1;
    }
}

__global__ void k_enc_first_ord(EncRec G, const uint32_t* __restrict__ kidx, const unsigned long long* __restrict__ K, const uint32_t* __restrict__ rid,
                                uint32_t* __restrict__ rfirst) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= *K) return;
    const uint32_t o = G.ord[kidx[j]], run = rid[j] - 1;
    if (rfirst[run] > o) atomicMin(rfirst + run, o);
}

__device__ __forceinline__ uint32_t enc_section(uint32_t qs, unsigned long long key) {
    return ((uint32_t)key == JG_NULL_ELEM ? 2u : 0u) + (qs & 1u);
}

// run sort keys: seg << 32 | (removeSet ? first ord : 0), stable over runs in (query, side, id) order; padding ~0
__global__ void k_enc_run_keys(EncRec G, const uint32_t* __restrict__ kidx, const uint32_t* __restrict__ rstart, const uint32_t* __restrict__ rfirst,
                               const unsigned long long* __restrict__ nruns, uint64_t R, unsigned long long* __restrict__ rkey, uint32_t* __restrict__ rval) {
    const uint64_t run = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (run >= R) return;
    unsigned long long k = ~0ull;
    if (run < *nruns) {
        const uint32_t r = kidx[rstart[run]];
        const uint32_t qs = G.qs[r], sec = enc_section(qs, G.key[r]);
        const unsigned long long seg = (unsigned long long)(qs >> 1) * 4 + sec;
        k = seg << 32 | (sec == 1 ? rfirst[run] : 0u);
    }
    rkey[run] = k;
    rval[run] = (uint32_t)run;
}

// per run in output order (rank): its rank, record count, text length; the per-(query, section) bytes and first rank
__global__ void k_enc_run_len(EncRec G, Names N, const uint32_t* __restrict__ kidx, const uint32_t* __restrict__ rstart, const uint32_t* __restrict__ rend,
                              const unsigned long long* __restrict__ skey, const uint32_t* __restrict__ srun, const unsigned long long* __restrict__ nruns,
                              uint64_t R, uint32_t* __restrict__ rrank, unsigned long long* __restrict__ cnt, unsigned long long* __restrict__ tlen,
                              unsigned long long* __restrict__ qsec, uint32_t* __restrict__ sfirst, unsigned* __restrict__ err) {
    const uint64_t rank = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (rank >= R) return;
    if (rank >= *nruns) {
        cnt[rank] = 0;
        tlen[rank] = 0;
        return;
    }
    const uint32_t run = srun[rank];
    rrank[run] = (uint32_t)rank;
    const uint32_t c = rend[run] - rstart[run];
    const unsigned long long key = G.key[kidx[rstart[run]]];
    const uint32_t seg = (uint32_t)(skey[rank] >> 32), sec = seg & 3;
    unsigned long long len = 38ull * c + (c - 1);
    if (sec < 2) {
        const uint32_t g = itab_find(N, (uint32_t)(key >> 32), (uint32_t)key);
        if (g == kNoName) {
            atomicOr(err, 1u);
        } else {
            len += 1 + enc_escape<false>(N.pool + N.off[g], N.len[g], nullptr) + 3 + 1;
            if (rank > 0 && (uint32_t)(skey[rank - 1] >> 32) == seg) len += 1;  // ',' before a later element
        }
    }
    cnt[rank] = c;
    tlen[rank] = len;
    atomicAdd(qsec + seg, len);
    if (sfirst[seg] > rank) atomicMin(sfirst + seg, (uint32_t)rank);
}

// record sort keys: output rank of its run << 32 | ord (stable: the store's tag order breaks ord ties); padding ~0
__global__ void k_enc_rec_keys(EncRec G, const uint32_t* __restrict__ kidx, const unsigned long long* __restrict__ K, const uint32_t* __restrict__ rid,
                               const uint32_t* __restrict__ rrank, uint64_t R, unsigned long long* __restrict__ key, uint32_t* __restrict__ val) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= R) return;
    key[j] = j < *K ? (unsigned long long)rrank[rid[j] - 1] << 32 | G.ord[kidx[j]] : ~0ull;
    val[j] = (uint32_t)j;
}

__global__ void k_enc_qlen(const unsigned long long* __restrict__ qsec, uint64_t n, unsigned long long* __restrict__ qlen) {
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q < n) qlen[q] = kEncFixed + qsec[4 * q] + qsec[4 * q + 1] + qsec[4 * q + 2] + qsec[4 * q + 3];
    if (q == n) qlen[q] = 0;
}

// where a section's text starts in query q's state
__device__ __forceinline__ unsigned long long enc_sec_at(const unsigned long long* qoff, const unsigned long long* qsec, uint32_t q, uint32_t sec) {
    unsigned long long p = qoff[q] + kEncBefore[sec];
    for (uint32_t s = 0; s < sec; ++s) p += qsec[4 * q + s];
    return p;
}

__global__ void k_enc_fixed(const unsigned long long* __restrict__ qoff, const unsigned long long* __restrict__ qsec, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (q >= n) return;
    uint8_t* o = out + qoff[q];
    enc_put(o, "{\"addSet\":{");
    enc_put(out + enc_sec_at(qoff, qsec, (uint32_t)q, 1) - 15, "},\"removeSet\":{");
    enc_put(out + enc_sec_at(qoff, qsec, (uint32_t)q, 2) - 17, "},\"nullAddGuid\":[");
    enc_put(out + enc_sec_at(qoff, qsec, (uint32_t)q, 3) - 20, "],\"nullRemoveGuid\":[");
    enc_put(out + qoff[q + 1] - 2, "]}");
}

// each run's element header / closing bracket; rtags[rank] = where its first tag goes
__global__ void k_enc_run_text(EncRec G, Names N, const uint32_t* __restrict__ kidx, const uint32_t* __restrict__ rstart,
                               const unsigned long long* __restrict__ skey, const uint32_t* __restrict__ srun, const unsigned long long* __restrict__ nruns,
                               const unsigned long long* __restrict__ rpos, const unsigned long long* __restrict__ tlen, const uint32_t* __restrict__ sfirst,
                               const unsigned long long* __restrict__ qoff, const unsigned long long* __restrict__ qsec, unsigned long long* __restrict__ rtags,
                               uint8_t* __restrict__ out) {
    const uint64_t rank = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (rank >= *nruns) return;
    const uint32_t seg = (uint32_t)(skey[rank] >> 32), sec = seg & 3, q = seg >> 2;
    unsigned long long p = enc_sec_at(qoff, qsec, q, sec) + (rpos[rank] - rpos[sfirst[seg]]);
    if (sec < 2) {
        const unsigned long long key = G.key[kidx[rstart[srun[rank]]]];
        const uint32_t g = itab_find(N, (uint32_t)(key >> 32), (uint32_t)key);
        if (rank > 0 && (uint32_t)(skey[rank - 1] >> 32) == seg) out[p++] = ',';
        out[p++] = '"';
        p += enc_escape<true>(N.pool + N.off[g], N.len[g], out + p);
        out[p++] = '"', out[p++] = ':', out[p++] = '[';
        out[enc_sec_at(qoff, qsec, q, sec) + (rpos[rank] - rpos[sfirst[seg]]) + tlen[rank] - 1] = ']';
    }
    rtags[rank] = p;
}

// each record's tag text: ',' before every tag but a run's first
__global__ void k_enc_rec_text(EncRec G, const uint32_t* __restrict__ kidx, const unsigned long long* __restrict__ K, const uint32_t* __restrict__ srec,
                               const uint32_t* __restrict__ rid, const uint32_t* __restrict__ rrank, const unsigned long long* __restrict__ cpos,
                               const unsigned long long* __restrict__ rtags, uint8_t* __restrict__ out) {
    const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (p >= *K) return;
    const uint32_t j = srec[p], rank = rrank[rid[j] - 1], r = kidx[j];
    const unsigned long long k = p - cpos[rank];
    unsigned long long at = rtags[rank] + 39 * k;
    if (k) out[at - 1] = ',';
    enc_guid(out + at, G.tlo[r], G.thi[r]);
}

}  // namespace

// check_id_room's per-set tier: every message's entry count added to its set (cnt[set_cap + 1] flags a set id past
// the table), then each set's next id + its count against the id space (cnt[set_cap] flags an overflow).
__global__ void k_id_room_count(const unsigned long long* __restrict__ ne, const uint32_t* __restrict__ mset, uint64_t n, uint64_t set_cap,
                                unsigned long long* cnt) {
    for (uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long c = ne[m];
        if (c == 0) continue;
        const uint32_t st = mset[m];
        if (st < set_cap) atomicAdd(cnt + st, c);
        else atomicOr(cnt + set_cap + 1, 1ull);
    }
}

__global__ void k_id_room_check(const uint32_t* __restrict__ next_id, const unsigned long long* __restrict__ cnt, uint64_t set_cap,
                                unsigned long long* over) {
    for (uint64_t st = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; st < set_cap; st += (uint64_t)gridDim.x * blockDim.x)
        if (cnt[st] && (uint64_t)next_id[st] + cnt[st] > (uint64_t)JG_NULL_ELEM - 1) atomicOr(over, 1ull);
}

// Element table + open wave of one store.
struct jg_orset_wire {
    // element table
    jg::DevBuf tab, nset, nid, ngen, nlen, noff, nkey, pool, set_gen, next_id;
    uint64_t tab_cap = 0, n_names = 0, name_cap = 0, pool_used = 0, pool_cap = 0, set_cap = 0;
    jg::DevBuf ikey, ival;  // (set, id) -> name index (Names::ikey), every name issued
    uint64_t itab_cap = 0;
    // an upper bound of every set's next element id (names_sync's next ids, plus every name a commit issued since);
    // a fast check only: when it would refuse a wave it is first tightened to the exact max (tight_id_bound)
    uint64_t id_bound = 0;
    jg::DevBuf idmax;  // the device max of next_id (tight_id_bound)
    jg::DevBuf idcnt;  // per-set entry counts of the wave + two flag words (check_id_room's per-set tier)
    // open wave: payload, offsets, set per message, per-message counts / errors
    jg::DevBuf bytes, off, mset, ne, nt, na, err, eoff, toff, slow;  // slow: k_ow_group's per-message flags
    // the wave's payload / offsets / set ids: the buffers above (jg_orset_wave_*), or a node's
    // (csrc/node.hip: every kind's messages uploaded once, set id kSkipIdx for another kind's)
    uint8_t* vbytes = nullptr;
    uint64_t* voff = nullptr;
    uint32_t* vmset = nullptr;
    bool external = false;
    uint64_t wn = 0, wnb = 0, cap_msgs = 0, cap_bytes = 0;
    uint32_t max_set = 0;
    bool open = false, checked = false, any_set = false;
    uint64_t first_bad = kNone, n_ent = 0, n_tag = 0;
    // entries, groups, tags, records
    jg::DevBuf ekey, eval, enoff, emsg, emeta, epos, epfx, eset, skey, sval, hs, seg, impure, label, gid, eid;
    jg::DevBuf sp_key, sp_noff, sp_pfx, sp_meta, sp_pos, sp_set, sp_sid, sp_tref, sp_tval, sp_trk;  // pass 1's sparse regions (by byte offset)
    jg::DevBuf tref, tval, rkey, rside, dtab, dmin, dk[2], dt[2], ds[2], rk, rk2, perm[2], perm2[2];
    jg::DevBuf newk, newv, snk, snv, status, cub;
    jg::DevBuf cnk, fsel, fslot, fidx;  // commit: compacted new-string keys; dedup marks, slots, compacted indices
    jg_orset* recs = nullptr;  // a committed wave's records, sorted (the merge source), reused
    // ids issued by the last commit: names [g0, g1), pool bytes [p0, p1)
    uint64_t g0 = 0, g1 = 0, p0 = 0, p1 = 0;
    // string-hash mask: all bits; tests narrow it (JANUS_TEST_NAME_HASH_BITS) to force collisions
    uint64_t kmask = ~0ull;
    uint64_t salt = 0;  // name_key's per-store salt (random, drawn at first use)
    // key bits the entry sort orders on; tests narrow it (JANUS_TEST_ENTRY_SORT_BITS) so runs mix full keys
    int sort_bits = 32;
    uint64_t resorts = 0;  // waves whose entries were sorted again on full keys (a long impure run)
    // the wave's string and record tables (orset_tables.hpp), filled after each chunk's parse; `tables` =
    // they are being filled this wave, `tables_ok` = the check found them complete (no overflow)
    jg::DevBuf st_slot, st_list, rt_slot, rt_list, sid_id, ovf;  // 16-byte table slots (orset_tables.hpp); ovf: overflow word, sub-list counts
    jg::DevBuf st_packed, rt_packed, loffs;  // the sub-lists packed for the commit
    jg::DevBuf cb;                           // the bucket commit's places and bucket orders (orset_commit.hpp)
    // the bucket counts the tables' claimants take (Claims, orset_tables.hpp): zeroed per wave for cb_cap sets,
    // and one place per string / record slot
    jg::DevBuf cbc, splace, rplace;
    uint64_t cb_cap = 0;
    uint64_t waves_claimed = 0;  // bucket commits whose counts came from the claims (tests read them)
    // the check queued the commit's first steps ahead of its one read (lists packed, the claims' counts scanned:
    // spec_h = k_cb_scan's eight status words), for a commit of the whole wave from the tables
    bool spec = false;
    unsigned long long spec_h[9] = {};  // [8]: k_cb_scatter_claimed's bound flag (orset_commit.hpp)
    jg::DevBuf specst;
    uint64_t waves_bucketed = 0;             // table commits that took the bucket path (tests read them)
    uint64_t st_cap = 0, rt_cap = 0;     // slots in use this wave (a power of two, <= the allocations)
    uint64_t st_alloc = 0, rt_alloc = 0, seen_s = 0, seen_r = 0;  // allocated slots; the last checked wave's distinct strings / records
    bool tables = false, tables_ok = false;
    std::vector<unsigned long long> lc;  // host copy of ovf (overflow word, sub-list counts) taken by the check
    uint64_t waves_fast = 0, waves_sorted = 0;  // commits from the tables / by the sort path (tests read them)
    uint64_t last_cnt[2] = {0, 0};  // distinct records (add, tombstone) the last commit merged: the next wave's estimate
    // (names held, pool bytes used) after each commit / names_sync: where a names_since pull starts in the pool
    std::vector<std::pair<uint64_t, uint64_t>> marks;
    void mark() {
        if (!marks.empty() && marks.back().first == n_names) return;
        marks.emplace_back(n_names, pool_used);
        if (marks.size() > 4096) marks.erase(marks.begin(), marks.begin() + 2048);
    }
    // the names a commit issued, copied into page-locked memory right behind the commit (one queue of copies,
    // no wait): jg_orset_wave_names then waits on `ev` instead of five pageable copies and their syncs
    // (~0.6 ms of every ORSetWorkload wave, the host mirror reads them after each wave)
    struct NamesOut {
        uint8_t* host = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        uint64_t g0 = 0, g1 = 0, p0 = 0, p1 = 0;  // what the queued copy holds (g0 == g1: nothing queued)
        // or what jg_orset_names_since staged: names [since_from, since_to), pool [since_pool0, since_pool1)
        uint64_t since_from = UINT64_MAX, since_to = 0, since_pool0 = 0, since_pool1 = 0, since_bytes = 0;
    } nout;
    jg::DevBuf enc_g, enc;       // jg_orset_encode_json: the gathered records, the encoder's arrays
    std::vector<void*> retired;  // blocks the element table outgrew (grow_keep), freed at the next idle point
    ~jg_orset_wire() {
        for (void* p : retired) (void)hipFree(p);
        if (nout.ev) (void)hipEventSynchronize(nout.ev);
        if (nout.host) (void)hipHostFree(nout.host);
        if (nout.ev) (void)hipEventDestroy(nout.ev);
    }
};

namespace {

void ensure(jg::DevBuf& b, size_t bytes) {
    if (b.bytes < bytes) b.alloc(bytes + bytes / 4 + 256);
}

// Grow to `need` bytes keeping the first `keep` bytes; the new tail is zeroed when `zero`.
// retire: the old block goes there instead of hipFree (the element table grows wave after wave, and each
// hipFree costs ~0.2 ms of host time on the box: six arrays per growth); freed by jg::orset_free_retired at the
// end of the wave (node wave, synchronous merge).
void grow_keep(jg_ctx* ctx, jg::DevBuf& b, size_t need, size_t keep, bool zero = false, std::vector<void*>* retire = nullptr) {
    if (b.bytes >= need) return;
    if (ctx->copy) JG_HIP(hipStreamSynchronize(ctx->copy));  // uploads still landing in the old block
    jg::DevBuf nb;
    nb.alloc(need + need / 2);
    if (zero) JG_HIP(hipMemsetAsync(nb.p, 0, nb.bytes, ctx->stream));
    keep = std::min(keep, b.p ? b.bytes : 0);
    if (keep) JG_HIP(hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, ctx->stream));
    // a retired block lives until the wave has drained: the kernels queued before this copy may still use it, and
    // those queued after it use the new one (stream order) — no host wait in the middle of a commit (~30 us each,
    // six arrays per names growth).  A block freed right here needs the stream idle first.
    if (!retire) JG_HIP(hipStreamSynchronize(ctx->stream));
    std::swap(nb.p, b.p);
    std::swap(nb.bytes, b.bytes);
    if (retire && nb.p) {
        retire->push_back(nb.p);
        nb.p = nullptr;
        nb.bytes = 0;
    }
}

jg_orset_wire* wire_of(jg_orset* s) {
    if (!s->wire) {
        s->wire = new jg_orset_wire();
        s->wire->status.alloc(128);
        std::random_device rd;
        s->wire->salt = ((uint64_t)rd() << 32 ^ rd()) | 1;
        if (const char* e = std::getenv("JANUS_TEST_NAME_HASH_BITS")) {
            const int bits = std::atoi(e);
            if (bits > 0 && bits < 64) s->wire->kmask = (1ull << bits) - 1;
        }
        if (const char* e = std::getenv("JANUS_TEST_ENTRY_SORT_BITS")) {
            const int bits = std::atoi(e);
            if (bits > 0 && bits <= 64) s->wire->sort_bits = bits;
        }
    }
    return s->wire;
}

Names names_of(jg_orset_wire* w) {
    return Names{w->tab.as<unsigned long long>(), w->tab_cap - 1, w->nset.as<uint32_t>(), w->nid.as<uint32_t>(), w->ngen.as<uint32_t>(),
                 w->nlen.as<uint32_t>(), w->noff.as<unsigned long long>(), w->nkey.as<unsigned long long>(), w->pool.as<uint8_t>(),
                 w->set_gen.as<uint32_t>(), w->next_id.as<uint32_t>(), w->ikey.as<unsigned long long>(), w->ival.as<uint32_t>(),
                 w->itab_cap ? w->itab_cap - 1 : 0};
}

void ensure_sets(jg_ctx* ctx, jg_orset_wire* w, uint64_t n_sets) {
    if (n_sets <= w->set_cap) return;
    const uint64_t cap = std::max<uint64_t>(n_sets + n_sets / 2, 1024);
    grow_keep(ctx, w->set_gen, cap * 4, w->set_cap * 4, true, &w->retired);
    grow_keep(ctx, w->next_id, cap * 4, w->set_cap * 4, true, &w->retired);
    w->set_cap = w->set_gen.bytes / 4;
}

// Room for `incoming` more names with `pool_bytes` more pool bytes; the table keeps load <= 1/2 (a
// rebuild keeps live names only).
void ensure_names(jg_ctx* ctx, jg_orset_wire* w, uint64_t incoming, uint64_t pool_bytes) {
    const uint64_t total = w->n_names + incoming;
    JG_REQUIRE(total < 0xFFFFFFF0ull, JG_ESTATE, "OR-Set element table: more than 2^32 names");
    if (total > w->name_cap) {
        const uint64_t cap = std::max<uint64_t>(total + total / 2, 4096);
        grow_keep(ctx, w->nset, cap * 4, w->n_names * 4, false, &w->retired);
        grow_keep(ctx, w->nid, cap * 4, w->n_names * 4, false, &w->retired);
        grow_keep(ctx, w->ngen, cap * 4, w->n_names * 4, false, &w->retired);
        grow_keep(ctx, w->nlen, cap * 4, w->n_names * 4, false, &w->retired);
        grow_keep(ctx, w->noff, cap * 8, w->n_names * 8, false, &w->retired);
        grow_keep(ctx, w->nkey, cap * 8, w->n_names * 8, false, &w->retired);
        w->name_cap = std::min({w->nset.bytes / 4, w->nid.bytes / 4, w->ngen.bytes / 4, w->nlen.bytes / 4, w->noff.bytes / 8, w->nkey.bytes / 8});
    }
    if (w->pool_used + pool_bytes > w->pool_cap) {  // x1.5: a pool grown to the exact need grew again every wave
        grow_keep(ctx, w->pool, std::max<uint64_t>({w->pool_used + pool_bytes, w->pool_cap + w->pool_cap / 2, 1 << 20}), w->pool_used, false,
                  &w->retired);
        w->pool_cap = w->pool.bytes;
    }
    if (w->tab_cap == 0 || 2 * total > w->tab_cap) {
        const uint64_t cap = pow2_at_least(4 * total);
        if (w->tab.p) {  // retired, not freed (see grow_keep)
            w->retired.push_back(w->tab.p);
            w->tab.p = nullptr;
            w->tab.bytes = 0;
        }
        w->tab.alloc(cap * 8);
        w->tab_cap = cap;
        JG_HIP(hipMemsetAsync(w->tab.p, 0, cap * 8, ctx->stream));
        if (w->n_names) {
            hipLaunchKernelGGL(k_names_rebuild, dim3(blocks_for(w->n_names)), dim3(kBlock), 0, ctx->stream, names_of(w), w->n_names);
            JG_HIP(hipGetLastError());
        }
    }
    if (w->itab_cap == 0 || 2 * total > w->itab_cap) {  // the (set, id) index: every name, load <= 1/2
        const uint64_t cap = pow2_at_least(4 * total);
        for (jg::DevBuf* b : {&w->ikey, &w->ival})
            if (b->p) {
                w->retired.push_back(b->p);
                b->p = nullptr;
                b->bytes = 0;
            }
        w->ikey.alloc(cap * 8);
        w->ival.alloc(cap * 4);
        w->itab_cap = cap;
        JG_HIP(hipMemsetAsync(w->ikey.p, 0, cap * 8, ctx->stream));
        if (w->n_names) {
            hipLaunchKernelGGL(k_itab_rebuild, dim3(blocks_for(w->n_names)), dim3(kBlock), 0, ctx->stream, names_of(w), w->n_names);
            JG_HIP(hipGetLastError());
        }
    }
}

unsigned long long* status_words(jg_orset_wire* w) { return w->status.as<unsigned long long>(); }

void read_words(jg_ctx* ctx, const unsigned long long* d, unsigned long long* h, int n) {
    jg::pin_get(ctx, 0, d, n * 8);
    jg::pin_sync(ctx);
    std::memcpy(h, jg::pin_at(ctx, 0), n * 8);
}

// Page-locked layout of a names copy: set [n] u32 | id [n] u32 | len [n] u32 | pad | pool offset [n] u64 | pool bytes.
size_t names_out_bytes(uint64_t n, uint64_t nb) { return ((n * 12 + 15) & ~15ull) + n * 8 + nb; }

// Queue the copy of the names [g0, g1) / pool bytes [p0, p1) the last commit issued (async on ctx->stream).
void queue_names(jg_ctx* ctx, jg_orset_wire* w) {
    auto& o = w->nout;
    o.g0 = o.g1 = 0;
    o.since_from = UINT64_MAX;  // the staging is about to hold this commit's names
    const uint64_t n = w->g1 - w->g0, nb = w->p1 - w->p0;
    if (n == 0) return;
    const size_t need = names_out_bytes(n, nb);
    if (o.cap < need) {
        if (o.ev) JG_HIP(hipEventSynchronize(o.ev));  // no earlier copy may still land in the old block
        if (o.host) JG_HIP(hipHostFree(o.host));
        o.host = nullptr;
        o.cap = 0;
        void* p = nullptr;
        JG_HIP(hipHostMalloc(&p, need + need / 2, hipHostMallocDefault));
        o.host = static_cast<uint8_t*>(p);
        o.cap = need + need / 2;
    }
    if (!o.ev) JG_HIP(hipEventCreateWithFlags(&o.ev, hipEventDisableTiming));
    // on the copy queue (idle once a wave's uploads are in), behind the commit's kernels: the record sorts and
    // the union behind them on ctx->stream do not wait for these copies.  The names arrays are only ever
    // appended to past g1 / p1 or reallocated, and a reallocation (grow_keep) syncs the copy queue first.
    hipStream_t q = ctx->copy ? ctx->copy : ctx->stream;
    if (q != ctx->stream) {
        JG_HIP(hipEventRecord(o.ev, ctx->stream));
        JG_HIP(hipStreamWaitEvent(q, o.ev, 0));
    }
    uint8_t* h = o.host;
    JG_HIP(hipMemcpyAsync(h, w->nset.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, q));
    JG_HIP(hipMemcpyAsync(h + n * 4, w->nid.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, q));
    JG_HIP(hipMemcpyAsync(h + n * 8, w->nlen.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, q));
    const size_t po = (n * 12 + 15) & ~15ull;
    JG_HIP(hipMemcpyAsync(h + po, w->noff.as<unsigned long long>() + w->g0, n * 8, hipMemcpyDeviceToHost, q));
    if (nb) JG_HIP(hipMemcpyAsync(h + po + n * 8, w->pool.as<uint8_t>() + w->p0, nb, hipMemcpyDeviceToHost, q));
    JG_HIP(hipEventRecord(o.ev, q));
    o.g0 = w->g0, o.g1 = w->g1, o.p0 = w->p0, o.p1 = w->p1;
}

void* cub_temp(jg_orset_wire* w, size_t bytes) {
    ensure(w->cub, bytes);
    return w->cub.p;
}

// id_bound sums the names every commit issued over ALL sets, so on a store with many sets it grows far past any
// one set's next id and would refuse waves every set still has room for.  Before refusing, the
// bound is tightened to the exact largest per-set next id (one device max over the sets, one round trip); the
// check then asks whether that set plus every name of the wave could pass 2^32 - 2 — still conservative (all
// names counted against the fullest set), exact in the case that matters (a set near its limit).
uint64_t tight_id_bound(jg_ctx* ctx, jg_orset_wire* w) {
    if (w->set_cap == 0) return w->id_bound = 0;
    ensure(w->idmax, 16);
    size_t temp = 0;
    const uint32_t* nx = w->next_id.as<uint32_t>();
    JG_HIP(hipcub::DeviceReduce::Max(nullptr, temp, nx, w->idmax.as<uint32_t>(), (int)w->set_cap, ctx->stream));
    JG_HIP(hipcub::DeviceReduce::Max(cub_temp(w, temp), temp, nx, w->idmax.as<uint32_t>(), (int)w->set_cap, ctx->stream));
    jg::pin_get(ctx, 0, w->idmax.p, 4);
    jg::pin_sync(ctx);
    uint32_t mx;
    std::memcpy(&mx, jg::pin_at(ctx, 0), 4);
    return w->id_bound = mx;
}

// A wave must not take any set's element ids past JG_NULL_ELEM - 1 (checked before anything commits).  Three
// tiers: id_bound + every name of the wave (host, free); the exact largest next id + every name (one device max);
// then per set, that set's next id + the wave's entries naming it (two small kernels, one round trip) — exact
// per set up to repeated strings, so one set synced near its limit does not block waves on the others.
void check_id_room(jg_ctx* ctx, jg_orset_wire* w, uint64_t incoming, uint64_t n_msgs) {
    if (w->id_bound + incoming <= JG_NULL_ELEM - 1) return;
    if (tight_id_bound(ctx, w) + incoming <= JG_NULL_ELEM - 1) return;
    ensure(w->idcnt, (w->set_cap + 2) * 8);
    auto* cnt = w->idcnt.as<unsigned long long>();
    JG_HIP(hipMemsetAsync(cnt, 0, (w->set_cap + 2) * 8, ctx->stream));
    if (n_msgs)
        hipLaunchKernelGGL(k_id_room_count, dim3(blocks_for(n_msgs)), dim3(kBlock), 0, ctx->stream, w->ne.as<unsigned long long>(), w->vmset, n_msgs,
                           w->set_cap, cnt);
    hipLaunchKernelGGL(k_id_room_check, dim3(blocks_for(w->set_cap)), dim3(kBlock), 0, ctx->stream, w->next_id.as<uint32_t>(), cnt, w->set_cap,
                       cnt + w->set_cap);
    JG_HIP(hipGetLastError());
    jg::pin_get(ctx, 0, cnt + w->set_cap, 16);
    jg::pin_sync(ctx);
    unsigned long long h[2];
    std::memcpy(h, jg::pin_at(ctx, 0), 16);
    JG_REQUIRE(h[0] == 0 && h[1] == 0, JG_ESTATE, "jg_orset_wave: a set's element ids would pass an OR-Set's 2^32 - 2 ids in this wave (largest next id %llu)",
               (unsigned long long)w->id_bound);
}

template <class K, class V>
void sort_pairs(jg_ctx* ctx, jg_orset_wire* w, const K* kin, K* kout, const V* vin, V* vout, uint64_t n, int end_bit) {
    if (n == 0) return;
    size_t temp = 0;
    JG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, kin, kout, vin, vout, (int)n, 0, end_bit, ctx->stream));
    JG_HIP(hipcub::DeviceRadixSort::SortPairs(cub_temp(w, temp), temp, kin, kout, vin, vout, (int)n, 0, end_bit, ctx->stream));
}

// Indices i in [0, n) with pred(i), in order, into idx; their number into *count (device).
template <class Pred> void select_marked(jg_ctx* ctx, jg_orset_wire* w, Pred pred, uint64_t n, uint32_t* idx, unsigned long long* count) {
    hipcub::CountingInputIterator<uint32_t> it(0);
    size_t temp = 0;
    JG_HIP(hipcub::DeviceSelect::If(nullptr, temp, it, idx, count, (int)n, pred, ctx->stream));
    JG_HIP(hipcub::DeviceSelect::If(cub_temp(w, temp), temp, it, idx, count, (int)n, pred, ctx->stream));
}

void grow_wave(jg_ctx* ctx, jg_orset_wire* w, uint64_t msgs, uint64_t bytes) {
    const uint64_t m = w->wn;
    if (msgs > w->cap_msgs) {
        const uint64_t cap = std::max<uint64_t>(msgs + msgs / 2, 1024);
        grow_keep(ctx, w->ne, (cap + 1) * 8, m * 8);
        grow_keep(ctx, w->nt, (cap + 1) * 8, m * 8);
        grow_keep(ctx, w->na, cap * 4, m * 4);
        grow_keep(ctx, w->err, cap * 8, m * 8);
        grow_keep(ctx, w->slow, cap, m);
        w->cap_msgs = cap;
    }
    if (bytes > w->cap_bytes) {
        const uint64_t cap = std::max<uint64_t>(bytes + bytes / 2, 1 << 16);
        const uint64_t es = cap / kEntryDiv + 2, ts = cap / kTagDiv + 2;
        const uint64_t ke = (w->wnb + kEntryDiv - 1) / kEntryDiv + 1, kt = (w->wnb + kTagDiv - 1) / kTagDiv + 1;  // slots in use
        grow_keep(ctx, w->sp_key, es * 8, ke * 8);
        grow_keep(ctx, w->sp_noff, es * 8, ke * 8);
        grow_keep(ctx, w->sp_pfx, es * 8, ke * 8);
        grow_keep(ctx, w->sp_meta, es * 4, ke * 4);
        grow_keep(ctx, w->sp_pos, es * 4, ke * 4);
        grow_keep(ctx, w->sp_set, es * 4, ke * 4);
        grow_keep(ctx, w->sp_sid, es * 4, ke * 4);
        grow_keep(ctx, w->sp_trk, ts * 8, kt * 8);
        grow_keep(ctx, w->sp_tref, ts * 8, kt * 8);
        grow_keep(ctx, w->sp_tval, ts * 16, kt * 16);
        w->cap_bytes = cap;
    }
    if (w->external) return;  // a node's buffers
    // the store's own upload targets (sized on their own: a node wave grows only the arrays above)
    if (w->off.bytes < (msgs + 1) * 8 || w->mset.bytes < msgs * 4) {
        const uint64_t cap = std::max<uint64_t>(msgs + msgs / 2, 1024);
        grow_keep(ctx, w->off, (cap + 1) * 8, (m + 1) * 8);
        grow_keep(ctx, w->mset, cap * 4, m * 4);
    }
    if (w->bytes.bytes < ((bytes + 15) & ~15ull) + 16) {
        const uint64_t cap = std::max<uint64_t>(bytes + bytes / 2, 1 << 16);
        grow_keep(ctx, w->bytes, ((cap + 15) & ~15ull) + 16, w->wnb);  // the cursor reads aligned 16-byte windows
    }
    w->vbytes = w->bytes.as<uint8_t>();
    w->voff = w->off.as<uint64_t>();
    w->vmset = w->mset.as<uint32_t>();
}

Sparse sparse_of(jg_orset_wire* w) {
    return Sparse{w->sp_key.as<unsigned long long>(), w->sp_noff.as<unsigned long long>(), w->sp_pfx.as<unsigned long long>(),
                  w->sp_meta.as<uint32_t>(), w->sp_pos.as<uint32_t>(), w->sp_set.as<uint32_t>(), w->sp_sid.as<uint32_t>(),
                  w->sp_tref.as<unsigned long long>(), w->sp_tval.as<Tag16>(), w->sp_trk.as<unsigned long long>()};
}

Entries entries_of(jg_orset_wire* w) {
    return Entries{w->ekey.as<unsigned long long>(), w->eval.as<uint32_t>(), w->enoff.as<unsigned long long>(), w->emsg.as<uint32_t>(),
                   w->emeta.as<uint32_t>(), w->epos.as<uint32_t>(), w->epfx.as<unsigned long long>(), w->eset.as<uint32_t>()};
}

// Pass 1 over messages [m0, m1) of the open wave (queued on the compute stream).
StrTab str_tab(jg_orset_wire* w) {
    return StrTab{w->st_slot.as<StrSlot>(), w->st_cap - 1, w->st_list.as<uint32_t>(),
                  w->ovf.as<unsigned long long>() + kCountStride, w->st_cap / 8};
}
RecTab rec_tab(jg_orset_wire* w) {
    return RecTab{w->rt_slot.as<RecSlot>(), w->rt_cap - 1, w->rt_list.as<uint32_t>(),
                  w->ovf.as<unsigned long long>() + (1 + kLists) * kCountStride, w->rt_cap / 8};
}

// A wave opens: size and clear its string / record tables (queued on the compute stream, ahead of the first
// chunk's parse).  A compact entry needs >= 43 payload bytes ("":["<guid>"]) and a tag reference >= 38, so
// nbytes / 40 and nbytes / 38 bound the distinct strings and records; a streamed wave sized by its message
// count alone gets 16 strings / 32 records per message and falls back to the sort path if it holds more.
// JANUS_ORSET_TAIL=sort runs the sort path alone (read per wave: tests switch it).
void tables_begin(jg_ctx* ctx, jg_orset_wire* w, uint64_t n_msgs, uint64_t nbytes) {
    const char* e = std::getenv("JANUS_ORSET_TAIL");
    w->tables = !(e && std::strcmp(e, "sort") == 0) && nbytes / kEntryDiv + 2 < 0xFFFFFFFFull && nbytes / kTagDiv + 2 < 0xFFFFFFFFull;
    w->tables_ok = false;
    if (!w->tables) return;
    const uint64_t lim = 1ull << 30;  // slot ids < 2^31 (k_ow_strings packs the side above them); hipcub counts in int
    const uint64_t bound_s = 2 * std::max(nbytes / 40, n_msgs * 16) + 64, bound_r = 2 * std::max(nbytes / 38, n_msgs * 32) + 64;
    // The tables in use are sized from the previous wave's distinct strings / records, x4 (a quarter full at the
    // same mix, half full at twice as many), below the certain bound: that bound gave the ORSetWorkload wave
    // (~0.4M distinct strings and records) 16M-slot tables, ~0.5 GB probed at random, every probe a miss in
    // the 256 MB MALL.  A wave past the smaller tables' room overflows into the sort path (correct, slower) and
    // the next one sizes from the bound again.  JANUS_ORSET_TAIL=tables (no fall-back) keeps the bound.
    const bool strict = e && std::strcmp(e, "tables") == 0;
    const uint64_t want_s = w->seen_s && !strict ? std::min(bound_s, 4 * w->seen_s + 65536) : bound_s;
    const uint64_t want_r = w->seen_r && !strict ? std::min(bound_r, 4 * w->seen_r + 65536) : bound_r;
    const uint64_t sc = std::min(lim, pow2_at_least(std::max<uint64_t>(4096, want_s)));
    const uint64_t rc = std::min(lim, pow2_at_least(std::max<uint64_t>(4096, want_r)));
    if (w->st_alloc < sc) {  // allocations only grow; the active part is the first st_cap slots
        w->st_slot.alloc(sc * sizeof(StrSlot));
        w->st_list.alloc((sc / 8) * kLists * 4);  // sub-lists of cap / 8 (a table is at most half full)
        w->sid_id.alloc(sc * 4);
        w->splace.alloc(sc * 8);
        w->st_packed.alloc((sc / 8) * kLists * 4 + 4);  // the packed list (spec_commit_prep: no allocation behind the uploads)
        w->st_alloc = sc;
    }
    if (w->rt_alloc < rc) {
        w->rt_slot.alloc(rc * sizeof(RecSlot));
        w->rt_list.alloc((rc / 8) * kLists * 4);
        w->rplace.alloc(rc * 8);
        w->rt_packed.alloc((rc / 8) * kLists * 4 + 4);
        w->rt_alloc = rc;
    }
    w->st_cap = sc;
    w->rt_cap = rc;
    if (!w->ovf.p) w->ovf.alloc((1 + 2 * kLists) * kCountStride * 8);
    ensure(w->loffs, 2 * (kLists + 1) * 8);
    ensure(w->specst, sizeof w->spec_h);
    hipLaunchKernelGGL(k_str_clear, dim3((unsigned)std::min<uint64_t>(4096, (2 * w->st_cap + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       w->st_slot.as<uint4>(), w->st_cap);
    hipLaunchKernelGGL(k_tab_clear, dim3((unsigned)std::min<uint64_t>(4096, (w->rt_cap + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       w->rt_slot.as<uint4>(), w->rt_cap);
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemsetAsync(w->ovf.p, 0, (1 + 2 * kLists) * kCountStride * 8, ctx->stream));  // overflow, uncounted, sub-list counts
    // the claim-time bucket counts: one per set the store knows (a set past them sends the commit to k_cb_count)
    const uint64_t cap = std::min<uint64_t>(0x7FFFFFF0ull, std::max<uint64_t>({w->cb_cap, w->set_cap, (uint64_t)w->max_set + 1, 1024}));
    if (cap > w->cb_cap) {
        w->cbc.alloc(cb_counts_bytes(cap));
        w->cb_cap = cap;
    }
    JG_HIP(hipMemsetAsync(w->cbc.p, 0, cb_counts_bytes(w->cb_cap), ctx->stream));
    ensure(w->cb, cb_items_bytes(w->st_cap, w->rt_cap));
}

Claims claims_of(jg_orset_wire* w) {
    Claims C{};
    char* p = w->cbc.as<char>();
    const uint64_t c4 = cb_al((w->cb_cap + 1) * 4);
    C.scnt = reinterpret_cast<uint32_t*>(p);
    C.rcnt[0] = reinterpret_cast<uint32_t*>(p + c4);
    C.rcnt[1] = reinterpret_cast<uint32_t*>(p + 2 * c4);
    C.sbytes = reinterpret_cast<unsigned long long*>(p + 3 * c4);
    C.splace = w->splace.as<uint2>();
    C.rplace = w->rplace.as<uint2>();
    C.uncounted = w->ovf.as<unsigned long long>() + 1;  // ovf word 1: zeroed with the overflow word, read by the check
    C.cap = (uint32_t)w->cb_cap;
    return C;
}

// The bucket commit's arrays: the claims' counts, then places and bucket orders for every entry the two tables'
// lists can hold this wave (w->cb, sized by tables_begin, so the check can queue the scatter before its read).
Buckets buckets_of(jg_orset_wire* w) {
    const Claims C = claims_of(w);
    Buckets B{};
    B.scnt = C.scnt;  // the counts: cb_cap + 1 entries each (the scan covers the wave's n_sets + 1)
    B.rcnt[0] = C.rcnt[0];
    B.rcnt[1] = C.rcnt[1];
    B.sbytes = C.sbytes;
    const uint64_t s4 = cb_al((w->st_cap / 8) * kLists * 4 + 4), r4 = cb_al((w->rt_cap / 8) * kLists * 4 + 4);
    char* q = w->cb.as<char>();
    B.spos = reinterpret_cast<uint32_t*>(q);
    B.sset = reinterpret_cast<uint32_t*>(q + s4);
    B.sitem = reinterpret_cast<uint32_t*>(q + 2 * s4);
    q += 3 * s4;
    B.rpos = reinterpret_cast<uint32_t*>(q);
    B.rset = reinterpret_cast<uint32_t*>(q + r4);
    B.ritem[0] = reinterpret_cast<uint32_t*>(q + 2 * r4);
    B.ritem[1] = reinterpret_cast<uint32_t*>(q + 3 * r4);
    B.n_sets = (uint32_t)std::min<uint64_t>((uint64_t)w->max_set + 1, 0xFFFFFFFFull);
    return B;
}

// The chunk's strings and records into the wave's tables (after its parse, same stream).
void launch_tables(jg_ctx* ctx, jg_orset_wire* w, uint64_t m0, uint64_t m1) {
    const Sparse S = sparse_of(w);
    auto* ovf = w->ovf.as<unsigned long long>();
    // the element table and the sets' generation words as they stand (both only change at a commit); a wave
    // before the first commit has no table yet: every string is resolved by the commit
    const uint32_t set_lim = w->tab_cap ? (uint32_t)std::min<uint64_t>(w->set_cap, 0xFFFFFFFFull) : 0u;
    const dim3 grid((unsigned)((m1 - m0 + kTabWaves - 1) / kTabWaves));  // one message per wave
    const dim3 grid_m((unsigned)((m1 - m0 + kTabWaves * kMsgsPerWave - 1) / (kTabWaves * kMsgsPerWave)));  // kMsgsPerWave messages per wave
    hipLaunchKernelGGL(k_ow_strings, grid, dim3(kBlock), 0, ctx->stream, S, w->voff, w->vmset, w->vbytes, w->ne.as<unsigned long long>(),
                       w->na.as<uint32_t>(), m0, m1, str_tab(w), w->err.as<unsigned long long>(), ovf, names_of(w), set_lim,
                       w->sid_id.as<uint32_t>(), claims_of(w));
    hipLaunchKernelGGL(k_ow_rkeys, grid_m, dim3(kBlock), 0, ctx->stream, S, w->voff, w->vmset, w->nt.as<unsigned long long>(), m0, m1);
    hipLaunchKernelGGL(k_ow_rins, grid_m, dim3(kBlock), 0, ctx->stream, S, w->voff, w->vmset, w->nt.as<unsigned long long>(), m0, m1, rec_tab(w), ovf,
                       claims_of(w));
    JG_HIP(hipGetLastError());
}

// One wave per message (k_ow_group, orset_group.hpp), then the serial parse of the messages it left;
// JANUS_ORSET_PARSE=serial runs the serial parse alone, =group the group parse alone (read per chunk: tests
// switch it).
void launch_parse(jg_ctx* ctx, jg_orset_wire* w, uint64_t m0, uint64_t m1) {
    if (m1 <= m0) return;
    const char* e = std::getenv("JANUS_ORSET_PARSE");
    const bool serial = e && std::strcmp(e, "serial") == 0, strict = e && std::strcmp(e, "group") == 0;
    uint8_t* slow = nullptr;
    if (!serial) {
        slow = w->slow.as<uint8_t>();
        hipLaunchKernelGGL(k_ow_group, dim3((unsigned)((m1 - m0 + kOgWaves - 1) / kOgWaves)), dim3(kBlock), 0, ctx->stream, w->vbytes, w->voff,
                           w->vmset, m0, m1, sparse_of(w), w->kmask, w->salt, w->ne.as<unsigned long long>(), w->nt.as<unsigned long long>(),
                           w->na.as<uint32_t>(), w->err.as<unsigned long long>(), slow);
        JG_HIP(hipGetLastError());
    }
    if (strict)
        hipLaunchKernelGGL(k_ow_reject_slow, dim3(blocks_for(m1 - m0)), dim3(kBlock), 0, ctx->stream, slow, m0, m1, w->ne.as<unsigned long long>(),
                           w->nt.as<unsigned long long>(), w->na.as<uint32_t>(), w->err.as<unsigned long long>());
    else
        hipLaunchKernelGGL(k_ow_parse, dim3(blocks_for(m1 - m0)), dim3(kBlock), 0, ctx->stream, w->vbytes, w->voff, w->vmset, m0, m1,
                           sparse_of(w), w->kmask, w->salt, w->ne.as<unsigned long long>(), w->nt.as<unsigned long long>(), w->na.as<uint32_t>(),
                           w->err.as<unsigned long long>(), slow);
    JG_HIP(hipGetLastError());
    if (w->tables) launch_tables(ctx, w, m0, m1);
}

// JANUS_TRACE_MERGE: host times (us) from the check's read to the commit's first launch
double g_tmark[6] = {};
double tnow_us() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e6; }

// Queued by the check of a table wave before its one read, for a commit of the whole wave from the claims'
// counts (commit_buckets): both lists packed from offsets computed on the device, and the per-set counts
// scanned into bucket offsets (k_cb_scan's totals come back with the check's read).  A commit that cannot
// use them (a limit, an uncounted claim, an overflowed table, JANUS_ORSET_COMMIT=radix / count) repacks or
// recounts as before; this only writes the packed lists, the counts and specst.
void spec_commit_prep(jg_ctx* ctx, jg_orset_wire* w) {
    const char* e = std::getenv("JANUS_ORSET_COMMIT");
    const uint64_t n_sets = (uint64_t)w->max_set + 1;
    const char* sp = std::getenv("JANUS_ORSET_SPEC");  // =0: the commit packs and scans after the check (A/B runs)
    w->spec = !(e && (std::strcmp(e, "radix") == 0 || std::strcmp(e, "count") == 0)) && !(sp && std::strcmp(sp, "0") == 0) && n_sets <= w->cb_cap;
    if (!w->spec) return;
    const StrTab ST = str_tab(w);
    const RecTab RT = rec_tab(w);
    const uint64_t cs = kLists * ST.sub_cap, cr = kLists * RT.sub_cap;
    // buffers sized by tables_begin: an allocation here (hipFree / hipMalloc behind the uploads) cost ~0.5 ms
    if (w->st_packed.bytes < cs * 4 + 4 || w->rt_packed.bytes < cr * 4 + 4 || !w->loffs.p || !w->specst.p ||
        w->cb.bytes < cb_items_bytes(w->st_cap, w->rt_cap)) {
        w->spec = false;
        return;
    }
    auto* doffs = w->loffs.as<unsigned long long>();
    auto* spec_words = w->specst.as<unsigned long long>();
    hipLaunchKernelGGL(k_list_offs, dim3(1), dim3(64), 0, ctx->stream, ST.n, ST.sub_cap, RT.n, RT.sub_cap, doffs, spec_words + 8);
    // grid-stride over the packed lists: enough workgroups for the last wave's distinct strings / records
    auto grid = [](uint64_t seen, uint64_t cap) {
        return dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks_for(seen ? std::min(cap, 2 * seen + 4096) : cap), 4096)));
    };
    hipLaunchKernelGGL(k_list_pack, grid(w->seen_s, cs), dim3(kBlock), 0, ctx->stream, ST.list, ST.sub_cap, doffs, w->st_packed.as<uint32_t>());
    hipLaunchKernelGGL(k_list_pack, grid(w->seen_r, cr), dim3(kBlock), 0, ctx->stream, RT.list, RT.sub_cap, doffs + kLists + 1, w->rt_packed.as<uint32_t>());
    const Claims C = claims_of(w);
    const Buckets B = buckets_of(w);
    hipLaunchKernelGGL(k_cb_scan, dim3(4), dim3(kScanThreads), 0, ctx->stream, B, n_sets + 1, w->specst.as<unsigned long long>());
    // and every item of the PACKED lists into its bucket (a no-op when a claim went uncounted or a table overflowed)
    StrTab PT = ST;
    RecTab PR = RT;
    PT.list = w->st_packed.as<uint32_t>();
    PR.list = w->rt_packed.as<uint32_t>();
    hipLaunchKernelGGL(k_cb_scatter_claimed, grid(w->seen_s + w->seen_r, cs + cr), dim3(kBlock), 0, ctx->stream, doffs, PT, PR, C, B,
                       w->ovf.as<unsigned long long>(), spec_words + 8);
    JG_HIP(hipGetLastError());
}

// Passes 2 + grouping over the whole wave; sets w->first_bad.  Returns the first bad message's code.
int check_wave(jg_orset* s, jg_orset_wire* w) {
    jg_ctx* ctx = s->ctx;
    const uint64_t n = w->wn;
    w->checked = true;
    w->first_bad = kNone;
    w->n_ent = w->n_tag = 0;
    w->tables_ok = false;
    if (n == 0) return JG_OK;
    if (w->tables) {  // the chunks filled the tables (and reported repeated names): the first bad message is all
        unsigned long long* st = status_words(w);  // that is left, unless a table overflowed
        JG_HIP(hipMemsetAsync(st, 0xFF, 8, ctx->stream));
        hipLaunchKernelGGL(k_ow_first_bad, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, w->err.as<unsigned long long>(), n, st);
        JG_HIP(hipGetLastError());
        spec_commit_prep(ctx, w);
        // the overflow word and the tables' sub-list counts (the commit's) come back with the first bad message,
        // and with them the claims' bucket totals: one round trip, page-locked
        w->lc.resize((1 + 2 * kLists) * kCountStride);
        const size_t at_spec = 64 + w->lc.size() * 8;
        jg::pin_get(ctx, 0, st, 8);
        jg::pin_get(ctx, 64, w->ovf.p, w->lc.size() * 8);
        if (w->spec) jg::pin_get(ctx, at_spec, w->specst.p, sizeof w->spec_h);
        jg::pin_sync(ctx);
        g_tmark[0] = tnow_us();
        std::memcpy(w->lc.data(), jg::pin_at(ctx, 64), w->lc.size() * 8);
        if (w->spec) std::memcpy(w->spec_h, jg::pin_at(ctx, at_spec), sizeof w->spec_h);
        unsigned long long h[2];
        std::memcpy(h, jg::pin_at(ctx, 0), 8);
        h[1] = w->lc[0];
        // the speculative scatter found a claimed place outside its arrays in a wave whose claims all counted: the
        // tables are inconsistent, and nothing of the wave may commit (it would commit a bucket with a stale slot)
        JG_REQUIRE(!(w->spec && h[1] == 0 && w->lc[1] == 0 && w->spec_h[8] != 0), JG_EHIP,
                   "OR-Set wave check: the claims' scatter found places outside the bucket arrays (flags %llx): internal table inconsistency",
                   w->spec_h[8]);
        const char* e = std::getenv("JANUS_ORSET_TAIL");  // =tables (tests): no fall-back, an overflow is an error
        JG_REQUIRE(h[1] == 0 || !(e && std::strcmp(e, "tables") == 0), JG_ESTATE, "OR-Set wave tables overflowed (JANUS_ORSET_TAIL=tables)");
        w->seen_s = w->seen_r = 0;  // an overflowed wave: the next one sizes its tables from the bound
        if (h[1] == 0) {
            w->tables_ok = true;
            for (uint32_t j = 0; j < kLists; ++j) {  // the next wave's table sizes (tables_begin)
                w->seen_s += w->lc[(1 + j) * kCountStride];
                w->seen_r += w->lc[(1 + kLists + j) * kCountStride];
            }
            // a set's element ids cannot run out in this wave's commit: every set's next id is at most the
            // names issued so far, and the wave adds at most one per distinct (set, string) — checked here,
            // before a node wave commits anything (the commit's own check then never fires mid-wave)
            uint64_t ns = 0;
            for (uint32_t j = 0; j < kLists; ++j) ns += w->lc[(1 + j) * kCountStride];
            check_id_room(ctx, w, ns, n);
            g_tmark[1] = tnow_us();
            if (h[0] == kNone) return JG_OK;
            unsigned long long e;
            JG_HIP(hipMemcpyAsync(&e, w->err.as<unsigned long long>() + h[0], 8, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            w->first_bad = h[0];
            return (e & 3) == kKindState ? JG_ESTATE : JG_EINVAL;
        }
    }
    // offsets: exclusive sums with a zero sentinel at [n]
    JG_HIP(hipMemsetAsync(w->ne.as<unsigned long long>() + n, 0, 8, ctx->stream));
    JG_HIP(hipMemsetAsync(w->nt.as<unsigned long long>() + n, 0, 8, ctx->stream));
    ensure(w->eoff, (n + 1) * 8);
    ensure(w->toff, (n + 1) * 8);
    size_t temp = 0;
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, w->ne.as<unsigned long long>(), w->eoff.as<unsigned long long>(), (int)(n + 1), ctx->stream));
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(cub_temp(w, temp), temp, w->ne.as<unsigned long long>(), w->eoff.as<unsigned long long>(), (int)(n + 1),
                                            ctx->stream));
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(cub_temp(w, temp), temp, w->nt.as<unsigned long long>(), w->toff.as<unsigned long long>(), (int)(n + 1),
                                            ctx->stream));
    unsigned long long tot[2];
    JG_HIP(hipMemcpyAsync(&tot[0], w->eoff.as<unsigned long long>() + n, 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipMemcpyAsync(&tot[1], w->toff.as<unsigned long long>() + n, 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    const uint64_t ne = tot[0], nt = tot[1];
    JG_REQUIRE(ne < 0x7FFFFFF0ull && nt < 0x7FFFFFF0ull, JG_EINVAL, "jg_orset_wave: %llu entries / %llu tags exceed one wave (2^31)",
               (unsigned long long)ne, (unsigned long long)nt);
    check_id_room(ctx, w, ne, n);
    w->n_ent = ne;
    w->n_tag = nt;
    ensure(w->ekey, ne * 8 + 8);
    ensure(w->eval, ne * 4 + 4);
    ensure(w->enoff, ne * 8 + 8);
    ensure(w->emsg, ne * 4 + 4);
    ensure(w->emeta, ne * 4 + 4);
    ensure(w->epos, ne * 4 + 4);
    ensure(w->epfx, ne * 8 + 8);
    ensure(w->eset, ne * 4 + 4);
    ensure(w->tref, nt * 8 + 8);
    ensure(w->tval, nt * 16 + 16);
    const Entries E = entries_of(w);
    hipLaunchKernelGGL(k_ow_compact, dim3((unsigned)((n + kCompactMsgs - 1) / kCompactMsgs)), dim3(kBlock), 0, ctx->stream, w->voff, n, w->ne.as<unsigned long long>(),
                       w->nt.as<unsigned long long>(), w->na.as<uint32_t>(), w->eoff.as<unsigned long long>(), w->toff.as<unsigned long long>(),
                       w->vmset, w->vbytes, sparse_of(w), E, w->tref.as<unsigned long long>(), w->tval.as<Tag16>());
    JG_HIP(hipGetLastError());
    if (ne) {
        ensure(w->skey, ne * 8);
        ensure(w->sval, ne * 4);
        ensure(w->hs, ne * 4);
        ensure(w->seg, ne * 4);
        ensure(w->impure, ne);
        ensure(w->label, ne * 4);
        sort_pairs(ctx, w, E.key, w->skey.as<unsigned long long>(), E.val, w->sval.as<uint32_t>(), ne, w->sort_bits);
        const unsigned long long run_mask = w->sort_bits >= 64 ? ~0ull : (1ull << w->sort_bits) - 1;
        hipLaunchKernelGGL(k_ow_head, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, w->skey.as<unsigned long long>(), ne, run_mask,
                           w->hs.as<uint32_t>());
        JG_HIP(hipGetLastError());
        temp = 0;
        JG_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, temp, w->hs.as<uint32_t>(), w->seg.as<uint32_t>(), hipcub::Max(), (int)ne, ctx->stream));
        JG_HIP(hipcub::DeviceScan::InclusiveScan(cub_temp(w, temp), temp, w->hs.as<uint32_t>(), w->seg.as<uint32_t>(), hipcub::Max(), (int)ne,
                                                 ctx->stream));
        JG_HIP(hipMemsetAsync(w->impure.p, 0, ne, ctx->stream));
        hipLaunchKernelGGL(k_ow_link, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->vbytes,
                           w->sval.as<uint32_t>(), w->seg.as<uint32_t>(), ne, w->impure.as<uint8_t>());
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemsetAsync(status_words(w) + 1, 0, 8, ctx->stream));
        hipLaunchKernelGGL(k_ow_label, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->vbytes,
                           w->sval.as<uint32_t>(), w->seg.as<uint32_t>(), w->impure.as<uint8_t>(), ne, w->label.as<uint32_t>(),
                           w->err.as<unsigned long long>(), kImpureScan, status_words(w) + 1);
        JG_HIP(hipGetLastError());
    }
    unsigned long long* st = status_words(w);
    JG_HIP(hipMemsetAsync(st, 0xFF, 8, ctx->stream));
    hipLaunchKernelGGL(k_ow_first_bad, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, w->err.as<unsigned long long>(), n, st);
    JG_HIP(hipGetLastError());
    unsigned long long words[2] = {kNone, 0};
    read_words(ctx, st, words, ne ? 2 : 1);
    if (words[1]) {  // a long impure run: entries again by their whole 64-bit keys, then label without a limit
        const Entries E = entries_of(w);
        sort_pairs(ctx, w, E.key, w->skey.as<unsigned long long>(), E.val, w->sval.as<uint32_t>(), ne, 64);
        hipLaunchKernelGGL(k_ow_head, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, w->skey.as<unsigned long long>(), ne, ~0ull,
                           w->hs.as<uint32_t>());
        JG_HIP(hipGetLastError());
        size_t temp = 0;
        JG_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, temp, w->hs.as<uint32_t>(), w->seg.as<uint32_t>(), hipcub::Max(), (int)ne, ctx->stream));
        JG_HIP(hipcub::DeviceScan::InclusiveScan(cub_temp(w, temp), temp, w->hs.as<uint32_t>(), w->seg.as<uint32_t>(), hipcub::Max(), (int)ne,
                                                 ctx->stream));
        JG_HIP(hipMemsetAsync(w->impure.p, 0, ne, ctx->stream));
        hipLaunchKernelGGL(k_ow_link, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->vbytes, w->sval.as<uint32_t>(),
                           w->seg.as<uint32_t>(), ne, w->impure.as<uint8_t>());
        hipLaunchKernelGGL(k_ow_label, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->vbytes, w->sval.as<uint32_t>(),
                           w->seg.as<uint32_t>(), w->impure.as<uint8_t>(), ne, w->label.as<uint32_t>(), w->err.as<unsigned long long>(),
                           UINT32_MAX, st + 1);
        JG_HIP(hipGetLastError());
        JG_HIP(hipMemsetAsync(st, 0xFF, 8, ctx->stream));
        hipLaunchKernelGGL(k_ow_first_bad, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, w->err.as<unsigned long long>(), n, st);
        JG_HIP(hipGetLastError());
        read_words(ctx, st, words, 1);
        ++w->resorts;
    }
    const unsigned long long bad = words[0];
    if (bad == kNone) return JG_OK;
    unsigned long long e;
    JG_HIP(hipMemcpyAsync(&e, w->err.as<unsigned long long>() + bad, 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    w->first_bad = bad;
    return (e & 3) == kKindState ? JG_ESTATE : JG_EINVAL;
}

// Sort one side's distinct records by (key, tag.lo, tag.hi) into a dense stream; ords = first tag index in the
// wave (< nt = the stream's next).  begin: one radix sort by key, then each key's few tags ordered in place
// (k_fix_runs), queued without a wait — *long_run (device) flags a key with more than kRunFix new tags;
// end (after the caller read both sides' flags in one sync): such a side is sorted again by all three words
// (three stable LSD passes), then the records are gathered in order.
void sort_side_begin(jg_ctx* ctx, jg_orset_wire* w, int sd, uint64_t n, int key_bits, uint64_t nt, jg_stream_soa& out,
                     unsigned long long* long_run) {
    jg::set_dense(ctx, out, n);
    out.next = nt;
    JG_HIP(hipMemsetAsync(long_run, 0, 8, ctx->stream));
    if (n == 0) return;
    ensure(w->rk, n * 8);
    ensure(w->rk2, n * 8);
    ensure(w->perm[sd], n * 4);
    ensure(w->perm2[sd], n * 4);
    const auto* dk = w->dk[sd].as<unsigned long long>();
    const auto* dt = w->dt[sd].as<Tag16>();
    uint32_t* p = w->perm[sd].as<uint32_t>();
    uint32_t* q = w->perm2[sd].as<uint32_t>();
    hipLaunchKernelGGL(k_iota, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, p, n);
    hipLaunchKernelGGL(k_gather_radix, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, dk, dt, p, n, 2, w->rk.as<unsigned long long>());
    JG_HIP(hipGetLastError());
    sort_pairs(ctx, w, w->rk.as<unsigned long long>(), w->rk2.as<unsigned long long>(), p, q, n, key_bits);
    hipLaunchKernelGGL(k_fix_runs, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, w->rk2.as<unsigned long long>(), dt, q, n, long_run);
    JG_HIP(hipGetLastError());
}

void sort_side_end(jg_ctx* ctx, jg_orset_wire* w, int sd, uint64_t n, int key_bits, jg_stream_soa& out, bool long_run, const uint32_t* mint,
                   uint32_t mstride) {
    if (n == 0) return;
    const auto* dk = w->dk[sd].as<unsigned long long>();
    const auto* dt = w->dt[sd].as<Tag16>();
    uint32_t* p = w->perm2[sd].as<uint32_t>();  // the key sort's output, runs fixed
    if (long_run) {
        p = w->perm[sd].as<uint32_t>();
        uint32_t* q = w->perm2[sd].as<uint32_t>();
        hipLaunchKernelGGL(k_iota, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, p, n);
        for (int which = 0; which < 3; ++which) {
            hipLaunchKernelGGL(k_gather_radix, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, dk, dt, p, n, which, w->rk.as<unsigned long long>());
            JG_HIP(hipGetLastError());
            sort_pairs(ctx, w, w->rk.as<unsigned long long>(), w->rk2.as<unsigned long long>(), p, q, n, which == 2 ? key_bits : 64);
            std::swap(p, q);
        }
    }
    hipLaunchKernelGGL(k_gather_recs, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, dk, dt, w->ds[sd].as<uint32_t>(), mint, mstride,
                       p, n, out.key.as<unsigned long long>(), out.tag.as<Tag16>(), out.ord.as<uint32_t>());
    JG_HIP(hipGetLastError());
}

void commit_packed(jg_orset* s, jg_orset_wire* w, StrTab ST, RecTab RT, uint64_t ns, uint64_t nrec, uint32_t csi_lim, uint32_t t_lim,
                   uint64_t t_next, double* tc, bool tr);

// The bucket commit (orset_commit.hpp): false if a set's bucket is past the LDS sorts (or JANUS_ORSET_COMMIT=radix),
// with nothing changed but the resolved ids of known strings (the radix path writes them again).
bool commit_buckets(jg_orset* s, jg_orset_wire* w, const StrTab& ST, const RecTab& RT, uint64_t ns, uint64_t nrec, uint32_t csi_lim,
                    uint32_t t_lim, uint64_t t_next) {
    // JANUS_ORSET_COMMIT (read per wave: tests switch it): radix = the radix path alone; buckets = no fall-back (a
    // wave the bucket path cannot take is an error)
    const char* e = std::getenv("JANUS_ORSET_COMMIT");
    if (e && std::strcmp(e, "radix") == 0) return false;
    const bool strict = e && std::strcmp(e, "buckets") == 0;
    jg_ctx* ctx = s->ctx;
    const uint64_t n_sets = (uint64_t)w->max_set + 1;
    // one count per set id up to the wave's largest: sparse set ids (far more ids than items) take the radix path
    if (n_sets >= 0x7FFFFFFFull || ns + nrec >= 0xFFFFFFF0ull || n_sets > 4 * (ns + nrec) + (1u << 20)) {
        JG_REQUIRE(!strict, JG_ESTATE, "OR-Set bucket commit: %llu set ids for %llu items (JANUS_ORSET_COMMIT=buckets)", (unsigned long long)n_sets,
                   (unsigned long long)(ns + nrec));
        return false;
    }
    // the whole wave commits and every claim counted (the check read the uncounted word): the claimants' counts
    // and places stand, and neither k_cb_count nor its memsets run
    // (only a wave the check prepared: its scatter's bound flag was read with the check's words)
    const bool claimed = w->spec && csi_lim == 0xFFFFFFFFu && t_lim == 0xFFFFFFFFu && w->lc.size() > 1 && w->lc[1] == 0 && n_sets <= w->cb_cap &&
                         !(e && std::strcmp(e, "count") == 0);  // JANUS_ORSET_COMMIT=count: the counting pass always (tests)
    ensure(w->cb, cb_items_bytes(w->st_cap, w->rt_cap));  // (sized by tables_begin)
    Buckets B = buckets_of(w);
    unsigned long long* st = status_words(w);
    if (n_sets > w->cb_cap) {  // (a set the wave's claims could not count) room for every set's counts
        w->cbc.alloc(cb_counts_bytes(n_sets));  // the tables' claims are done with the old block (same stream)
        w->cb_cap = n_sets;
        const Claims C2 = claims_of(w);
        B.scnt = C2.scnt, B.rcnt[0] = C2.rcnt[0], B.rcnt[1] = C2.rcnt[1], B.sbytes = C2.sbytes;
    }
    // not from the claims: the counts again from the lists (the check may have scanned the claims' counts in place)
    if (!claimed) JG_HIP(hipMemsetAsync(w->cbc.p, 0, cb_counts_bytes(w->cb_cap), ctx->stream));  // the four count arrays (and their trailing zeros)
    // the scan's words (and k_cb_strings' id flag, a device-side guard no host reads: the check ruled the overflow
    // out); a commit from the check's scan reads no word here, and skips the call (~25-40 us of host time right
    // behind the check's sync, with the device idle)
    if (!(claimed && w->spec)) JG_HIP(hipMemsetAsync(st, 0, 9 * 8, ctx->stream));
    static const bool trm = std::getenv("JANUS_TRACE_MERGE") != nullptr;
    if (trm) {
        g_tmark[5] = tnow_us();
        std::fprintf(stderr, "commit host: read -> check end %.0f us, -> commit %.0f, -> names %.0f, names %.0f, -> first launch %.0f\n", g_tmark[1] - g_tmark[0],
                     g_tmark[2] - g_tmark[1], g_tmark[3] - g_tmark[2], g_tmark[4] - g_tmark[3], g_tmark[5] - g_tmark[4]);
    }
    const Sparse S = sparse_of(w);
    const Names N = names_of(w);
    unsigned long long h[8];  // totals: new strings, their bytes, records per side; then the largest buckets
    if (claimed) {  // scanned by the check, totals read with it (spec_commit_prep)
        std::memcpy(h, w->spec_h, sizeof h);
    } else {
        if (ns + nrec) {
            hipLaunchKernelGGL(k_cb_count, dim3(blocks_for(ns + nrec)), dim3(kBlock), 0, ctx->stream, S, w->vbytes, ST, RT, ns, nrec, csi_lim, t_lim, N,
                               w->sid_id.as<uint32_t>(), B);
        }
        hipLaunchKernelGGL(k_cb_scan, dim3(4), dim3(kScanThreads), 0, ctx->stream, B, n_sets + 1, st);
        JG_HIP(hipGetLastError());
        read_words(ctx, st, h, 8);
    }
    if (h[4] > kCbMax || h[6] > kCbMax || h[7] > kCbMax) {
        JG_REQUIRE(!strict, JG_ESTATE, "OR-Set bucket commit: a set holds %llu new strings / %llu + %llu records of the wave (> %u, JANUS_ORSET_COMMIT=buckets)",
                   h[4], h[6], h[7], kCbMax);
        return false;
    }
    const uint64_t n_new = h[0], nb = h[1], cnt[2] = {h[2], h[3]};
    if (!claimed && ns + nrec)  // (a claimed wave was scattered by the check: spec_commit_prep)
        hipLaunchKernelGGL(k_cb_scatter, dim3(blocks_for(ns + nrec)), dim3(kBlock), 0, ctx->stream, ns, nrec, ST, RT, B);
    if (claimed) ++w->waves_claimed;
    // LDS and threads for the largest bucket (orset_commit.hpp)
    auto cb_threads = [](uint32_t P) { return std::min<uint32_t>(kCbBlock, std::max<uint32_t>(64, P)); };
    const uint32_t Ps = pow2_ge(std::max<uint32_t>(1, (uint32_t)h[4])), Pr = pow2_ge(std::max<uint32_t>(1, (uint32_t)std::max(h[6], h[7])));
    if (n_new)
        hipLaunchKernelGGL(k_cb_strings, dim3((unsigned)n_sets), dim3(cb_threads(Ps)), cb_strings_lds(Ps), ctx->stream, S, w->vbytes, ST, B, w->n_names,
                           w->pool_used, N, w->sid_id.as<uint32_t>(), st);
    JG_HIP(hipGetLastError());
    ++w->waves_bucketed;
    // ids issued (the check ruled out running past 2^32 - 2: id_bound), names in (set, first entry) order
    w->n_names += n_new;
    w->id_bound += n_new;
    w->pool_used += nb;
    w->g1 = w->n_names;
    w->p1 = w->pool_used;
    queue_names(ctx, w);
    w->mark();
    w->last_cnt[0] = cnt[0], w->last_cnt[1] = cnt[1];
    if (cnt[0] + cnt[1] == 0) return true;
    if (!w->recs) {
        w->recs = new jg_orset();
        w->recs->ctx = ctx;
    }
    jg::set_dense(ctx, w->recs->add, cnt[0]);
    jg::set_dense(ctx, w->recs->rem, cnt[1]);
    w->recs->add.next = w->recs->rem.next = t_next;
    jg_stream_soa& a = w->recs->add;
    jg_stream_soa& r = w->recs->rem;
    hipLaunchKernelGGL(k_cb_records, dim3((unsigned)n_sets, 2), dim3(cb_threads(Pr)), cb_records_lds(Pr), ctx->stream, S, ST, RT, B, w->sid_id.as<uint32_t>(),
                       a.key.as<unsigned long long>(), a.tag.as<Tag16>(), a.ord.as<uint32_t>(), r.key.as<unsigned long long>(), r.tag.as<Tag16>(),
                       r.ord.as<uint32_t>());
    JG_HIP(hipGetLastError());
    jg::orset_merge_store(s, w->recs, w->external);  // a node wave: the node's final read brings the counts
    return true;
}

// Commit from the wave's tables: the distinct strings whose first entry lies before the limit resolved against
// the element table (new ones take ids in (set, first entry) order), the distinct records before the limit
// keyed, sorted and unioned into the store; ords = first tag slot (ordered like commit order, < next).
void commit_tables(jg_orset* s, jg_orset_wire* w, uint64_t limit) {
    jg_ctx* ctx = s->ctx;
    const uint64_t n = w->wn;
    static const bool tr = std::getenv("JANUS_TRACE_MERGE") != nullptr;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e6; };
    double tc[5] = {tr ? now() : 0};
    g_tmark[2] = tc[0];
    uint64_t lim_off = w->wnb;
    if (limit < n) {  // the limit message's byte offset
        jg::pin_get(ctx, 0, w->voff + limit, 8);
        jg::pin_sync(ctx);
        std::memcpy(&lim_off, jg::pin_at(ctx, 0), 8);
    }
    const uint32_t csi_lim = limit < n ? (uint32_t)((lim_off + kEntryDiv - 1) / kEntryDiv) : 0xFFFFFFFFu;
    const uint32_t t_lim = limit < n ? (uint32_t)((lim_off + kTagDiv - 1) / kTagDiv) : 0xFFFFFFFFu;
    const uint64_t t_next = (w->wnb + kTagDiv - 1) / kTagDiv + 1;  // every tag slot of the wave is below this
    ensure_sets(ctx, w, (uint64_t)w->max_set + 1);
    ensure_names(ctx, w, 0, 0);
    StrTab ST = str_tab(w);
    RecTab RT = rec_tab(w);
    // the wave's strings (the table's list; those first named past the limit are skipped)
    // the sub-lists packed into one list each (offsets from the counts: one read, one pack launch per table)
    const std::vector<unsigned long long>& lc = w->lc;  // read by the check with the first bad message
    if (w->spec) {  // packed by the check (spec_commit_prep): the offsets on the device gave the same layout
        uint64_t ns = 0, nrec = 0;
        for (uint32_t j = 0; j < kLists; ++j) ns += lc[(1 + j) * kCountStride], nrec += lc[(1 + kLists + j) * kCountStride];
        ST.list = w->st_packed.as<uint32_t>();
        RT.list = w->rt_packed.as<uint32_t>();
        commit_packed(s, w, ST, RT, ns, nrec, csi_lim, t_lim, t_next, tc, tr);
        return;
    }
    unsigned long long offs[2][kLists + 1];
    for (int t = 0; t < 2; ++t) {
        offs[t][0] = 0;
        for (uint32_t j = 0; j < kLists; ++j) offs[t][j + 1] = offs[t][j] + lc[(1 + t * kLists + j) * kCountStride];
    }
    const uint64_t ns = offs[0][kLists], nrec = offs[1][kLists];
    ensure(w->loffs, sizeof offs);
    ensure(w->st_packed, ns * 4 + 4);
    ensure(w->rt_packed, nrec * 4 + 4);
    // from the context's page-locked write area (a pageable source is staged by the runtime, a host round trip);
    // nothing else writes there before this wave's commit has synced
    static_assert(sizeof offs <= jg::kPinBytes - jg::kPinRead, "offsets fit the page-locked write area");
    void* hoffs = static_cast<char*>(ctx->hstat) + jg::kPinRead;
    std::memcpy(hoffs, offs, sizeof offs);
    JG_HIP(hipMemcpyAsync(w->loffs.p, hoffs, sizeof offs, hipMemcpyHostToDevice, ctx->stream));
    const auto* doffs = w->loffs.as<unsigned long long>();
    if (ns)
        hipLaunchKernelGGL(k_list_pack, dim3(blocks_for(ns)), dim3(kBlock), 0, ctx->stream, ST.list, ST.sub_cap, doffs, w->st_packed.as<uint32_t>());
    if (nrec)
        hipLaunchKernelGGL(k_list_pack, dim3(blocks_for(nrec)), dim3(kBlock), 0, ctx->stream, RT.list, RT.sub_cap, doffs + kLists + 1,
                           w->rt_packed.as<uint32_t>());
    JG_HIP(hipGetLastError());
    ST.list = w->st_packed.as<uint32_t>();  // the commit kernels read the packed lists
    RT.list = w->rt_packed.as<uint32_t>();
    commit_packed(s, w, ST, RT, ns, nrec, csi_lim, t_lim, t_next, tc, tr);
}

// The table commit from the packed lists: the bucket commit, or the radix path.
void commit_packed(jg_orset* s, jg_orset_wire* w, StrTab ST, RecTab RT, uint64_t ns, uint64_t nrec, uint32_t csi_lim, uint32_t t_lim,
                   uint64_t t_next, double* tc, bool tr) {
    jg_ctx* ctx = s->ctx;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() * 1e6; };
    unsigned long long* st = status_words(w);
    const Sparse S = sparse_of(w);
    // room for every listed string (an upper bound of the new ones: the element tables then grow ahead of the
    // names, not at each doubling of exact counts — measured, the exact count moved a table rebuild into the
    // timed waves) and their bytes: exactly the claims' total when the check scanned them for a whole-wave commit
    // (both commit paths issue exactly those names), else the wave's bytes
    const bool exact = w->spec && csi_lim == 0xFFFFFFFFu && t_lim == 0xFFFFFFFFu && w->lc.size() > 1 && w->lc[1] == 0;
    if (tr) g_tmark[3] = now();
    if (ns) ensure_names(ctx, w, ns, exact ? w->spec_h[1] : w->wnb);
    if (tr) g_tmark[4] = now();
    if (commit_buckets(s, w, ST, RT, ns, nrec, csi_lim, t_lim, t_next)) {
        if (tr) std::fprintf(stderr, "commit_tables: bucket commit %.0f us (%llu strings, %llu records listed)\n", now() - tc[0],
                             (unsigned long long)ns, (unsigned long long)nrec);
        return;
    }
    // strings: each looked up (new ones keyed by (set, first entry), known ones kNone), all sorted by that key
    // (known last), new ids assigned in that order; no host round trip until the record counts are read
    const unsigned long long init[4] = {0, 0, w->pool_used, 0};
    JG_HIP(hipMemcpyAsync(st, init, sizeof init, hipMemcpyHostToDevice, ctx->stream));
    if (ns) {
        ensure(w->newk, ns * 8);
        ensure(w->snk, ns * 8);
        ensure(w->snv, ns * 4);
        hipLaunchKernelGGL(k_ow_sresolve, dim3(blocks_for(ns)), dim3(kBlock), 0, ctx->stream, S, w->vbytes, ST, ns, csi_lim, names_of(w),
                           w->sid_id.as<uint32_t>(), w->newk.as<unsigned long long>());
        JG_HIP(hipGetLastError());
        sort_pairs(ctx, w, w->newk.as<unsigned long long>(), w->snk.as<unsigned long long>(), ST.list, w->snv.as<uint32_t>(), ns, 64);
        hipLaunchKernelGGL(k_ow_sassign, dim3(blocks_for(ns)), dim3(kBlock), 0, ctx->stream, S, w->vbytes, ST, w->snk.as<unsigned long long>(),
                           w->snv.as<uint32_t>(), ns, w->n_names, names_of(w), w->sid_id.as<uint32_t>(), st);
        JG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_ow_snext_ids, dim3(blocks_for(ns)), dim3(kBlock), 0, ctx->stream, w->snk.as<unsigned long long>(), ns, names_of(w));
        JG_HIP(hipGetLastError());
    }
    // the wave's records (the table's list), per side, first occurring before the limit
    ensure(w->fidx, nrec * 4 + 4);
    ensure(w->fslot, nrec * 4 + 4);
    JG_HIP(hipMemsetAsync(st + 4, 0, 16, ctx->stream));
    if (nrec) {
        select_marked(ctx, w, RecLive{RT.list, RT.slot, S.trk, t_lim, 0}, nrec, w->fidx.as<uint32_t>(), st + 4);
        select_marked(ctx, w, RecLive{RT.list, RT.slot, S.trk, t_lim, 1}, nrec, w->fslot.as<uint32_t>(), st + 5);
    }
    unsigned long long hh[6];  // [1] new strings, [2] pool bytes used, [3] id overflow, [4] [5] records per side
    if (tr) tc[1] = now();
    read_words(ctx, st, hh, 6);
    if (tr) tc[2] = now();
    JG_REQUIRE(hh[3] == 0, JG_ESTATE, "jg_orset_wave_commit: too many elements in one OR-Set (2^32 - 2 ids)");
    w->n_names += hh[1];
    w->id_bound += hh[1];
    w->pool_used = hh[2];
    w->g1 = w->n_names;
    w->p1 = w->pool_used;
    queue_names(ctx, w);
    w->mark();
    const unsigned long long cnt[2] = {hh[4], hh[5]};
    w->last_cnt[0] = cnt[0], w->last_cnt[1] = cnt[1];
    if (cnt[0] + cnt[1] == 0) return;
    for (int sd = 0; sd < 2; ++sd) {
        ensure(w->dk[sd], cnt[sd] * 8 + 8);
        ensure(w->dt[sd], cnt[sd] * 16 + 16);
        ensure(w->ds[sd], cnt[sd] * 4 + 4);
        if (cnt[sd] == 0) continue;
        hipLaunchKernelGGL(k_ow_rgather, dim3(blocks_for(cnt[sd])), dim3(kBlock), 0, ctx->stream, S, ST, RT, w->sid_id.as<uint32_t>(),
                           (sd ? w->fslot : w->fidx).as<uint32_t>(), st + 4 + sd, w->dk[sd].as<unsigned long long>(), w->dt[sd].as<Tag16>(),
                           w->ds[sd].as<uint32_t>());
        JG_HIP(hipGetLastError());
    }
    if (!w->recs) {
        w->recs = new jg_orset();
        w->recs->ctx = ctx;
    }
    const int key_bits = 32 + bits_for(w->max_set);
    const uint64_t nmax = std::max(cnt[0], cnt[1]);
    ensure(w->rk, nmax * 8);
    ensure(w->rk2, nmax * 8);
    sort_side_begin(ctx, w, 0, cnt[0], key_bits, t_next, w->recs->add, st + 6);
    sort_side_begin(ctx, w, 1, cnt[1], key_bits, t_next, w->recs->rem, st + 7);
    unsigned long long long_run[2];
    read_words(ctx, st + 6, long_run, 2);
    if (tr) tc[3] = now();
    sort_side_end(ctx, w, 0, cnt[0], key_bits, w->recs->add, long_run[0] != 0, &RT.slot[0].mint, 4);
    sort_side_end(ctx, w, 1, cnt[1], key_bits, w->recs->rem, long_run[1] != 0, &RT.slot[0].mint, 4);
    jg::orset_merge_store(s, w->recs, w->external);  // a node wave: the node's final read brings the counts
    if (tr) {
        tc[4] = now();
        std::fprintf(stderr, "commit_tables: strings queued %.0f us, counts read %.0f, record sorts + long-run read %.0f, union %.0f (%llu strings, %llu + %llu records)\n",
                     tc[1] - tc[0], tc[2] - tc[1], tc[3] - tc[2], tc[4] - tc[3], (unsigned long long)ns, cnt[0], cnt[1]);
    }
}

void commit_wave(jg_orset* s, jg_orset_wire* w, uint64_t limit) {
    jg_ctx* ctx = s->ctx;
    w->g0 = w->g1 = w->n_names;
    w->p0 = w->p1 = w->pool_used;
    if (limit == 0) return;
    if (w->tables_ok) {
        ++w->waves_fast;
        commit_tables(s, w, limit);
        return;
    }
    ++w->waves_sorted;
    const uint64_t ne = w->n_ent, nt = w->n_tag;
    w->g0 = w->g1 = w->n_names;
    w->p0 = w->p1 = w->pool_used;
    if (limit == 0 || (ne == 0 && nt == 0)) return;
    ensure_sets(ctx, w, (uint64_t)w->max_set + 1);
    ensure_names(ctx, w, 0, 0);
    unsigned long long* st = status_words(w);
    const Entries E = entries_of(w);
    ensure(w->gid, ne * 4 + 4);
    ensure(w->eid, ne * 4 + 4);
    uint64_t nnew = 0;
    if (ne) {
        ensure(w->newk, ne * 8);
        ensure(w->newv, ne * 4);
        JG_HIP(hipMemsetAsync(st, 0, 64, ctx->stream));
        hipLaunchKernelGGL(k_ow_resolve, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->vbytes,
                           w->skey.as<unsigned long long>(), w->sval.as<uint32_t>(), w->label.as<uint32_t>(), ne, limit, names_of(w),
                           w->gid.as<uint32_t>(), w->newk.as<unsigned long long>());
        JG_HIP(hipGetLastError());
        // the marked sorted indices compacted (count into st[1]) and their keys gathered; the sort below
        // orders them by (set, first entry)
        ensure(w->cnk, ne * 8);
        select_marked(ctx, w, IsNewAt{w->newk.as<unsigned long long>()}, ne, w->newv.as<uint32_t>(), st + 1);
        hipLaunchKernelGGL(k_ow_gather_new, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, w->newk.as<unsigned long long>(),
                           w->newv.as<uint32_t>(), st + 1, w->cnk.as<unsigned long long>());
        JG_HIP(hipGetLastError());
        unsigned long long h[2];
        read_words(ctx, st, h, 2);
        nnew = h[1];
    }
    if (nnew) {
        ensure_names(ctx, w, nnew, w->wnb);
        ensure(w->snk, nnew * 8);
        ensure(w->snv, nnew * 4);
        sort_pairs(ctx, w, w->cnk.as<unsigned long long>(), w->snk.as<unsigned long long>(), w->newv.as<uint32_t>(), w->snv.as<uint32_t>(), nnew,
                   32 + bits_for(w->max_set));
        const unsigned long long init[4] = {0, 0, w->pool_used, 0};
        JG_HIP(hipMemcpyAsync(st, init, sizeof init, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(k_ow_assign, dim3(blocks_for(nnew)), dim3(kBlock), 0, ctx->stream, E, w->vbytes, w->skey.as<unsigned long long>(),
                           w->snk.as<unsigned long long>(), w->snv.as<uint32_t>(), nnew, w->n_names, names_of(w), w->gid.as<uint32_t>(), st);
        JG_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_ow_next_ids, dim3(blocks_for(nnew)), dim3(kBlock), 0, ctx->stream, w->snk.as<unsigned long long>(), nnew, names_of(w));
        JG_HIP(hipGetLastError());
        unsigned long long h[4];
        read_words(ctx, st, h, 4);
        JG_REQUIRE(h[3] == 0, JG_ESTATE, "jg_orset_wave_commit: too many elements in one OR-Set (2^32 - 2 ids)");
        w->n_names += nnew;
        w->id_bound += nnew;
        w->pool_used = h[2];
        w->g1 = w->n_names;
        w->p1 = w->pool_used;
        queue_names(ctx, w);
        w->mark();
    }
    if (ne) {
        hipLaunchKernelGGL(k_ow_entry_ids, dim3(blocks_for(ne)), dim3(kBlock), 0, ctx->stream, w->sval.as<uint32_t>(), w->label.as<uint32_t>(),
                           w->gid.as<uint32_t>(), ne, w->eid.as<uint32_t>());
        JG_HIP(hipGetLastError());
    }
    // tag records: keys, de-duplication, sort, union into the store
    ensure(w->rkey, nt * 8 + 8);
    ensure(w->rside, nt + 1);
    const uint64_t tcap = pow2_at_least(2 * nt);
    ensure(w->dtab, tcap * 8);
    ensure(w->dmin, tcap * 4);
    for (int sd = 0; sd < 2; ++sd) {
        ensure(w->dk[sd], nt * 8 + 8);
        ensure(w->dt[sd], nt * 16 + 16);
        ensure(w->ds[sd], nt * 4 + 4);
    }
    hipLaunchKernelGGL(k_ow_rec_keys, dim3(blocks_for(nt)), dim3(kBlock), 0, ctx->stream, E, w->vmset, w->tref.as<unsigned long long>(),
                       w->eid.as<uint32_t>(), nt, limit, w->rkey.as<unsigned long long>(), w->rside.as<uint8_t>());
    JG_HIP(hipGetLastError());
    JG_HIP(hipMemsetAsync(w->dtab.p, 0, tcap * 8, ctx->stream));
    JG_HIP(hipMemsetAsync(w->dmin.p, 0xFF, tcap * 4, ctx->stream));
    JG_HIP(hipMemsetAsync(st + 4, 0, 16, ctx->stream));
    ensure(w->fsel, nt + 1);
    ensure(w->fslot, nt * 4 + 4);
    ensure(w->fidx, nt * 4 + 4);
    hipLaunchKernelGGL(k_ow_dedup, dim3(blocks_for(nt)), dim3(kBlock), 0, ctx->stream, w->rkey.as<unsigned long long>(), w->rside.as<uint8_t>(),
                       w->tval.as<Tag16>(), nt, w->dtab.as<unsigned long long>(), tcap - 1, w->dmin.as<uint32_t>(), w->fsel.as<uint8_t>(),
                       w->fslot.as<uint32_t>());
    JG_HIP(hipGetLastError());
    for (int sd = 0; sd < 2; ++sd) {  // each side's distinct records, compacted in tag order
        select_marked(ctx, w, OnSide{w->fsel.as<uint8_t>(), (uint8_t)(1 + sd)}, nt, w->fidx.as<uint32_t>(), st + 4 + sd);
        hipLaunchKernelGGL(k_ow_gather_side, dim3(blocks_for(nt)), dim3(kBlock), 0, ctx->stream, w->fidx.as<uint32_t>(), st + 4 + sd,
                           w->rkey.as<unsigned long long>(), w->tval.as<Tag16>(), w->fslot.as<uint32_t>(), w->dk[sd].as<unsigned long long>(),
                           w->dt[sd].as<Tag16>(), w->ds[sd].as<uint32_t>());
        JG_HIP(hipGetLastError());
    }
    unsigned long long cnt[2];
    read_words(ctx, st + 4, cnt, 2);
    w->last_cnt[0] = cnt[0], w->last_cnt[1] = cnt[1];
    if (cnt[0] + cnt[1] == 0) return;
    if (!w->recs) {  // the wave's sorted records: kept across waves (no allocation per commit)
        w->recs = new jg_orset();
        w->recs->ctx = ctx;
    }
    const int key_bits = 32 + bits_for(w->max_set);
    const uint64_t nmax = std::max(cnt[0], cnt[1]);  // the radix-key buffers serve both sides: sized once,
    ensure(w->rk, nmax * 8);                           // so no reallocation frees one that queued work reads
    ensure(w->rk2, nmax * 8);
    sort_side_begin(ctx, w, 0, cnt[0], key_bits, nt, w->recs->add, st + 6);
    sort_side_begin(ctx, w, 1, cnt[1], key_bits, nt, w->recs->rem, st + 7);
    unsigned long long long_run[2];
    read_words(ctx, st + 6, long_run, 2);
    sort_side_end(ctx, w, 0, cnt[0], key_bits, w->recs->add, long_run[0] != 0, w->dmin.as<uint32_t>(), 1);
    sort_side_end(ctx, w, 1, cnt[1], key_bits, w->recs->rem, long_run[1] != 0, w->dmin.as<uint32_t>(), 1);
    jg::orset_merge_store(s, w->recs, w->external);  // a node wave: the node's final read brings the counts
}

void close_wave(jg_orset_wire* w) {
    w->open = false;
    w->spec = false;
    w->external = false;
    w->checked = false;
    w->wn = w->wnb = 0;
    w->max_set = 0;
    w->first_bad = kNone;
}


// jg_orset_encode_json: gather the sets' records below the limits, order them (runs by section and element, tags
// by ord), size every state, then write them (see the kernels' header comment).  Two round trips: the record
// count (gather) and the states' offsets; a third copy brings the bytes.
void encode_sets(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* add_lim, const uint64_t* rem_lim, uint64_t* off, uint8_t* out,
                 uint64_t cap, uint8_t* sha) {
    jg_ctx* ctx = s->ctx;
    jg_orset_wire* w = wire_of(s);
    if (!w->itab_cap || !w->tab_cap) ensure_names(ctx, w, 0, 0);  // a store that never saw a name: empty tables
    const bool lim = add_lim != nullptr;
    auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
    char* q0 = static_cast<char*>(jg::scratch(ctx, ctx->scratch, al(n * 4) + (lim ? al(2 * n * 8) : 0) + 256));
    auto* d_sets = reinterpret_cast<uint32_t*>(q0);
    auto* d_lim = lim ? reinterpret_cast<unsigned long long*>(q0 + al(n * 4)) : nullptr;
    JG_HIP(hipMemcpyAsync(d_sets, set, n * 4, hipMemcpyHostToDevice, ctx->stream));
    if (lim) {
        std::vector<unsigned long long> l(2 * n);
        for (uint64_t i = 0; i < n; ++i) l[2 * i] = add_lim[i], l[2 * i + 1] = rem_lim[i];
        JG_HIP(hipMemcpyAsync(d_lim, l.data(), 2 * n * 8, hipMemcpyHostToDevice, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));  // l is a local
    }
    const jg::OrsetGathered G = jg::orset_gather_sets(s, n, d_sets, d_lim, w->enc_g);
    const uint64_t R = G.R;
    const EncRec E{G.key, G.tlo, G.thi, G.ord, G.qs};
    // the encoder's arrays, one block
    const uint64_t R1 = R + 1;
    const uint64_t sz[] = {al(R * 4), 256, al(R * 4), al(R * 4), al(R * 4), al(R * 4), al(R * 4), 256, al(R * 8), al(R * 4), al(R * 8), al(R * 4),
                           al(R * 4), al(R1 * 8), al(R1 * 8), al(R1 * 8), al(R1 * 8), al(4 * n * 8), al(4 * n * 4), al((n + 1) * 8), al((n + 1) * 8),
                           al(R * 8), al(R * 4), al(R * 8), al(R * 4), al(R * 8), 256};
    uint64_t tot = 0;
    for (uint64_t x : sz) tot += x;
    ensure(w->enc, tot);
    char* p = w->enc.as<char>();
    auto take = [&](int i) { char* r = p; p += sz[i]; return r; };
    auto* kidx = reinterpret_cast<uint32_t*>(take(0));
    auto* K = reinterpret_cast<unsigned long long*>(take(1));
    auto* hf = reinterpret_cast<uint32_t*>(take(2));
    auto* rid = reinterpret_cast<uint32_t*>(take(3));
    auto* rstart = reinterpret_cast<uint32_t*>(take(4));
    auto* rend = reinterpret_cast<uint32_t*>(take(5));
    auto* rfirst = reinterpret_cast<uint32_t*>(take(6));
    auto* nruns = reinterpret_cast<unsigned long long*>(take(7));
    auto* rkey = reinterpret_cast<unsigned long long*>(take(8));
    auto* rval = reinterpret_cast<uint32_t*>(take(9));
    auto* skey = reinterpret_cast<unsigned long long*>(take(10));
    auto* srun = reinterpret_cast<uint32_t*>(take(11));
    auto* rrank = reinterpret_cast<uint32_t*>(take(12));
    auto* cnt = reinterpret_cast<unsigned long long*>(take(13));
    auto* tlen = reinterpret_cast<unsigned long long*>(take(14));
    auto* rpos = reinterpret_cast<unsigned long long*>(take(15));
    auto* cpos = reinterpret_cast<unsigned long long*>(take(16));
    auto* qsec = reinterpret_cast<unsigned long long*>(take(17));
    auto* sfirst = reinterpret_cast<uint32_t*>(take(18));
    auto* qlen = reinterpret_cast<unsigned long long*>(take(19));
    auto* qoff = reinterpret_cast<unsigned long long*>(take(20));
    auto* reck = reinterpret_cast<unsigned long long*>(take(21));
    auto* recv = reinterpret_cast<uint32_t*>(take(22));
    auto* reck2 = reinterpret_cast<unsigned long long*>(take(23));
    auto* srec = reinterpret_cast<uint32_t*>(take(24));
    auto* rtags = reinterpret_cast<unsigned long long*>(take(25));
    auto* err = reinterpret_cast<unsigned*>(take(26));
    JG_HIP(hipMemsetAsync(qsec, 0, 4 * n * 8, ctx->stream));
    JG_HIP(hipMemsetAsync(sfirst, 0xFF, 4 * n * 4, ctx->stream));
    JG_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
    JG_HIP(hipMemsetAsync(K, 0, 8, ctx->stream));
    JG_HIP(hipMemsetAsync(nruns, 0, 8, ctx->stream));
    const Names N = names_of(w);
    const unsigned gR = blocks_for(R);
    if (R) {
        size_t temp = 0;
        hipcub::CountingInputIterator<uint32_t> iota(0);
        JG_HIP(hipcub::DeviceSelect::Flagged(nullptr, temp, iota, G.keep, kidx, K, (int)R, ctx->stream));
        JG_HIP(hipcub::DeviceSelect::Flagged(cub_temp(w, temp), temp, iota, G.keep, kidx, K, (int)R, ctx->stream));
        hipLaunchKernelGGL(k_enc_heads, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, K, R, hf);
        JG_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, temp, hf, rid, (int)R, ctx->stream));
        JG_HIP(hipcub::DeviceScan::InclusiveSum(cub_temp(w, temp), temp, hf, rid, (int)R, ctx->stream));
        hipLaunchKernelGGL(k_enc_runs, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, K, rid, rstart, rend, rfirst, nruns);
        hipLaunchKernelGGL(k_enc_first_ord, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, K, rid, rfirst);
        hipLaunchKernelGGL(k_enc_run_keys, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, rstart, rfirst, nruns, R, rkey, rval);
        JG_HIP(hipGetLastError());
        JG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, rkey, skey, rval, srun, (int)R, 0, 64, ctx->stream));
        JG_HIP(hipcub::DeviceRadixSort::SortPairs(cub_temp(w, temp), temp, rkey, skey, rval, srun, (int)R, 0, 64, ctx->stream));
        hipLaunchKernelGGL(k_enc_run_len, dim3(gR), dim3(kBlock), 0, ctx->stream, E, N, kidx, rstart, rend, skey, srun, nruns, R, rrank, cnt, tlen, qsec,
                           sfirst, err);
        hipLaunchKernelGGL(k_enc_rec_keys, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, K, rid, rrank, R, reck, recv);
        JG_HIP(hipGetLastError());
        JG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, reck, reck2, recv, srec, (int)R, 0, 64, ctx->stream));
        JG_HIP(hipcub::DeviceRadixSort::SortPairs(cub_temp(w, temp), temp, reck, reck2, recv, srec, (int)R, 0, 64, ctx->stream));
        JG_HIP(hipMemsetAsync(tlen + R, 0, 8, ctx->stream));
        JG_HIP(hipMemsetAsync(cnt + R, 0, 8, ctx->stream));
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, tlen, rpos, (int)R1, ctx->stream));
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(cub_temp(w, temp), temp, tlen, rpos, (int)R1, ctx->stream));
        JG_HIP(hipcub::DeviceScan::ExclusiveSum(cub_temp(w, temp), temp, cnt, cpos, (int)R1, ctx->stream));
    }
    hipLaunchKernelGGL(k_enc_qlen, dim3(blocks_for(n + 1)), dim3(kBlock), 0, ctx->stream, qsec, n, qlen);
    JG_HIP(hipGetLastError());
    size_t temp = 0;
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, qlen, qoff, (int)(n + 1), ctx->stream));
    JG_HIP(hipcub::DeviceScan::ExclusiveSum(cub_temp(w, temp), temp, qlen, qoff, (int)(n + 1), ctx->stream));
    JG_HIP(hipMemcpyAsync(off, qoff, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    jg::pin_get(ctx, 0, err, 4);
    jg::pin_sync(ctx);  // the stream's copies above are done too
    unsigned e;
    std::memcpy(&e, jg::pin_at(ctx, 0), 4);
    JG_REQUIRE(e == 0, JG_ESTATE, "jg_orset_encode_json: a record names an element id the store's element table does not hold (names not synced)");
    if (!out) return;  // size query
    JG_REQUIRE(off[n] <= cap, JG_ESTATE, "jg_orset_encode_json: %llu bytes exceed cap %llu", (unsigned long long)off[n], (unsigned long long)cap);
    auto* dout = static_cast<uint8_t*>(jg::scratch(ctx, ctx->scratch2, off[n] + 64));
    hipLaunchKernelGGL(k_enc_fixed, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, qoff, qsec, n, dout);
    if (R) {
        hipLaunchKernelGGL(k_enc_run_text, dim3(gR), dim3(kBlock), 0, ctx->stream, E, N, kidx, rstart, skey, srun, nruns, rpos, tlen, sfirst, qoff, qsec,
                           rtags, dout);
        hipLaunchKernelGGL(k_enc_rec_text, dim3(gR), dim3(kBlock), 0, ctx->stream, E, kidx, K, srec, rid, rrank, cpos, rtags, dout);
    }
    JG_HIP(hipGetLastError());
    if (sha) jg::sha256_device(ctx, dout, reinterpret_cast<const uint64_t*>(qoff), n, sha);  // each state's SHA-256 (ComputeDigest's first level)
    JG_HIP(hipMemcpyAsync(out, dout, off[n], hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
}
}  // namespace

namespace {
// The check and the commit of the open wave: the ABI's (which a held store refuses) and a node wave's own
// (orset_node_check / orset_node_commit, which hold the store).
int wave_check_call(jg_orset* s, uint64_t* bad_msg, bool node) {
    if (bad_msg) *bad_msg = UINT64_MAX;
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        if (!node) jg::require_writable(s, "jg_orset_wave_check");
        JG_REQUIRE(s && s->wire && s->wire->open, JG_EINVAL, "jg_orset_wave_check: no open wave (jg_orset_wave_begin)");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg_orset_wire* w = s->wire;
        if (!w->checked) check_wave(s, w);
        if (w->first_bad == kNone) return;
        if (bad_msg) *bad_msg = w->first_bad;
        unsigned long long e;
        JG_HIP(hipMemcpyAsync(&e, w->err.as<unsigned long long>() + w->first_bad, 8, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        const bool state = (e & 3) == kKindState;
        jg::fail(state ? JG_ESTATE : JG_EINVAL, "OR-Set state message %llu is rejected by ORSetMsg.Decode / Merge (%s at byte %llu)",
                 (unsigned long long)w->first_bad, state ? "an element with an empty tag set" : "JsonException", (unsigned long long)(e >> 2));
    });
}

int wave_commit_call(jg_orset* s, uint64_t limit, bool node) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        if (!node) jg::require_writable(s, "jg_orset_wave_commit");
        JG_REQUIRE(s && s->wire && s->wire->open, JG_EINVAL, "jg_orset_wave_commit: no open wave (jg_orset_wave_begin)");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg_orset_wire* w = s->wire;
        if (!w->checked) check_wave(s, w);
        JG_REQUIRE(limit <= w->wn, JG_EINVAL, "jg_orset_wave_commit: limit %llu beyond the wave (%llu messages)", (unsigned long long)limit,
                   (unsigned long long)w->wn);
        JG_REQUIRE(w->first_bad == kNone || limit <= w->first_bad, JG_EINVAL, "jg_orset_wave_commit: limit %llu passes the bad message %llu",
                   (unsigned long long)limit, (unsigned long long)w->first_bad);
        try {
            commit_wave(s, w, limit);
        } catch (...) {
            close_wave(w);
            throw;
        }
        close_wave(w);
    });
}
}  // namespace

namespace jg {
// ---- node waves (csrc/node.hip): the node's buffers hold every kind's messages; mset[m] = kSkipIdx for
// another kind's.  begin sizes the per-message arrays for n messages / nbytes payload bytes.
void orset_node_begin(jg_orset* s, uint8_t* bytes, uint64_t* off, uint32_t* mset, uint64_t n, uint64_t nbytes, uint32_t max_set) {
    jg_ctx* ctx = s->ctx;
    jg_orset_wire* w = wire_of(s);
    close_wave(w);
    w->external = true;
    w->vbytes = bytes;
    w->voff = off;
    w->vmset = mset;
    grow_wave(ctx, w, std::max<uint64_t>(n, 1), std::max<uint64_t>(nbytes, 1));
    tables_begin(ctx, w, n, nbytes);
    w->wn = n;
    w->wnb = nbytes;
    w->max_set = max_set;
    w->any_set = true;
    w->open = true;
}
void orset_node_parse(jg_orset* s, uint64_t m0, uint64_t m1) { launch_parse(s->ctx, s->wire, m0, m1); }
// JG_OK, or the code of the first rejected message (*bad, why).
int orset_node_check(jg_orset* s, uint64_t n, uint64_t nbytes, uint64_t* bad, std::string* why) {
    *bad = UINT64_MAX;
    s->wire->wn = n;
    s->wire->wnb = nbytes;
    // the union targets sized for the store plus twice the last wave's distinct records while this wave's
    // uploads are still in flight (a growing store reallocates here, not behind the last upload)
    const uint64_t* lc = s->wire->last_cnt;
    static const bool tr = std::getenv("JANUS_TRACE_MERGE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    orset_reserve_union(s, 2 * lc[0] + 4096, 2 * lc[1] + 4096);
    if (tr) std::fprintf(stderr, "orset_node_check: union targets reserved in %.0f us\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
    const int rc = wave_check_call(s, bad, true);
    if (rc != JG_OK) {
        char buf[1024];
        jg_last_error(buf, sizeof buf);
        *why = buf;
    }
    return rc;
}
void orset_node_commit(jg_orset* s, uint64_t limit) {
    const int rc = wave_commit_call(s, limit, true);
    if (rc != JG_OK) {
        char buf[1024];
        jg_last_error(buf, sizeof buf);
        fail(rc, "%s", buf);
    }
}
void orset_node_abort(jg_orset* s) {
    if (s->wire) close_wave(s->wire);
}
// No element ids issued yet by this call (jg_orset_wave_names reports the last commit's: a node call that
// ends before committing must not leave the previous call's there).
void orset_node_no_names(jg_orset* s) {
    if (!s->wire) return;
    s->wire->g0 = s->wire->g1 = s->wire->n_names;
    s->wire->p0 = s->wire->p1 = s->wire->pool_used;
}

void orset_wire_free(jg_orset_wire* w) {
    if (w) delete w->recs;
    delete w;
}

void orset_wire_free_retired(jg_orset_wire* w) {
    for (void* p : w->retired) (void)hipFree(p);
    w->retired.clear();
}
}  // namespace jg

extern "C" {

int jg_orset_names_sync(jg_orset* s, uint64_t n_sets, const uint32_t* set, const uint32_t* next_id, const uint8_t* cleared, uint64_t n_names,
                        const uint32_t* name_set, const uint32_t* name_id, const uint64_t* off, const uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_names_sync");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_names_sync: store is NULL");
        JG_REQUIRE((n_sets == 0 || (set && next_id && cleared)) && (n_names == 0 || (name_set && name_id && off && bytes)), JG_EINVAL,
                   "jg_orset_names_sync: NULL argument");
        JG_REQUIRE(n_names == 0 || off[0] == 0, JG_EINVAL, "jg_orset_names_sync: off[0] must be 0");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg_orset_wire* w = wire_of(s);
        JG_REQUIRE(!w->open, JG_EINVAL, "jg_orset_names_sync: a wave is open");
        uint64_t mx = 0, idb = 0;
        for (uint64_t i = 0; i < n_sets; ++i) mx = std::max<uint64_t>(mx, (uint64_t)set[i] + 1), idb = std::max<uint64_t>(idb, next_id[i]);
        for (uint64_t i = 0; i < n_names; ++i) {
            JG_REQUIRE(off[i + 1] >= off[i] && off[i + 1] - off[i] < 0x7FFFFFFFull, JG_EINVAL, "jg_orset_names_sync: bad offsets at name %llu",
                       (unsigned long long)i);
            JG_REQUIRE(name_id[i] < JG_NULL_ELEM - 1, JG_EINVAL, "jg_orset_names_sync: id %u out of range", name_id[i]);
            mx = std::max<uint64_t>(mx, (uint64_t)name_set[i] + 1);
        }
        if (mx == 0) return;
        ensure_sets(ctx, w, mx);
        const uint64_t nb = n_names ? off[n_names] : 0;
        ensure_names(ctx, w, n_names, nb);
        const size_t need = n_sets * 9 + n_names * 8 + (n_names + 1) * 8 + 64;
        char* stage = static_cast<char*>(jg::scratch(ctx, ctx->scratch, need));
        auto* d_set = reinterpret_cast<uint32_t*>(stage);
        auto* d_next = d_set + n_sets;
        auto* d_nset = d_next + n_sets;
        auto* d_nid = d_nset + n_names;
        auto* d_off = reinterpret_cast<uint64_t*>(stage + (((n_sets * 8 + n_names * 8) + 15) & ~15ull));
        auto* d_clr = reinterpret_cast<uint8_t*>(d_off + n_names + 1);
        if (n_sets) {
            JG_HIP(hipMemcpyAsync(d_set, set, n_sets * 4, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync(d_next, next_id, n_sets * 4, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync(d_clr, cleared, n_sets, hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(k_sets_update, dim3(blocks_for(n_sets)), dim3(kBlock), 0, ctx->stream, names_of(w), d_set, d_next, d_clr, n_sets);
            JG_HIP(hipGetLastError());
        }
        if (n_names) {
            JG_HIP(hipMemcpyAsync(d_nset, name_set, n_names * 4, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync(d_nid, name_id, n_names * 4, hipMemcpyHostToDevice, ctx->stream));
            JG_HIP(hipMemcpyAsync(d_off, off, (n_names + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
            if (nb) JG_HIP(hipMemcpyAsync(w->pool.as<uint8_t>() + w->pool_used, bytes, nb, hipMemcpyHostToDevice, ctx->stream));
            hipLaunchKernelGGL(k_names_put, dim3(blocks_for(n_names)), dim3(kBlock), 0, ctx->stream, names_of(w), w->n_names, w->pool_used, d_nset, d_nid,
                               d_off, n_names, w->kmask, w->salt);
            JG_HIP(hipGetLastError());
        }
        JG_HIP(hipStreamSynchronize(ctx->stream));
        w->n_names += n_names;
        w->id_bound = std::max(w->id_bound, idb);
        w->pool_used += nb;
        w->mark();
    });
}

int jg_orset_wave_begin(jg_orset* s, uint64_t cap_msgs, uint64_t cap_bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_wave_begin");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_wave_begin: store is NULL");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        jg_orset_wire* w = wire_of(s);
        close_wave(w);
        grow_wave(ctx, w, std::max<uint64_t>(cap_msgs, 1), std::max<uint64_t>(cap_bytes, 1));
        tables_begin(ctx, w, cap_msgs, cap_bytes);
        JG_HIP(hipMemsetAsync(w->off.p, 0, 8, ctx->stream));  // off[0] = 0
        // the uploads run on ctx->copy: the previous wave's kernels must be done with these buffers
        JG_HIP(hipStreamSynchronize(ctx->stream));
        w->open = true;
    });
}

int jg_orset_wave_append(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* off, const uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_wave_append");
        JG_REQUIRE(s && s->wire && s->wire->open, JG_EINVAL, "jg_orset_wave_append: no open wave (jg_orset_wave_begin)");
        jg_orset_wire* w = s->wire;
        JG_REQUIRE(!w->checked, JG_EINVAL, "jg_orset_wave_append: the wave was already checked");
        if (n == 0) return;
        JG_REQUIRE(set && off && bytes, JG_EINVAL, "jg_orset_wave_append: NULL argument");
        JG_REQUIRE(off[0] == 0, JG_EINVAL, "jg_orset_wave_append: off[0] must be 0");
        JG_REQUIRE(w->wn + n < 0x7FFFFFF0ull, JG_EINVAL, "jg_orset_wave_append: at most 2^31 messages per wave");
        uint32_t mx = w->max_set;
        for (uint64_t i = 0; i < n; ++i) {
            JG_REQUIRE(off[i + 1] >= off[i], JG_EINVAL, "jg_orset_wave_append: offsets decrease at message %llu", (unsigned long long)i);
            JG_REQUIRE(set[i] < 0xFFFFFFF0u, JG_EINVAL, "jg_orset_wave_append: set id %u out of range", set[i]);
            mx = std::max(mx, set[i]);
        }
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        const uint64_t m0 = w->wn, b0 = w->wnb, nb = off[n];
        grow_wave(ctx, w, m0 + n, b0 + nb);
        // chunk k+1's upload (copy stream) overlaps chunk k's parse (compute stream)
        if (nb) JG_HIP(hipMemcpyAsync(w->bytes.as<uint8_t>() + b0, bytes, nb, hipMemcpyHostToDevice, ctx->copy));
        JG_HIP(hipMemcpyAsync(w->off.as<uint64_t>() + m0 + 1, off + 1, n * 8, hipMemcpyHostToDevice, ctx->copy));
        JG_HIP(hipMemcpyAsync(w->mset.as<uint32_t>() + m0, set, n * 4, hipMemcpyHostToDevice, ctx->copy));
        jg::upload_done(ctx);
        if (b0) hipLaunchKernelGGL(k_ow_rebase, dim3(blocks_for(n)), dim3(kBlock), 0, ctx->stream, w->off.as<uint64_t>() + m0 + 1, n, b0);
        launch_parse(ctx, w, m0, m0 + n);
        w->wn = m0 + n;
        w->wnb = b0 + nb;
        w->max_set = mx;
        w->any_set = true;
    });
}

int jg_orset_wave_check(jg_orset* s, uint64_t* bad_msg) { return wave_check_call(s, bad_msg, false); }
int jg_orset_wave_commit(jg_orset* s, uint64_t limit) { return wave_commit_call(s, limit, false); }

int jg_orset_wave_abort(jg_orset* s) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        jg::require_writable(s, "jg_orset_wave_abort");
        JG_REQUIRE(s, JG_EINVAL, "jg_orset_wave_abort: store is NULL");
        jg::ensure_device(s->ctx);
        JG_HIP(hipStreamSynchronize(s->ctx->stream));
        JG_HIP(hipStreamSynchronize(s->ctx->copy));  // the caller's chunk buffers are released after this
        if (s->wire) {
            close_wave(s->wire);
            s->wire->g0 = s->wire->g1 = s->wire->n_names;
            s->wire->p0 = s->wire->p1 = s->wire->pool_used;
        }
    });
}

int jg_orset_wave_names(jg_orset* s, uint64_t* n_names, uint64_t* n_bytes, uint32_t* set, uint32_t* id, uint64_t* off, uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s && n_names && n_bytes, JG_EINVAL, "jg_orset_wave_names: NULL argument");
        jg_orset_wire* w = s->wire;
        const uint64_t n = w ? w->g1 - w->g0 : 0, nb = w ? w->p1 - w->p0 : 0;
        *n_names = n;
        *n_bytes = nb;
        if (!set || n == 0) return;
        JG_REQUIRE(id && off && (bytes || nb == 0), JG_EINVAL, "jg_orset_wave_names: NULL buffer");
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        const auto& o = w->nout;
        if (o.g0 != o.g1 && o.g0 == w->g0 && o.g1 == w->g1 && o.p0 == w->p0 && o.p1 == w->p1) {  // queued by the commit
            JG_HIP(hipEventSynchronize(o.ev));
            const uint8_t* h = o.host;
            const auto* hlen = reinterpret_cast<const uint32_t*>(h + n * 8);
            const auto* hpo = reinterpret_cast<const unsigned long long*>(h + ((n * 12 + 15) & ~15ull));
            const uint8_t* hpool = reinterpret_cast<const uint8_t*>(hpo + n);
            std::memcpy(set, h, n * 4);
            std::memcpy(id, h + n * 4, n * 4);
            off[0] = 0;
            for (uint64_t i = 0; i < n; ++i) {
                off[i + 1] = off[i] + hlen[i];
                if (hlen[i]) std::memcpy(bytes + off[i], hpool + (hpo[i] - w->p0), hlen[i]);
            }
            return;
        }
        std::vector<uint32_t> len(n);
        std::vector<unsigned long long> po(n);
        std::vector<uint8_t> pool(nb);
        JG_HIP(hipMemcpyAsync(set, w->nset.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(id, w->nid.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(len.data(), w->nlen.as<uint32_t>() + w->g0, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipMemcpyAsync(po.data(), w->noff.as<unsigned long long>() + w->g0, n * 8, hipMemcpyDeviceToHost, ctx->stream));
        if (nb) JG_HIP(hipMemcpyAsync(pool.data(), w->pool.as<uint8_t>() + w->p0, nb, hipMemcpyDeviceToHost, ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        off[0] = 0;
        for (uint64_t i = 0; i < n; ++i) {
            off[i + 1] = off[i] + len[i];
            if (len[i]) std::copy(pool.begin() + (po[i] - w->p0), pool.begin() + (po[i] - w->p0) + len[i], bytes + off[i]);
        }
    });
}

int jg_orset_names_since(jg_orset* s, uint64_t from, uint64_t* to, uint64_t* n_bytes, uint32_t* set, uint32_t* id, uint64_t* off, uint8_t* bytes) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);
        JG_REQUIRE(s && to && n_bytes, JG_EINVAL, "jg_orset_names_since: NULL argument");
        jg_orset_wire* w = s->wire;
        const uint64_t total = w ? w->n_names : 0;
        JG_REQUIRE(from <= total, JG_EINVAL, "jg_orset_names_since: from %llu past the %llu names held", (unsigned long long)from,
                   (unsigned long long)total);
        *to = total;
        *n_bytes = 0;
        const uint64_t n = total - from;
        if (n == 0) return;
        jg_ctx* ctx = s->ctx;
        jg::ensure_device(ctx);
        auto& o = w->nout;
        if (!(o.since_from == from && o.since_to == total && o.since_pool1 == w->pool_used)) {
            // A commit's new names take their pool bytes by atomics (not in name order), so the bytes of names
            // [from, total) lie in the pool range that starts at the last mark at or before `from` (every name
            // past a mark was made after it) and ends at pool_used.  One queue of copies into page-locked
            // staging, one wait; kept for the second call of a size query + fill.
            uint64_t pool0 = 0;
            for (auto it = w->marks.rbegin(); it != w->marks.rend(); ++it)
                if (it->first <= from) { pool0 = it->second; break; }
            const uint64_t nb = w->pool_used - pool0;
            const size_t need = names_out_bytes(n, nb);
            if (o.ev) JG_HIP(hipEventSynchronize(o.ev));
            o.g0 = o.g1 = 0;  // the staging is reused here: a queued wave-names copy is gone
            if (o.cap < need) {
                if (o.host) JG_HIP(hipHostFree(o.host));
                o.host = nullptr;
                o.cap = 0;
                void* p = nullptr;
                JG_HIP(hipHostMalloc(&p, need + need / 2, hipHostMallocDefault));
                o.host = static_cast<uint8_t*>(p);
                o.cap = need + need / 2;
            }
            uint8_t* h = o.host;
            const size_t po = (n * 12 + 15) & ~15ull;
            JG_HIP(hipMemcpyAsync(h, w->nset.as<uint32_t>() + from, n * 4, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipMemcpyAsync(h + n * 4, w->nid.as<uint32_t>() + from, n * 4, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipMemcpyAsync(h + n * 8, w->nlen.as<uint32_t>() + from, n * 4, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipMemcpyAsync(h + po, w->noff.as<unsigned long long>() + from, n * 8, hipMemcpyDeviceToHost, ctx->stream));
            if (nb) JG_HIP(hipMemcpyAsync(h + po + n * 8, w->pool.as<uint8_t>() + pool0, nb, hipMemcpyDeviceToHost, ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            const auto* hlen = reinterpret_cast<const uint32_t*>(h + n * 8);
            const auto* hpo = reinterpret_cast<const unsigned long long*>(h + po);
            uint64_t sum = 0;
            for (uint64_t i = 0; i < n; ++i) {
                JG_REQUIRE(hpo[i] >= pool0 && hpo[i] + hlen[i] <= w->pool_used, JG_ESTATE,
                           "jg_orset_names_since: name %llu's bytes lie outside the pool range of its log position", (unsigned long long)(from + i));
                sum += hlen[i];
            }
            o.since_from = from, o.since_to = total, o.since_pool0 = pool0, o.since_pool1 = w->pool_used, o.since_bytes = sum;
        }
        *n_bytes = o.since_bytes;
        if (!set) return;
        JG_REQUIRE(id && off && (bytes || o.since_bytes == 0), JG_EINVAL, "jg_orset_names_since: NULL buffer");
        const uint8_t* h = o.host;
        const size_t po = (n * 12 + 15) & ~15ull;
        const auto* hlen = reinterpret_cast<const uint32_t*>(h + n * 8);
        const auto* hpo = reinterpret_cast<const unsigned long long*>(h + po);
        const uint8_t* hpool = reinterpret_cast<const uint8_t*>(hpo + n);
        std::memcpy(set, h, n * 4);
        std::memcpy(id, h + n * 4, n * 4);
        off[0] = 0;
        for (uint64_t i = 0; i < n; ++i) {
            off[i + 1] = off[i] + hlen[i];
            if (hlen[i]) std::memcpy(bytes + off[i], hpool + (hpo[i] - o.since_pool0), hlen[i]);
        }
    });
}

int jg_orset_merge_json(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* off, const uint8_t* bytes, uint64_t* bad_msg) {
    auto lk_ = jg::lock(s);  // the whole begin/append/check/commit sequence under the context lock
    if (bad_msg) *bad_msg = UINT64_MAX;
    if (!s || (n && (!set || !off || !bytes)))
        return jg::guard([&] { jg::fail(JG_EINVAL, "jg_orset_merge_json: NULL argument"); });
    int rc = jg_orset_wave_begin(s, n, n ? off[n] : 0);
    if (rc == JG_OK) rc = jg_orset_wave_append(s, n, set, off, bytes);
    if (rc == JG_OK) rc = jg_orset_wave_check(s, bad_msg);
    if (rc != JG_OK) {
        char keep[1024];
        jg_last_error(keep, sizeof keep);
        jg_orset_wave_abort(s);
        return jg::guard([&] { jg::fail(rc, "%s", keep); });
    }
    return jg_orset_wave_commit(s, n);
}


int jg_orset_encode_json(jg_orset* s, uint64_t n, const uint32_t* set, const uint64_t* add_lim, const uint64_t* rem_lim, uint64_t* off, uint8_t* out,
                         uint64_t cap, uint8_t* sha) {
    return jg::guard([&] {
        auto lk_ = jg::lock(s);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(s && off, JG_EINVAL, "jg_orset_encode_json: NULL argument");
        off[0] = 0;
        if (n == 0) return;
        JG_REQUIRE(set, JG_EINVAL, "jg_orset_encode_json: NULL set list");
        JG_REQUIRE(!add_lim == !rem_lim, JG_EINVAL, "jg_orset_encode_json: add_lim and rem_lim go together");
        JG_REQUIRE(n < (1ull << 29), JG_EINVAL, "jg_orset_encode_json: at most 2^29 states per call");
        jg::ensure_device(s->ctx);
        encode_sets(s, n, set, add_lim, rem_lim, off, out, cap, out ? sha : nullptr);
    });
}

}  // extern "C"
