// json_wave.hpp — passes A and B of json.hip with G lanes per message (included by json.hip only).
//
// One thread per message parses ~357 bytes byte-serially through 23 dependent window loads; a
// 131k-message chunk then fills 2 waves per SIMD and the pass runs at ~200 GB/s of payload.  Here a
// group of G lanes owns one message:
//
//   1  the lanes load the message's aligned 16-byte windows side by side (coalesced) into LDS and
//      mark, from registers, every '"' whose previous byte is '{' or ',' (a token start: a property
//      name or a vector entry); a prefix count over the group numbers the tokens.
//   2  the lane holding a token whose next byte is 'n' records the "nVector" token index.
//   3  token k goes to lane k mod G, which checks its bytes (`"pVector":{`, `"nVector":{`, or
//      `"<36-char Guid>":<int>`), where it ends, and that the next token starts exactly there; the
//      last token must close the message.  The chain proves the whole payload is the compact
//      form System.Text.Json writes — {"pVector":{E,...},"nVector":{E,...}}, E = "<guid D>":<int>,
//      no whitespace — which the serial parser accepts with the same entries.
//   4  each entry is looked up in its row's replica table, whose first G columns the lanes loaded
//      into LDS while the payload was in flight (pass A: a repeat among known replicas, found by an LDS
//      column mask per vector, sends the message to the serial parser; unknown replicas defer it; pass B:
//      atomicMax; pass C: the group's first lane appends new replicas in token order = Merge's order).
//
// A group never spans two waves, so the phases are separated by wave-level syncs, not block
// barriers: every wave runs its groups at its own pace.
//
// Any payload the chain does not prove (whitespace, nVector first, > kGroupBytes, or malformed) goes
// to the `slow` list, which the serial parser (scan_one / apply_one, one lane per message) handles in
// kernels of its own, so the group kernels carry none of its registers: the fast path accepts a subset
// of what the serial parser accepts, with identical entries, and never rejects.
#pragma once

constexpr uint32_t kGroupBytes = 512;              // LDS bytes per message: payload + its 16-B alignment offset
constexpr uint32_t kGroupTok = 16;                 // token slots (an entry spans >= 41 bytes, a name 11)
constexpr uint32_t kCompactMin = 27;               // {"pVector":{},"nVector":{}}
constexpr uint32_t kMaskCols = 64;                 // pass A's repeat check covers columns < 64 (else: serial parser)
enum : uint32_t { kSlow = 1, kMiss = 2, kDup = 4, kFail = 8 };

template <int G>
struct GroupShared {
    static constexpr int kGroups = kBlock / G;
    // one spare window per message: the 8 messages of a wave start 4 LDS banks apart, so that the entry
    // reads of phase 3 (lanes of different messages at similar offsets) do not all hit one bank
    uint4 buf[kGroups][kGroupBytes / 16 + 1];
    Guid16 cols[kGroups][G];                       // the row's first G replica columns
    uint16_t tok[kGroups][kGroupTok];
    uint32_t mask[kGroups][2 * kMaskCols / 32];    // pass A: columns seen per vector (LDS: 7 workgroups per CU, not 6)
    uint32_t tk[kGroups];                          // tokens | the "nVector" token << 8 | "nVector" tokens seen << 16
    uint32_t flags[kGroups];
    // alignment offset | length << 4 | the row's cached column count << 14 | (fused pass A) entries the message
    // raised (its undo records) << 23: one word, so the block's LDS (23,040 B) stays a whole number of 512-B
    // allocation granules below a seventh of the CU's 160 KB
    uint32_t geo[kGroups], row[kGroups];
};
__device__ __forceinline__ uint32_t geo_len(uint32_t geo) { return (geo >> 4) & 0x3FFu; }
__device__ __forceinline__ uint32_t geo_nc(uint32_t geo) { return (geo >> 14) & 0x1FFu; }
constexpr uint32_t kGeoNr = 23;
static_assert(kGroupBytes <= 0x3FFu && kMaxJsonReplicas <= 0x1FFu && kEmitMax <= 0x1FFu, "geo's fields fit");
__device__ __forceinline__ uint32_t tk_ntok(uint32_t tk) { return tk & 0xFFu; }
__device__ __forceinline__ uint32_t tk_kn(uint32_t tk) { return (tk >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t tk_nn(uint32_t tk) { return tk >> 16; }

// Inclusive prefix sum over the G lanes of a group (g = lane in group): row_shr DPP moves for groups inside
// one 16-lane row (no LDS round trip, no address arithmetic), ds_bpermute shuffles past that.
template <int D>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t x) {  // lane - D of the same 16-lane row, 0 past its start
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + D, 0xF, 0xF, true);
}
template <int G>
__device__ __forceinline__ uint32_t group_scan(uint32_t x, uint32_t g) {
    if constexpr (G <= 16) {
        if constexpr (G > 1) { const uint32_t y = dpp_shr<1>(x); x += g >= 1 ? y : 0u; }
        if constexpr (G > 2) { const uint32_t y = dpp_shr<2>(x); x += g >= 2 ? y : 0u; }
        if constexpr (G > 4) { const uint32_t y = dpp_shr<4>(x); x += g >= 4 ? y : 0u; }
        if constexpr (G > 8) { const uint32_t y = dpp_shr<8>(x); x += g >= 8 ? y : 0u; }
    } else {
#pragma unroll
        for (int d = 1; d < G; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, G);
            if (g >= (uint32_t)d) x += y;
        }
    }
    return x;
}
// x of the group's last lane, on every lane of the group (ds_swizzle in bitmask mode within 32 lanes)
template <int G>
__device__ __forceinline__ uint32_t group_last(uint32_t x) {
    if constexpr (G <= 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (int)((0x1Fu & ~(uint32_t)(G - 1)) | (uint32_t)(G - 1) << 5));
    else return __shfl(x, G - 1, G);
}

__device__ __forceinline__ bool same(const Guid16& a, const Guid16& b) { return a.lo == b.lo && a.hi == b.hi; }

// Lanes with `want` get consecutive slots of *counter, one returning atomic per wave (rare paths only:
// a counter every wave waits on serialises the grid).  Every lane of the wave calls it.
__device__ __forceinline__ unsigned long long wave_slot(bool want, unsigned long long* counter) {
    const unsigned long long mask = __ballot(want);
    if (!mask) return 0;
    const int leader = __ffsll((long long)mask) - 1;
    const uint32_t lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if ((int)lane == leader) base = atomicAdd(counter, (unsigned long long)__popcll(mask));
    base = __shfl(base, leader);
    return base + (unsigned long long)__popcll(mask & ((1ull << lane) - 1ull));
}


// `<36-char Guid>":<int>` at LDS byte q (the byte after the opening quote), read_guid's and read_int's
// grammar without whitespace; *tend = offset from q of the byte after the number.
template <int EB>
__device__ __forceinline__ bool entry_at(const uint8_t* base, uint32_t q, Guid16& g, long long& out, uint32_t* tend) {
    constexpr uint32_t kMaxDigits = EB == 4 ? 10 : 19;
    constexpr int kYW = (kMaxDigits + 1 + 3) / 4;  // words holding the longest run and the character after it
    uint32_t X[10 + kYW];                           // characters 0 .. 40 + 4 kYW
    // 8-byte reads: ds_read_b64 moves twice the bytes per LDS cycle of the ds_read2_b32 pairs 4-byte reads compile
    // to, over 64 banks (round 6, tools/json_lds_ab.sh: LDS-active cycles 190M -> 152M per bench leg, bank-conflict
    // cycles 66M -> 49M; the kernel's time did not move — it waits on memory, not on LDS)
    lds_words_b64<10 + kYW>(base, q, X);
    bool ok = jgw::guid_d(X, g.lo, g.hi);
    ok &= (X[9] & 0xFFFFu) == ('"' | ':' << 8);
    // -?(0|[1-9][0-9]*) from character 38; more digits than the width can hold never pass the limit
    const uint32_t neg = ((X[9] >> 16) & 0xFFu) == '-' ? 1u : 0u;
    uint32_t Y[kYW];
#pragma unroll
    for (int k = 0; k < kYW; ++k) Y[k] = __builtin_amdgcn_alignbyte(X[10 + k], X[9 + k], 2 + neg);
    // the run of digits ends at the first non-digit: its flag bit (8j + 7 of word j / 4) by find-first-set per
    // word, 32 k added with saturation so that a word of four digits (no bit: ~0) never wins the min.  (A
    // 20-bit digit mask built with bits4 took ~100 VALU per entry.)
    uint32_t first = UINT32_MAX;
#pragma unroll
    for (int k = 0; k < kYW; ++k) {
        const uint32_t nd = ~digit_bytes(Y[k]) & 0x80808080u;
        const uint32_t b = nd ? (uint32_t)__builtin_ctz(nd) : UINT32_MAX;
        first = min(first, __builtin_elementwise_add_sat(b, 32u * (uint32_t)k));
    }
    const uint32_t run = first == UINT32_MAX ? 4u * kYW : (first - 7) >> 3;  // > kMaxDigits either way when all are digits
    ok &= run >= 1 && run <= kMaxDigits && !((Y[0] & 0xFFu) == '0' && run > 1);
    // digits while any lane of the wave still has one (magnitudes of a few digits are the common
    // case); the first 7 in 24-bit multiply-adds (full rate: < 10^7), the rest in 64 bits
    unsigned long long mag = 0;
    uint32_t m24 = 0;
#pragma unroll
    for (uint32_t j = 0; j < kMaxDigits; ++j) {
        if (!__builtin_amdgcn_ballot_w64(j < run)) break;  // wave-uniform
        const uint32_t d = (Y[j >> 2] >> (8 * (j & 3))) & 0xFu;
        if (j < 7) m24 = j < run ? __umul24(m24, 10u) + d : m24;
        else {
            if (j == 7) mag = m24;
            mag = j < run ? mag * 10 + d : mag;
        }
    }
    if (run < 8) mag = m24;
    const unsigned long long lim = EB == 4 ? (neg ? 0x80000000ull : 0x7FFFFFFFull) : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
    ok &= mag <= lim;
    out = neg ? (long long)(0ull - mag) : (long long)mag;
    *tend = 38 + neg + run;
    return ok;
}

// `Vector":{` at LDS byte q (the byte after 'p' / 'n'): three realigned words instead of nine byte reads.
__device__ __forceinline__ bool lds_name_tail(const uint8_t* base, uint32_t q) {
    uint32_t X[3];
    lds_words<3>(base, q, X);
    return X[0] == ('V' | 'e' << 8 | 'c' << 16 | (uint32_t)'t' << 24) && X[1] == ('o' | 'r' << 8 | '"' << 16 | (uint32_t)':' << 24) &&
           (X[2] & 0xFFu) == '{';
}

// A wave's parse result.  The entry tokens (every token but the two names) of the wave's 64 / G groups,
// in group order, are dealt over its 64 lanes: round u of a lane holds wave entry lane + 64u, tg = its
// group << 16 | its token index there.  The two names are checked by lanes 0 and 1 of their group.  (All
// tokens dealt, C5's ~7 tokens per message overflowed the 64 lanes of 8 messages in ~10 % of the waves,
// and those paid a second round of the entry parse for a handful of tokens.)
template <int EB, int G>
struct GroupParse {
    static constexpr int kRounds = ((64 / G) * ((int)kGroupTok - 2) + 63) / 64;
    static_assert(64 % G == 0 && G >= 2 && kRounds * 64 >= (64 / G) * ((int)kGroupTok - 2),
                  "every entry of the wave must have a lane: an unchecked token would pass the chain");
    Guid16 eg[kRounds];
    long long ev[kRounds];
    uint32_t tg[kRounds];
    bool has[kRounds];
};

// The group's row: its first G columns, loaded before the payload so that both latencies overlap; lane g
// holds column g.  The row's column COUNT is not read: a column slot at or past the count is all-zero (the
// table starts zeroed, columns are appended in order, and every roll-back of a count zeroes the slots it
// drops, k_rollback), so the columns are the row's leading non-zero slots.  That saves each message a
// random line for 4 bytes (the count array is as large as the row count; round 5 PMC: the count, the
// columns and the P / N lines were ~290 of the ~560 bytes per message pass A moved).  A hit is therefore
// always a real column; a replica whose Guid is all-zero (or any column after it) reads as a miss, which
// the deferred path resolves against the true count (slower, same result).
struct RowCache {
    uint32_t row = 0, nc = 0;  // nc: the row's leading non-zero slots among the first G, or t.R when all G are
    Guid16 cg{0, 0};           // (then the lookup walks on in global memory up to the first zero slot)
    bool has = false;
};

template <int G>
__device__ __forceinline__ RowCache row_cache(const Table& t, const uint32_t* __restrict__ rows, uint64_t m, bool live, uint32_t g) {
    RowCache rc;
    if (live) {
        rc.row = rows[m];
        if (g < t.R) {
            rc.cg = t.cols[(uint64_t)rc.row * t.R + g];
            rc.has = true;
        }
    }
    const unsigned long long b = __ballot(rc.has && (rc.cg.lo | rc.cg.hi) != 0);  // every lane of the wave
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long gm = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
    const unsigned long long bits = (b >> (lane - g)) & gm;
    const uint32_t lead = bits == gm ? (uint32_t)G : (uint32_t)__ffsll((long long)~bits) - 1;
    rc.nc = lead == (uint32_t)G && t.R > (uint32_t)G ? t.R : lead;
    return rc;
}

// Column of Guid x in the row (find_col's answer), from the LDS cache and, past G columns, global (up to
// the first zero slot, the end of the row's columns).
template <int G>
__device__ __forceinline__ uint32_t cached_col(const Guid16* cache, const Guid16* __restrict__ gcols, uint32_t nc, const Guid16& x,
                                               uint32_t hint) {
    const uint32_t ncache = nc < (uint32_t)G ? nc : (uint32_t)G;
    if (hint < ncache && same(cache[hint], x)) return hint;
    for (uint32_t j = 0; j < ncache; ++j)
        if (same(cache[j], x)) return j;
    for (uint32_t j = ncache; j < nc; ++j) {
        const Guid16 h = gcols[j];
        if ((h.lo | h.hi) == 0) break;
        if (same(h, x)) return j;
    }
    return UINT32_MAX;
}

// Phases 1-3 for message m on every lane of the group; on return sh.flags[grp] & kSlow is clear iff
// the payload is proven compact, and the row cache is in sh.cols / sh.row / sh.geo.
template <int EB, int G>
__device__ __forceinline__ void group_parse(GroupShared<G>& sh, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                            uint64_t m, bool live, const RowCache& rc, GroupParse<EB, G>& gp) {
    // 32-byte windows (two aligned 16-byte loads per lane per round): at 8 lanes two rounds cover a message
    // (16-byte windows took four, the fourth for the quarter of C5's messages past 384 bytes, and every round
    // pays the group scan, the range mask and the token loop's set-up)
    constexpr uint32_t NW = (kGroupBytes / 32 + G - 1) / G;  // windows per lane
    const uint32_t grp = threadIdx.x / G, g = threadIdx.x % G;
    uint64_t beg = 0, len = 0;
    if (live) {
        beg = off[m];
        len = off[m + 1] - beg;
    }
    const uint32_t a = (uint32_t)(beg & 15);
    const bool fit = live && len >= kCompactMin && len + a <= kGroupBytes;
    const uint32_t L = fit ? (uint32_t)len : 0;
    // phase 1: every window load issued first, then stored to LDS and scanned for token starts
    uint4 v[NW][2];
    if (fit) {
        const uint8_t* src = bytes + (beg & ~15ull);
#pragma unroll
        for (uint32_t u = 0; u < NW; ++u) {
            const uint32_t w = u * G + g;
            v[u][0] = 32 * w < a + L ? *reinterpret_cast<const uint4*>(src + (uint64_t)w * 32) : make_uint4(0, 0, 0, 0);
            v[u][1] = 32 * w + 16 < a + L ? *reinterpret_cast<const uint4*>(src + (uint64_t)w * 32 + 16) : make_uint4(0, 0, 0, 0);
        }
    }
    if (rc.has && g < rc.nc) sh.cols[grp][g] = rc.cg;
    // token starts = the even-numbered quotes: in the compact form every string (the two property names,
    // each entry's Guid) is one pair of quotes with no escapes inside, so quote 2k opens token k.  A stray or
    // escaped quote shifts the pairing, and the token chain of phase 3 then fails: slow list (the serial
    // parser decides).  (The round-2 scan tested each quote's previous byte for '{' or ',' instead: two more
    // SWAR tests per word and a carried byte between lanes, ~40 VALU per window.)
    uint32_t nq = 0;  // quotes before this window, over the group
    if (fit) {
#pragma unroll
        for (uint32_t u = 0; u < NW; ++u) {
            const uint32_t w = u * G + g;
            if (u * G * 32 >= a + L) break;  // group-uniform
            if (32 * w < a + L) sh.buf[grp][2 * w] = v[u][0];
            if (32 * w + 16 < a + L) sh.buf[grp][2 * w + 1] = v[u][1];
            uint32_t qm = jgw::quote_mask16(v[u][0]) | jgw::quote_mask16(v[u][1]) << 16;
            const int base = (int)(32 * w) - (int)a;                     // message position of byte 0 of this window
            const int lo = base >= 1 ? 0 : 1 - base, hi = min((int)L - base, 32);  // bytes j with 1 <= base + j < L
            const uint32_t width = (uint32_t)(hi - lo);
            qm &= hi > lo ? (width >= 32 ? ~0u : (1u << width) - 1u) << lo : 0u;
            const uint32_t cnt = __popc(qm);
            const uint32_t incl = group_scan<G>(cnt, g);
            uint32_t q = nq + incl - cnt;  // index of this lane's first quote in the window
            if (q & 1) qm &= qm - 1, ++q;  // an odd quote closes a string: start from the next one
            while (qm) {  // every other quote from here opens a token
                const int j = __ffs(qm) - 1;
                if ((q >> 1) < kGroupTok) sh.tok[grp][q >> 1] = (uint16_t)(base + j);
                qm &= qm - 1;
                qm &= qm - 1;  // skip the closing quote
                q += 2;
            }
            nq += group_last<G>(incl);
        }
    }
    const uint32_t ntok = (nq & 1) ? kGroupTok + 1 : nq >> 1;  // an unpaired quote: not the compact form
    const bool go = fit && ntok <= kGroupTok && ntok >= 2;  // group-uniform
    const uint32_t nt = go ? ntok : 0;
    if (g == 0) {
        sh.flags[grp] = go ? 0 : kSlow;
        sh.tk[grp] = nt;
        sh.geo[grp] = a | L << 4 | rc.nc << 14;
        sh.row[grp] = rc.row;
    }
    for (uint32_t i = g; i < 2 * kMaskCols / 32; i += G) sh.mask[grp][i] = 0;
    wave_sync();
    // phase 2: the "nVector" token (index and count in one word: with one such token its index is exact)
    const uint8_t* buf = reinterpret_cast<const uint8_t*>(sh.buf[grp]);
    const uint8_t* c = buf + a;
    for (uint32_t k = g; k < nt; k += G) {
        const uint32_t p = sh.tok[grp][k];
        if (p + 1 < L && c[p + 1] == 'n') atomicAdd(&sh.tk[grp], 1u << 16 | k << 8);
    }
    wave_sync();
    // phase 3: the chain from token 0 to the closing brace.  The two names on lanes 0 and 1 of the group
    // ("pVector" opens the message at byte 1; "nVector" follows the pVector's '}'), each with what follows
    // its '{' (the vector's first entry, or '}' and then the next name / the message's end) ...
    if (nt && g < 2) {
        const uint32_t tk = sh.tk[grp], kn = tk_kn(tk);
        const uint32_t k = g ? min(kn, nt - 1) : 0;
        const uint32_t p = sh.tok[grp][k];
        bool bad = tk_nn(tk) != 1 || kn == 0 || p + 12 > L || c[p + 1] != (g ? 'n' : 'p') || (g == 0 && (p != 1 || c[0] != '{')) ||
                   !lds_name_tail(buf, a + p + 2);
        if (!bad) {
            const uint32_t q = p + 11;  // the byte after the name's '{'
            const uint32_t pn = k + 1 < nt ? sh.tok[grp][k + 1] : UINT32_MAX;
            if (c[q] == '}') bad = g ? (q + 2 != L || c[q + 1] != '}' || k + 1 != nt)    // empty nVector ends the message
                                     : (q + 2 >= L || c[q + 1] != ',' || pn != q + 2 || k + 1 != kn);  // empty pVector, then nVector
            else bad = pn != q || k + 1 == kn;  // the vector's first entry starts right after '{'
        }
        if (bad) atomicOr(&sh.flags[grp], (uint32_t)kSlow);
    }
    // ... and every entry, dealt over the wave
    constexpr uint32_t GW = 64 / G;  // groups per wave
    const uint32_t lane = threadIdx.x & 63, wg0 = (threadIdx.x >> 6) * GW;
    uint32_t base[GW + 1];
    base[0] = 0;
#pragma unroll
    for (uint32_t j = 0; j < GW; ++j) {
        const uint32_t t = tk_ntok(sh.tk[wg0 + j]);
        base[j + 1] = base[j] + (t >= 2 ? t - 2 : 0u);
    }
#pragma unroll
    for (int u = 0; u < GroupParse<EB, G>::kRounds; ++u) {
        gp.has[u] = false;
        gp.tg[u] = 0;
        const uint32_t tw = lane + 64u * (uint32_t)u;
        if (tw >= base[GW]) continue;
        uint32_t j = 0, bj = 0;
#pragma unroll
        for (uint32_t i = 1; i < GW; ++i)
            if (tw >= base[i]) { j = i; bj = base[i]; }
        const uint32_t gq = wg0 + j, e = tw - bj;
        const uint32_t geo = sh.geo[gq], aq = geo & 15u, Lq = geo_len(geo), tkq = sh.tk[gq], ntq = tk_ntok(tkq), kn = tk_kn(tkq);
        const uint32_t k = e + 1 + (e + 1 >= kn ? 1u : 0u);  // entry e's token: tokens 0 and kn are the names
        const uint8_t* cq = reinterpret_cast<const uint8_t*>(sh.buf[gq]) + aq;
        bool bad = false;
        do {  // "<guid>":<int>
            const uint32_t p = sh.tok[gq][k];
            const uint32_t pn = k + 1 < ntq ? sh.tok[gq][k + 1] : UINT32_MAX;
            if (p + 41 > Lq) { bad = true; break; }
            uint32_t tr;
            const bool ok = entry_at<EB>(reinterpret_cast<const uint8_t*>(sh.buf[gq]), aq + p + 1, gp.eg[u], gp.ev[u], &tr);
            const uint32_t t = p + 1 + tr;
            if (!ok || t >= Lq) { bad = true; break; }
            gp.has[u] = true;
            gp.tg[u] = gq << 16 | k;
            if (cq[t] == ',') bad = pn != t + 1 || k + 1 == kn;                                   // another entry of this vector
            else if (cq[t] != '}') bad = true;
            else if (k < kn) bad = t + 2 >= Lq || cq[t + 1] != ',' || pn != t + 2 || k + 1 != kn;  // pVector ends, nVector next
            else bad = t + 2 != Lq || cq[t + 1] != '}' || k + 1 != ntq;                        // nVector ends the message
        } while (false);
        if (bad) atomicOr(&sh.flags[gq], (uint32_t)kSlow);
    }
    wave_sync();
}

// Pass A (validation + replica lookup).  G == 1: the serial parser, one thread per message.
template <int EB, int G>
__global__ __launch_bounds__(kBlock) void k_scan(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ rows, uint64_t m0, uint64_t m1, Table t,
                                                 unsigned long long* __restrict__ status /* [0] first bad, [1] n deferred, [3] n slow */,
                                                 unsigned long long* __restrict__ deferred, uint8_t* __restrict__ emit,
                                                 Guid16* __restrict__ eguid, unsigned long long* __restrict__ slow, void* P, void* N,
                                                 bool fuse) {
    using T = typename ApplyVis<EB>::T;
    if constexpr (G == 1) {  // every accepted message not deferred also goes to the slow list
        const uint64_t m = m0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (m < m1) scan_one<EB>(bytes, off, rows, m, t, status, deferred, emit, slow);
    } else {
        __shared__ GroupShared<G> sh;
        const uint32_t grp = threadIdx.x / G, g = threadIdx.x % G;
        // workgroups take the messages from the wave's end: the fused apply then meets a key's newest state first
        // (states grow along a wave), and its older ones settle with a plain read instead of raising the cell
        // again (C1: ~3000 states per hot key per wave — in commit order each raised the cell, an atomic and an
        // undo record apiece)
        const uint64_t bx = gridDim.x - 1 - blockIdx.x;
        const uint64_t m = m0 + bx * GroupShared<G>::kGroups + grp;
        // a node wave (csrc/node.hip) holds every kind's messages: those of other kinds carry kSkipIdx
        const bool skip = m < m1 && rows[m] == jg::kSkipIdx;
        const bool live = m < m1 && !skip;
        const RowCache rc = row_cache<G>(t, rows, m, live, g);
        GroupParse<EB, G> gp;
        group_parse<EB, G>(sh, bytes, off, m, live, rc, gp);
        // each parsed entry (on the lane its token was dealt to): its column and the repeat check
        uint32_t colr[GroupParse<EB, G>::kRounds];
#pragma unroll
        for (int u = 0; u < GroupParse<EB, G>::kRounds; ++u) {
            colr[u] = UINT32_MAX;
            const uint32_t gq = gp.tg[u] >> 16, k = gp.tg[u] & 0xFFFFu;
            if (!gp.has[u] || (sh.flags[gq] & kSlow)) continue;
            const uint32_t kn = tk_kn(sh.tk[gq]), rq = sh.row[gq];
            const uint32_t vv = k < kn ? 0 : 1;
            const uint32_t col = cached_col<G>(sh.cols[gq], t.cols + (uint64_t)rq * t.R, geo_nc(sh.geo[gq]), gp.eg[u], vv ? k - kn - 1 : k - 1);
            colr[u] = col;
            if (col == UINT32_MAX) {
                atomicOr(&sh.flags[gq], (uint32_t)kMiss);
            } else if (col >= kMaskCols) {
                atomicOr(&sh.flags[gq], (uint32_t)kSlow);  // past the repeat mask: the serial parser decides
            } else {
                const uint32_t bit = 1u << (col & 31);
                if (atomicOr(&sh.mask[gq][vv * (kMaskCols / 32) + (col >> 5)], bit) & bit) atomicOr(&sh.flags[gq], (uint32_t)kDup);
            }
        }
        wave_sync();
        // the message's flags are final: its entries into the record pass B reads (a message with an unknown replica:
        // every entry by Guid, pass C resolves the columns) or — fused (the steady state: every replica known) — into
        // the cells right here, each entry that raised its cell recorded as (column, old value) so a wave that fails
        // later is undone exactly (k_undo_applied: the min of a cell's recorded old values is its value before the
        // wave; max has no inverse, the record is the inverse).  Pass B then has nothing to do for it.
#pragma unroll
        for (int u = 0; u < GroupParse<EB, G>::kRounds; ++u) {
            const uint32_t gq = gp.tg[u] >> 16, k = gp.tg[u] & 0xFFFFu;
            const uint32_t fq = sh.flags[gq];
            if (!gp.has[u] || (fq & (kSlow | kDup))) continue;
            const uint64_t mq = m0 + bx * GroupShared<G>::kGroups + gq;
            const uint32_t vv = k < tk_kn(sh.tk[gq]) ? 0 : 1;
            const uint32_t e = vv ? k - 2 : k - 1;  // entry index: tokens minus the names before it
            uint8_t* h = emit + mq * emit_stride(EB);
            const T v = (T)gp.ev[u];
            if (fq & kMiss) {
                eguid[mq * kEmitMax + e] = gp.eg[u];
                reinterpret_cast<uint16_t*>(h)[1 + e] = (uint16_t)(0x7FFF | vv << 15);
                reinterpret_cast<T*>(h + 32)[e] = v;
            } else if (fuse) {
                T* cell = static_cast<T*>(vv ? N : P) + (uint64_t)sh.row[gq] * t.R + colr[u];
                if (*cell < v) {  // most states repeat what the cell holds: a plain read settles them
                    const T old = atomicMax(cell, v);
                    if (old < v) {
                        const uint32_t r = atomicAdd(&sh.geo[gq], 1u << kGeoNr) >> kGeoNr;
                        reinterpret_cast<uint16_t*>(h)[1 + r] = (uint16_t)(colr[u] | vv << 15);
                        reinterpret_cast<T*>(h + 32)[r] = old;
                    }
                }
            } else {
                reinterpret_cast<uint16_t*>(h)[1 + e] = (uint16_t)(colr[u] | vv << 15);
                reinterpret_cast<T*>(h + 32)[e] = v;
            }
        }
        wave_sync();
        const uint32_t f = sh.flags[grp];
        // a Guid repeated among the known replicas of one vector (kDup): System.Text.Json keeps its LAST value at its
        // first place, which the serial parser visits (oracle/json.hpp) — the message goes to the slow list unapplied
        const bool fast = live && !(f & (kSlow | kDup));
        const bool deferred_msg = fast && (f & kMiss);
        const bool defer = g == 0 && deferred_msg;
        if (g == 0 && fast) deferred[m] = defer ? (unsigned long long)rc.row << 32 | m : kNotDeferred;
        if (defer) status[1] = 1;  // any deferral (select_deferred later overwrites it with the count)
        const bool to_slow = g == 0 && live && !fast;
        const unsigned long long at = wave_slot(to_slow, status + 3);
        if (to_slow) {
            slow[at] = m;  // k_scan_slow parses it (and marks / emits it) before the wave's status is read
            // its record header now, not only when k_scan_slow runs: an undo before then (a node wave cut or aborted
            // right after its chunks' pass A) must not read a header an earlier wave left here as an applied record
            *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) = kReparse;
        }
        if (g == 0 && skip) {  // no entries, not deferred
            *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) = 0;
            deferred[m] = kNotDeferred;
        }
        if (g == 0 && fast) {
            *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) =
                (fuse && !(f & kMiss)) ? (uint16_t)(kApplied | sh.geo[grp] >> kGeoNr)
                                       : (uint16_t)((tk_ntok(sh.tk[grp]) - 2) | ((f & kMiss) ? kNeedsCols : 0u));
        }
    }
}

// Pass A for the payloads the group parse did not prove compact: the serial parser, one lane per
// message of the slow list (count in status[3], read on the device).
template <int EB>
__global__ __launch_bounds__(kBlock) void k_scan_slow(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                      const uint32_t* __restrict__ rows, Table t, unsigned long long* __restrict__ status,
                                                      unsigned long long* __restrict__ deferred, uint8_t* __restrict__ emit,
                                                      const unsigned long long* __restrict__ slow) {
    const unsigned long long n = status[3];
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        scan_one<EB>(bytes, off, rows, slow[i], t, status, deferred, emit, nullptr);
}

// Pass B for the entries pass A resolved: kEmitLanes lanes per message, one entry each.
constexpr uint32_t kEmitLanes = 16;
static_assert(kEmitMax <= kEmitLanes && kGroupTok - 2 <= kEmitMax, "an entry slot per lane; every compact entry fits");

template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_emit(const uint8_t* __restrict__ emit, const uint32_t* __restrict__ rows, uint64_t n,
                                                       uint32_t R, void* P, void* N, const unsigned long long* __restrict__ guard) {
    using T = typename ApplyVis<EB>::T;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t e = (uint32_t)(tid % kEmitLanes);
    if (tid / kEmitLanes >= n || (guard && (guard[0] != ~0ull || guard[1] != 0))) return;  // guard: pass A failed or deferred
    // newest message first: a key's states grow along the wave (counters only increase), so its largest
    // value usually lands first and the older states' reads below settle without an atomic (max is
    // order-free; C1's 100 hot keys, ~3000 states each per wave: 292 us of serialised atomics in
    // commit order)
    const uint64_t m = n - 1 - tid / kEmitLanes;
    const uint8_t* h = emit + m * emit_stride(EB);
    const uint32_t cnt = *reinterpret_cast<const uint16_t*>(h);
    if (cnt == kReparse || (cnt & (kNeedsCols | kApplied)) || e >= cnt) return;  // kApplied: pass A applied it (fused)
    const uint32_t code = reinterpret_cast<const uint16_t*>(h)[1 + e];
    if ((code & 0x7FFF) == kVoidCol) return;  // an earlier entry of a key the vector repeats (pass C)
    const T v = reinterpret_cast<const T*>(h + 32)[e];
    T* cell = static_cast<T*>(code >> 15 ? N : P) + (uint64_t)rows[m] * R + (code & 0x7FFF);
    // a wave repeats hot keys (C1: 100 keys, ~3000 states each): most values do not raise the cell, and
    // a plain read settles those without an atomic on a hot address
    if (*cell < v) atomicMax(cell, v);
}

// The fused pass A undone (a wave that failed after it, or a node wave cut or aborted): every entry it recorded as
// having raised its cell takes the cell back down with atomicMin(old) — a cell's smallest recorded old value is
// what it held before the wave, whichever order the raises took.  Idempotent.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_undo_applied(const uint8_t* __restrict__ emit, const uint32_t* __restrict__ rows, uint64_t n,
                                                         uint32_t R, void* P, void* N) {
    using T = typename ApplyVis<EB>::T;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint32_t e = (uint32_t)(tid % kEmitLanes);
    const uint64_t m = tid / kEmitLanes;
    if (m >= n) return;
    const uint8_t* h = emit + m * emit_stride(EB);
    const uint32_t cnt = *reinterpret_cast<const uint16_t*>(h);
    if (cnt == kReparse || !(cnt & kApplied) || e >= (cnt & 0xFFu)) return;
    const uint32_t code = reinterpret_cast<const uint16_t*>(h)[1 + e];
    T* cell = static_cast<T*>(code >> 15 ? N : P) + (uint64_t)rows[m] * R + (code & 0x7FFF);
    atomicMin(cell, reinterpret_cast<const T*>(h + 32)[e]);
}

// Pass B for the messages left to the serial parser (list entries: [row << 32 |] message): parse again,
// every Guid now resolves, max into the cells.  With the group parse (G > 1) that is the slow list:
// compact deferred messages are applied from their resolved records by k_apply_emit.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_list(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ list,
                                                       uint64_t n, Table t, void* P, void* N, unsigned long long* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) apply_one<EB>(bytes, off, rows, (uint32_t)list[i], t, P, N, status);
}

// k_apply_list over the slow list with its count read on the device (status[3]), guarded like
// k_apply_emit: a no-op unless pass A accepted every message and deferred none.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_slow(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ list,
                                                       Table t, void* P, void* N, unsigned long long* __restrict__ status) {
    if (status[0] != ~0ull || status[1] != 0) return;
    const unsigned long long n = status[3];
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        apply_one<EB>(bytes, off, rows, (uint32_t)list[i], t, P, N, status);
}

// Pass C (new replicas appended in commit order) from pass A's records: no payload is parsed again.
// One lane per sorted deferred entry; the lane of a row's first entry walks the row's deferred messages
// in commit order, finds or appends each entry's Guid in token order (every pVector entry before any
// nVector entry, PNCounters.cs:133-143) against the row's columns, voids the earlier entries of a key its
// vector repeats (the last value counts), and writes the columns into the record for pass B.  At a message the group parse did not prove compact
// (record kReparse) the rest of the walk goes to k_resolve_resume (serial ResolveVis).  G == 1
// (JANUS_JSON_GROUP=1): the serial walk throughout (k_resolve_serial).  saved[i] = ncols before the walk
// (for roll-back).  The walk is serial per row either way; round 3 gave each row a 16-lane group whose
// first lane walked it (the others staged Guids into LDS): 16x the waves for the same serial work, 0.42 ms
// of a C5 wave whose rows mostly meet a new replica, all of it after the wave's last upload.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_resolve_serial(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                           const unsigned long long* __restrict__ keys, uint64_t nd, Table t,
                                                           uint32_t* __restrict__ saved, unsigned long long* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < nd) resolve_one<EB>(bytes, off, keys, nd, i, t, saved, status);
}

template <int EB>
__global__ __launch_bounds__(kBlock) void k_resolve_rows(const unsigned long long* __restrict__ keys, uint64_t nd, Table t,
                                                         uint8_t* __restrict__ emit, const Guid16* __restrict__ eguid,
                                                         uint32_t* __restrict__ saved, unsigned long long* __restrict__ status,
                                                         unsigned long long* __restrict__ resume) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nd) return;
    const uint32_t row = (uint32_t)(keys[i] >> 32);
    if (i > 0 && (uint32_t)(keys[i - 1] >> 32) == row) return;  // not a segment head
    Guid16* gcols = t.cols + (uint64_t)row * t.R;
    // the row's first kRC columns in registers, loaded together with its count (one round trip: the slots past
    // the count are zero, row_cache), and each message's first kRC Guids loaded before its walk — the walk was a
    // chain of dependent loads per entry (the Guid, then the columns one by one), 0.30 ms of a C5 wave's tail
    constexpr uint32_t kRC = 8;
    Guid16 rcol[kRC];
#pragma unroll
    for (uint32_t c = 0; c < kRC; ++c) rcol[c] = c < t.R ? gcols[c] : Guid16{0, 0};
    uint32_t nc = t.ncols[row];
    saved[i] = nc;
    for (uint64_t j = i; j < nd && (uint32_t)(keys[j] >> 32) == row; ++j) {
        const uint64_t m = (uint32_t)keys[j];
        uint8_t* h = emit + m * emit_stride(EB);
        const uint32_t hdr = *reinterpret_cast<const uint16_t*>(h);
        if (hdr == kReparse) {  // not compact: the serial walk takes over from message j
            t.ncols[row] = nc;
            resume[atomicAdd(status + 4, 1ull)] = j;
            return;
        }
        const uint32_t cnt = hdr & ~kNeedsCols;
        uint16_t* codes = reinterpret_cast<uint16_t*>(h) + 1;
        Guid16 xg[kRC];
#pragma unroll
        for (uint32_t e = 0; e < kRC; ++e) xg[e] = e < cnt ? eguid[m * kEmitMax + e] : Guid16{0, 0};
        Mask256 seen[2];  // columns met per vector
        uint32_t err = UINT32_MAX;
        for (uint32_t e = 0; e < cnt; ++e) {
            const uint32_t vv = codes[e] >> 15;
            Guid16 x = eguid[0];
            if (e < kRC) {
#pragma unroll
                for (uint32_t q = 0; q < kRC; ++q)
                    if (q == e) x = xg[q];
            } else {
                x = eguid[m * kEmitMax + e];
            }
            // the row's Guids are distinct: any match is the one find_col returns
            uint32_t col = UINT32_MAX;
#pragma unroll
            for (uint32_t c = 0; c < kRC; ++c)
                if (c < nc && same(rcol[c], x)) col = c;
            for (uint32_t c = kRC; col == UINT32_MAX && c < nc; ++c)
                if (same(gcols[c], x)) col = c;
            if (col == UINT32_MAX) {
                if (nc >= t.R) { err = kErrFull; break; }
                col = nc++;
                gcols[col] = x;
#pragma unroll
                for (uint32_t c = 0; c < kRC; ++c)
                    if (c == col) rcol[c] = x;
            }
            // a Guid repeated in one vector: System.Text.Json's Dictionary keeps its LAST value at its FIRST place
            // (oracle/json.hpp) — the column stays where the first occurrence put it, the earlier entries are voided
            if (vv ? seen[1].test_set(col) : seen[0].test_set(col))
                for (uint32_t q = 0; q < e; ++q)
                    if (codes[q] == (uint16_t)(col | vv << 15)) codes[q] = (uint16_t)(kVoidCol | vv << 15);
            codes[e] = (uint16_t)(col | vv << 15);
        }
        *reinterpret_cast<uint16_t*>(h) = (uint16_t)cnt;  // resolved: pass B applies the record
        if (err != UINT32_MAX) {
            atomicMin(status + 2, (unsigned long long)m << 2 | err);
            return;
        }
    }
    t.ncols[row] = nc;
}

// The rest of a row's walk from a message k_resolve_rows handed over (serial ResolveVis, one lane).  A
// compact message further on in the walk still has its record to resolve: its columns are looked up
// once its Guids are in the row, so pass B applies it from the record.
template <int EB>
__global__ __launch_bounds__(kBlock) void k_resolve_resume(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                           const unsigned long long* __restrict__ keys, uint64_t nd, Table t,
                                                           unsigned long long* __restrict__ status,
                                                           const unsigned long long* __restrict__ resume, uint8_t* __restrict__ emit,
                                                           const Guid16* __restrict__ eguid) {
    const unsigned long long nr = status[4];
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < nr; r += (uint64_t)gridDim.x * kBlock) {
        const uint64_t j0 = resume[r];
        const uint32_t row = (uint32_t)(keys[j0] >> 32);
        Guid16* gcols = t.cols + (uint64_t)row * t.R;
        for (uint64_t j = j0; j < nd && (uint32_t)(keys[j] >> 32) == row; ++j) {
            const uint64_t m = (uint32_t)keys[j];
            const uint32_t err = resolve_msg<EB>(bytes, off, m, gcols, t.ncols + row, t.R);
            if (err != UINT32_MAX) {
                atomicMin(status + 2, (unsigned long long)m << 2 | err);
                break;
            }
            uint16_t* h = reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB));
            if (h[0] != kReparse && (h[0] & kNeedsCols)) {
                const uint32_t cnt = h[0] & ~kNeedsCols;
                for (uint32_t e = 0; e < cnt; ++e) {
                    const uint32_t col = find_col(gcols, t.ncols[row], eguid[m * kEmitMax + e], UINT32_MAX);
                    const uint16_t code = (uint16_t)((col & 0x7FFF) | (h[1 + e] & 0x8000));
                    for (uint32_t q = 0; q < e; ++q)  // a repeated key: its last value only (as k_resolve_rows)
                        if (h[1 + q] == code) h[1 + q] = (uint16_t)(kVoidCol | (code & 0x8000));
                    h[1 + e] = code;
                }
                h[0] = (uint16_t)cnt;
            }
        }
    }
}

// Lanes per message: JANUS_JSON_GROUP = 1 (serial), 4, 8 (default), 16, 32 or 64; read on every launch.
inline int json_group() {
    const char* e = std::getenv("JANUS_JSON_GROUP");
    const int v = e ? std::atoi(e) : 8;
    return v == 1 || v == 4 || v == 16 || v == 32 || v == 64 ? v : 8;
}
inline unsigned json_blocks(uint64_t n, int G) { return (unsigned)((n * (uint64_t)G + kBlock - 1) / kBlock); }

template <int EB>
void launch_resolve_g(int G, hipStream_t st, const uint8_t* bytes, const uint64_t* off, const unsigned long long* keys, uint64_t nd,
                      const Table& t, uint8_t* emit, const Guid16* eguid, uint32_t* saved, unsigned long long* status,
                      unsigned long long* resume) {
    if (G == 1) {
        hipLaunchKernelGGL(k_resolve_serial<EB>, dim3(json_blocks(nd, 1)), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status);
    } else {
        hipLaunchKernelGGL(k_resolve_rows<EB>, dim3(json_blocks(nd, 1)), dim3(kBlock), 0, st, keys, nd, t, emit, eguid, saved, status, resume);
    }
}

template <int EB>
void launch_scan_g(int G, hipStream_t st, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t m0, uint64_t m1,
                   const Table& t, unsigned long long* status, unsigned long long* deferred, uint8_t* emit, Guid16* eguid,
                   unsigned long long* slow, void* P, void* N, bool fuse) {
    const unsigned gr = json_blocks(m1 - m0, G);
#define JG_SCAN(GG) hipLaunchKernelGGL((k_scan<EB, GG>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, eguid, slow, P, N, fuse)
    switch (G) {
        case 1: JG_SCAN(1); break;
        case 4: JG_SCAN(4); break;
        case 16: JG_SCAN(16); break;
        case 32: JG_SCAN(32); break;
        case 64: JG_SCAN(64); break;
        default: JG_SCAN(8); break;
    }
#undef JG_SCAN
}

