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
//      into LDS while the payload was in flight (pass A: repeats among known replicas via an LDS
//      column mask per vector, unknown replicas defer the message; pass B: atomicMax; pass C: the
//      group's first lane appends new replicas in token order = Merge's order).
//
// A group never spans two waves, so the phases are separated by wave-level syncs, not block
// barriers: every wave runs its groups at its own pace.
//
// Any payload the chain does not prove (whitespace, nVector first, > kGroupBytes, or malformed) is
// handed whole to the serial parser (scan_one / apply_one) on the group's first lane: the fast path
// accepts a subset of what the serial parser accepts, with identical entries, and never rejects.
#pragma once

constexpr uint32_t kGroupBytes = 512;              // LDS bytes per message: payload + its 16-B alignment offset
constexpr uint32_t kGroupTok = 16;                 // token slots (an entry spans >= 41 bytes, a name 11)
constexpr uint32_t kCompactMin = 27;               // {"pVector":{},"nVector":{}}
enum : uint32_t { kSlow = 1, kMiss = 2, kDup = 4, kFail = 8 };

template <int G>
struct GroupShared {
    static constexpr int kGroups = kBlock / G;
    uint4 buf[kGroups][kGroupBytes / 16];
    Guid16 cols[kGroups][G];                       // the row's first G replica columns
    Guid16 eg[kGroups][kGroupTok];                 // pass C: the entries' Guids by token
    uint16_t tok[kGroups][kGroupTok];
    uint32_t mask[kGroups][16];                    // pass A: columns seen, 256 bits per vector
    uint32_t ntok[kGroups], kn[kGroups], nn[kGroups], flags[kGroups];
};

// LDS written by some lanes of a wave, then read by others: order them (a group never spans waves).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ bool same(const Guid16& a, const Guid16& b) { return a.lo == b.lo && a.hi == b.hi; }

__device__ __forceinline__ bool lds_guid(const uint8_t* s, Guid16& g) {  // s[0..35], read_guid's layout
    uint32_t v = 0;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) { const int h = hexv(s[i]); ok &= h >= 0; v = v << 4 | (uint32_t)(h & 15); }
    unsigned long long lo = v;
    v = 0;
#pragma unroll
    for (int i = 9; i < 13; ++i) { const int h = hexv(s[i]); ok &= h >= 0; v = v << 4 | (uint32_t)(h & 15); }
    lo |= (unsigned long long)v << 32;
    v = 0;
#pragma unroll
    for (int i = 14; i < 18; ++i) { const int h = hexv(s[i]); ok &= h >= 0; v = v << 4 | (uint32_t)(h & 15); }
    lo |= (unsigned long long)v << 48;
    ok &= s[8] == '-' && s[13] == '-' && s[18] == '-' && s[23] == '-';
    unsigned long long hi = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int at = 19 + 2 * b + (b >= 2 ? 1 : 0);
        const int h = hexv(s[at]), l = hexv(s[at + 1]);
        ok &= h >= 0 && l >= 0;
        hi |= (unsigned long long)((h & 15) << 4 | (l & 15)) << (8 * b);
    }
    g.lo = lo;
    g.hi = hi;
    return ok;
}

// read_int's grammar and width limits over s[p, L); *t = the first byte after the number.
template <int EB>
__device__ __forceinline__ bool lds_int(const uint8_t* s, uint32_t p, uint32_t L, long long& out, uint32_t* t) {
    bool neg = false;
    if (p < L && s[p] == '-') { neg = true; ++p; }
    if (p >= L || s[p] < '0' || s[p] > '9') return false;
    unsigned long long mag = 0;
    if (s[p] == '0') {
        ++p;
        if (p < L && s[p] >= '0' && s[p] <= '9') return false;  // leading zero
    } else {
        while (p < L && s[p] >= '0' && s[p] <= '9') {
            const unsigned d = (unsigned)(s[p] - '0');
            if (mag > (~0ull - d) / 10) return false;
            mag = mag * 10 + d;
            ++p;
        }
    }
    const unsigned long long lim = EB == 4 ? (neg ? 0x80000000ull : 0x7FFFFFFFull) : (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull);
    if (mag > lim) return false;
    out = neg ? (long long)(0ull - mag) : (long long)mag;
    *t = p;
    return true;
}

__device__ __forceinline__ bool lds_name_tail(const uint8_t* s) {  // s = the byte after 'p' / 'n': Vector":{
    return s[0] == 'V' && s[1] == 'e' && s[2] == 'c' && s[3] == 't' && s[4] == 'o' && s[5] == 'r' && s[6] == '"' && s[7] == ':' &&
           s[8] == '{';
}

// A group's parse result: token k's entry (if any) on lane k mod G, slot k / G.
template <int EB, int G>
struct GroupParse {
    static constexpr int TPL = (kGroupTok + G - 1) / G;  // token slots per lane
    static_assert(TPL * G >= (int)kGroupTok, "every token slot must have a lane: an unchecked token would pass the chain");
    Guid16 eg[TPL];
    long long ev[TPL];
    bool has[TPL];
    uint32_t kn, nt;
};

// The group's row: its column count and first G columns, loaded before the payload so that both
// latencies overlap; lane g holds column g.
struct RowCache {
    uint32_t row = 0, nc = 0;
    Guid16 cg{0, 0};
    bool has = false;
};

__device__ __forceinline__ RowCache row_cache(const Table& t, const uint32_t* __restrict__ rows, uint64_t m, bool live, uint32_t g) {
    RowCache rc;
    if (live) {
        rc.row = rows[m];
        rc.nc = t.ncols[rc.row];
        if (g < t.R) {
            rc.cg = t.cols[(uint64_t)rc.row * t.R + g];
            rc.has = true;
        }
    }
    return rc;
}

// Column of Guid x in the row (find_col's answer), from the LDS cache and, past G columns, global.
template <int G>
__device__ __forceinline__ uint32_t cached_col(const Guid16* cache, const Guid16* __restrict__ gcols, uint32_t nc, const Guid16& x,
                                               uint32_t hint) {
    const uint32_t ncache = nc < (uint32_t)G ? nc : (uint32_t)G;
    if (hint < ncache && same(cache[hint], x)) return hint;
    for (uint32_t j = 0; j < ncache; ++j)
        if (same(cache[j], x)) return j;
    for (uint32_t j = ncache; j < nc; ++j)
        if (same(gcols[j], x)) return j;
    return UINT32_MAX;
}

// Phases 1-3 for message m on every lane of the group; on return sh.flags[grp] & kSlow is clear iff
// the payload is proven compact, and the row cache is in sh.cols.  STORE_EG: entry Guids to sh.eg.
template <int EB, int G, bool STORE_EG>
__device__ __forceinline__ void group_parse(GroupShared<G>& sh, const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                            uint64_t m, bool live, const RowCache& rc, GroupParse<EB, G>& gp) {
    constexpr uint32_t NW = (kGroupBytes / 16 + G - 1) / G;  // windows per lane
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
    uint4 v[NW];
    if (fit) {
        const uint8_t* src = bytes + (beg & ~15ull);
#pragma unroll
        for (uint32_t u = 0; u < NW; ++u) {
            const uint32_t w = u * G + g;
            v[u] = w * 16 < a + L ? *reinterpret_cast<const uint4*>(src + (uint64_t)w * 16) : make_uint4(0, 0, 0, 0);
        }
    }
    if (rc.has && g < rc.nc) sh.cols[grp][g] = rc.cg;
    uint32_t ntok = 0;
    if (fit) {
        uint32_t carry = 0;
#pragma unroll
        for (uint32_t u = 0; u < NW; ++u) {
            const uint32_t w = u * G + g;
            if (u * G * 16 >= a + L) break;  // group-uniform
            if (w * 16 < a + L) sh.buf[grp][w] = v[u];
            const uint32_t last = v[u].w >> 24;
            uint32_t prev = __shfl_up(last, 1, G);
            if (g == 0) prev = carry;
            carry = __shfl(last, G - 1, G);
            const int base = (int)(16 * w) - (int)a;  // message position of byte 0 of this window
            uint32_t cm = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t word = j < 4 ? v[u].x : j < 8 ? v[u].y : j < 12 ? v[u].z : v[u].w;
                const uint32_t ch = (word >> ((j & 3) * 8)) & 0xFF;
                if (ch == '"' && (prev == '{' || prev == ',') && base + j >= 1 && base + j < (int)L) cm |= 1u << j;
                prev = ch;
            }
            const uint32_t cnt = __popc(cm);
            uint32_t incl = cnt;
#pragma unroll
            for (int d = 1; d < G; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, G);
                if (g >= (uint32_t)d) incl += y;
            }
            uint32_t k = ntok + incl - cnt;
            while (cm) {
                const int j = __ffs(cm) - 1;
                cm &= cm - 1;
                if (k < kGroupTok) sh.tok[grp][k] = (uint16_t)(base + j);
                ++k;
            }
            ntok += __shfl(incl, G - 1, G);
        }
    }
    const bool go = fit && ntok <= kGroupTok && ntok >= 2;  // group-uniform
    if (g == 0) {
        sh.flags[grp] = go ? 0 : kSlow;
        sh.kn[grp] = 0;
        sh.nn[grp] = 0;
    }
    for (uint32_t i = g; i < 16; i += G) sh.mask[grp][i] = 0;
    wave_sync();
    // phase 2: the "nVector" token
    const uint8_t* c = reinterpret_cast<const uint8_t*>(sh.buf[grp]) + a;
    const uint32_t nt = go ? ntok : 0;
    gp.nt = nt;
    for (uint32_t k = g; k < nt; k += G) {
        const uint32_t p = sh.tok[grp][k];
        if (p + 1 < L && c[p + 1] == 'n') {
            sh.kn[grp] = k;
            atomicAdd(&sh.nn[grp], 1u);
        }
    }
    wave_sync();
    // phase 3: each token checked, the chain from token 0 to the closing brace
    const uint32_t kn = sh.kn[grp];
    gp.kn = kn;
    bool bad = go && (sh.nn[grp] != 1 || kn == 0 || c[0] != '{');
#pragma unroll
    for (int u = 0; u < GroupParse<EB, G>::TPL; ++u) {
        gp.has[u] = false;
        const uint32_t k = g + u * G;
        if (!go || bad || k >= nt) continue;
        const uint32_t p = sh.tok[grp][k];
        const uint32_t pn = k + 1 < nt ? sh.tok[grp][k + 1] : UINT32_MAX;
        const int c1 = p + 1 < L ? c[p + 1] : -1;
        uint32_t e = UINT32_MAX, next = UINT32_MAX;  // the '}' closing this token's vector / the next token's start
        if (c1 == 'p' || c1 == 'n') {                // property name
            if (p + 12 > L || !lds_name_tail(c + p + 2) || (c1 == 'p' && (k != 0 || p != 1))) { bad = true; continue; }
            const uint32_t q = p + 11;
            if (c[q] == '}') e = q;
            else next = q;
        } else {  // "<guid>":<int>
            if (k == 0 || p + 41 > L) { bad = true; continue; }
            Guid16 eg;
            long long val;
            uint32_t t;
            if (!lds_guid(c + p + 1, eg) || c[p + 37] != '"' || c[p + 38] != ':' || !lds_int<EB>(c, p + 39, L, val, &t) || t >= L) {
                bad = true;
                continue;
            }
            if (c[t] == ',') next = t + 1;
            else if (c[t] == '}') e = t;
            else { bad = true; continue; }
            gp.has[u] = true;
            gp.eg[u] = eg;
            gp.ev[u] = val;
            if (STORE_EG) sh.eg[grp][k] = eg;
        }
        if (next != UINT32_MAX) bad |= pn != next || k + 1 == kn;               // another entry of this vector
        else if (k < kn) bad |= e + 2 >= L || c[e + 1] != ',' || pn != e + 2 || k + 1 != kn;  // pVector ends, nVector next
        else bad |= e + 2 != L || c[e + 1] != '}' || k + 1 != nt;              // nVector ends the message
    }
    if (bad) atomicOr(&sh.flags[grp], (uint32_t)kSlow);
    wave_sync();
}

// Pass A (validation + replica lookup).  G == 1: the serial parser, one thread per message.
template <int EB, int G>
__global__ __launch_bounds__(kBlock) void k_scan(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                 const uint32_t* __restrict__ rows, uint64_t m0, uint64_t m1, Table t,
                                                 unsigned long long* __restrict__ status /* [0] first bad, [1] n deferred, [3] n slow */,
                                                 unsigned long long* __restrict__ deferred, uint8_t* __restrict__ emit,
                                                 unsigned long long* __restrict__ slow) {
    using T = typename ApplyVis<EB>::T;
    if constexpr (G == 1) {
        const uint64_t m = m0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (m < m1) scan_one<EB>(bytes, off, rows, m, t, status, deferred, emit, slow);
    } else {
        __shared__ GroupShared<G> sh;
        const uint32_t grp = threadIdx.x / G, g = threadIdx.x % G;
        const uint64_t m = m0 + (uint64_t)blockIdx.x * GroupShared<G>::kGroups + grp;
        const bool live = m < m1;
        const RowCache rc = row_cache(t, rows, m, live, g);
        GroupParse<EB, G> gp;
        group_parse<EB, G, false>(sh, bytes, off, m, live, rc, gp);
        const bool fast = live && !(sh.flags[grp] & kSlow);
        if (fast) {
            const Guid16* gcols = t.cols + (uint64_t)rc.row * t.R;
#pragma unroll
            for (int u = 0; u < GroupParse<EB, G>::TPL; ++u) {
                if (!gp.has[u]) continue;
                const uint32_t k = g + u * G;
                const uint32_t vv = k < gp.kn ? 0 : 1;
                const uint32_t col = cached_col<G>(sh.cols[grp], gcols, rc.nc, gp.eg[u], vv ? k - gp.kn - 1 : k - 1);
                if (col == UINT32_MAX) {
                    atomicOr(&sh.flags[grp], (uint32_t)kMiss);
                } else {
                    const uint32_t bit = 1u << (col & 31);
                    if (atomicOr(&sh.mask[grp][vv * 8 + (col >> 5)], bit) & bit) atomicOr(&sh.flags[grp], (uint32_t)kDup);
                    const uint32_t e = vv ? k - 2 : k - 1;  // entry index: tokens minus the names before it
                    uint8_t* h = emit + m * emit_stride(EB);
                    reinterpret_cast<uint16_t*>(h)[1 + e] = (uint16_t)(col | vv << 15);
                    reinterpret_cast<T*>(h + 32)[e] = (T)gp.ev[u];
                }
            }
        }
        wave_sync();
        if (g == 0 && live) {
            if (!fast) {
                scan_one<EB>(bytes, off, rows, m, t, status, deferred, emit, slow);
            } else {
                const uint32_t f = sh.flags[grp];
                *reinterpret_cast<uint16_t*>(emit + m * emit_stride(EB)) = (f & (kDup | kMiss)) ? kReparse : (uint16_t)(gp.nt - 2);
                if (f & kDup) {
                    atomicMin(status, (unsigned long long)m << 2 | kErrSyntax);
                } else if (f & kMiss) {
                    const unsigned long long at = atomicAdd(status + 1, 1ull);
                    deferred[at] = (unsigned long long)rc.row << 32 | m;
                }
            }
        }
    }
}

// Pass B for the entries pass A resolved: kEmitLanes lanes per message, one entry each.
constexpr uint32_t kEmitLanes = 16;
static_assert(kEmitMax <= kEmitLanes && kGroupTok - 2 <= kEmitMax, "an entry slot per lane; every compact entry fits");

template <int EB>
__global__ __launch_bounds__(kBlock) void k_apply_emit(const uint8_t* __restrict__ emit, const uint32_t* __restrict__ rows, uint64_t n,
                                                       uint32_t R, void* P, void* N) {
    using T = typename ApplyVis<EB>::T;
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t m = tid / kEmitLanes;
    const uint32_t e = (uint32_t)(tid % kEmitLanes);
    if (m >= n) return;
    const uint8_t* h = emit + m * emit_stride(EB);
    const uint32_t cnt = *reinterpret_cast<const uint16_t*>(h);
    if (cnt == kReparse || e >= cnt) return;
    const uint32_t code = reinterpret_cast<const uint16_t*>(h)[1 + e];
    const T v = reinterpret_cast<const T*>(h + 32)[e];
    atomicMax(static_cast<T*>(code >> 15 ? N : P) + (uint64_t)rows[m] * R + (code & 0x7FFF), v);
}

// Pass B for the messages pass A left (list entries: [row << 32 |] message): parse again, every Guid now
// resolves, max into the cells.
template <int EB, int G>
__global__ __launch_bounds__(kBlock) void k_apply(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                  const uint32_t* __restrict__ rows, const unsigned long long* __restrict__ list, uint64_t n,
                                                  Table t, void* P, void* N, unsigned long long* __restrict__ status) {
    if constexpr (G == 1) {
        const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (i < n) apply_one<EB>(bytes, off, rows, (uint32_t)list[i], t, P, N, status);
    } else {
        using T = typename ApplyVis<EB>::T;
        __shared__ GroupShared<G> sh;
        const uint32_t grp = threadIdx.x / G, g = threadIdx.x % G;
        const uint64_t i = (uint64_t)blockIdx.x * GroupShared<G>::kGroups + grp;
        const bool live = i < n;
        const uint64_t m = live ? (uint32_t)list[i] : 0;
        const RowCache rc = row_cache(t, rows, m, live, g);
        GroupParse<EB, G> gp;
        group_parse<EB, G, false>(sh, bytes, off, m, live, rc, gp);
        const bool fast = live && !(sh.flags[grp] & kSlow);
        if (fast) {
            const uint64_t base = (uint64_t)rc.row * t.R;
#pragma unroll
            for (int u = 0; u < GroupParse<EB, G>::TPL; ++u) {
                if (!gp.has[u]) continue;
                const uint32_t k = g + u * G;
                const uint32_t vv = k < gp.kn ? 0 : 1;
                const uint32_t col = cached_col<G>(sh.cols[grp], t.cols + base, rc.nc, gp.eg[u], vv ? k - gp.kn - 1 : k - 1);
                if (col == UINT32_MAX) atomicMin(status + 2, (unsigned long long)m << 2 | kErrInternal);
                else atomicMax(static_cast<T*>(vv ? N : P) + base + col, (T)gp.ev[u]);
            }
        } else if (live && g == 0) {
            apply_one<EB>(bytes, off, rows, m, t, P, N, status);
        }
    }
}

// Pass C (new replicas appended in commit order).  One group per sorted deferred entry; the group of a
// row's first entry walks the row's messages in commit order: each compact message is parsed by the
// group, then its first lane appends the unknown Guids in token order (every pVector entry before any
// nVector entry, PNCounters.cs:133-143), keeping the row's first G columns in LDS; other messages go
// through the serial ResolveVis on that lane.  saved[i] = ncols before the walk (for roll-back).
template <int EB, int G>
__global__ __launch_bounds__(kBlock) void k_resolve(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                    const unsigned long long* __restrict__ keys, uint64_t nd, Table t,
                                                    uint32_t* __restrict__ saved, unsigned long long* __restrict__ status) {
    if constexpr (G == 1) {
        const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
        if (i < nd) resolve_one<EB>(bytes, off, keys, nd, i, t, saved, status);
    } else {
        __shared__ GroupShared<G> sh;
        const uint32_t grp = threadIdx.x / G, g = threadIdx.x % G;
        const uint64_t i = (uint64_t)blockIdx.x * GroupShared<G>::kGroups + grp;
        const uint32_t row = i < nd ? (uint32_t)(keys[i] >> 32) : 0;
        if (i >= nd || (i > 0 && (uint32_t)(keys[i - 1] >> 32) == row)) return;  // not a segment head (group-uniform)
        Guid16* gcols = t.cols + (uint64_t)row * t.R;
        uint32_t nc = t.ncols[row];  // every lane tracks the count (lane 0 appends, then broadcasts)
        if (g == 0) saved[i] = nc;
        if (g < nc) sh.cols[grp][g] = gcols[g];
        RowCache none;
        for (uint64_t j = i; j < nd && (uint32_t)(keys[j] >> 32) == row; ++j) {
            const uint64_t m = (uint32_t)keys[j];
            GroupParse<EB, G> gp;
            group_parse<EB, G, true>(sh, bytes, off, m, true, none, gp);
            const bool fast = !(sh.flags[grp] & kSlow);
            if (g == 0) {
                uint32_t err = UINT32_MAX;
                if (fast) {
                    Mask256 seen;
                    for (uint32_t k = 1; k < gp.nt && err == UINT32_MAX; ++k) {
                        if (k == gp.kn) { seen.clear(); continue; }
                        const Guid16 x = sh.eg[grp][k];
                        uint32_t col = cached_col<G>(sh.cols[grp], gcols, nc, x, k < gp.kn ? k - 1 : k - gp.kn - 1);
                        if (col == UINT32_MAX) {
                            if (nc >= t.R) { err = kErrFull; break; }
                            col = nc++;
                            gcols[col] = x;
                            if (col < (uint32_t)G) sh.cols[grp][col] = x;
                        }
                        if (seen.test_set(col)) err = kErrSyntax;  // repeated Guid in one vector
                    }
                } else {
                    t.ncols[row] = nc;
                    err = resolve_msg<EB>(bytes, off, m, gcols, t.ncols + row, t.R);
                    const uint32_t nc2 = t.ncols[row];
                    for (uint32_t col = nc; col < nc2 && col < (uint32_t)G; ++col) sh.cols[grp][col] = gcols[col];
                    nc = nc2;
                }
                if (err != UINT32_MAX) atomicMin(status + 2, (unsigned long long)m << 2 | err);
                sh.flags[grp] = err != UINT32_MAX ? kFail : 0;
                sh.ntok[grp] = nc;
            }
            wave_sync();
            nc = sh.ntok[grp];
            if (sh.flags[grp] & kFail) return;
        }
        if (g == 0) t.ncols[row] = nc;
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
                      const Table& t, uint32_t* saved, unsigned long long* status) {
    const unsigned gr = json_blocks(nd, G);
    switch (G) {
        case 1: hipLaunchKernelGGL((k_resolve<EB, 1>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        case 4: hipLaunchKernelGGL((k_resolve<EB, 4>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        case 16: hipLaunchKernelGGL((k_resolve<EB, 16>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        case 8: hipLaunchKernelGGL((k_resolve<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        case 32: hipLaunchKernelGGL((k_resolve<EB, 32>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        case 64: hipLaunchKernelGGL((k_resolve<EB, 64>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
        default: hipLaunchKernelGGL((k_resolve<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, keys, nd, t, saved, status); break;
    }
}

template <int EB>
void launch_scan_g(int G, hipStream_t st, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, uint64_t m0, uint64_t m1,
                   const Table& t, unsigned long long* status, unsigned long long* deferred, uint8_t* emit, unsigned long long* slow) {
    const unsigned gr = json_blocks(m1 - m0, G);
    switch (G) {
        case 1: hipLaunchKernelGGL((k_scan<EB, 1>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        case 4: hipLaunchKernelGGL((k_scan<EB, 4>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        case 16: hipLaunchKernelGGL((k_scan<EB, 16>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        case 8: hipLaunchKernelGGL((k_scan<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        case 32: hipLaunchKernelGGL((k_scan<EB, 32>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        case 64: hipLaunchKernelGGL((k_scan<EB, 64>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
        default: hipLaunchKernelGGL((k_scan<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, m0, m1, t, status, deferred, emit, slow); break;
    }
}

template <int EB>
void launch_apply_g(int G, hipStream_t st, const uint8_t* bytes, const uint64_t* off, const uint32_t* rows, const unsigned long long* list,
                    uint64_t n, const Table& t, void* P, void* N, unsigned long long* status) {
    const unsigned gr = json_blocks(n, G);
    switch (G) {
        case 1: hipLaunchKernelGGL((k_apply<EB, 1>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        case 4: hipLaunchKernelGGL((k_apply<EB, 4>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        case 16: hipLaunchKernelGGL((k_apply<EB, 16>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        case 8: hipLaunchKernelGGL((k_apply<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        case 32: hipLaunchKernelGGL((k_apply<EB, 32>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        case 64: hipLaunchKernelGGL((k_apply<EB, 64>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
        default: hipLaunchKernelGGL((k_apply<EB, 8>), dim3(gr), dim3(kBlock), 0, st, bytes, off, rows, list, n, t, P, N, status); break;
    }
}
