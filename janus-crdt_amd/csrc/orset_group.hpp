// orset_group.hpp — pass 1 of orset_wire.hip with one WAVE per ORSetMsg (included by orset_wire.hip only).
//
// k_ow_parse gives each ~1.2 KB state to one thread, which walks it byte by byte through dependent window
// loads: a wave's 64 lanes then touch 64 payloads ~1.2 KB apart on every load, and the pass runs at ~75 GB/s
// of payload.  Here the 64 lanes of a wave own one message (ORSetMsg.Decode, MergeSharp/MergeSharp/CRDTs/
// ORSet.cs:56-69, over the form System.Text.Json writes):
//
//   1  the lanes load the message's aligned 16-byte windows side by side (coalesced) into LDS; SWAR tests
//      over the registers find every '"' and every byte the fast path does not take (a backslash, a
//      control character, a non-ASCII byte), and a wave prefix count numbers the quotes: with no
//      backslash, quote 2k opens string token k and quote 2k+1 closes it.
//   2  token k goes to lane k mod 64.  The bytes between two tokens (the "glue") must be one of ten short
//      strings of the compact form — {  :{  :[  ,  ],  ]},  :{},  :[],  and the closers ]}  :[]} — and the
//      glue before a token decides its role: a member name, an element name or a tag.  Wave prefix counts
//      over the tokens (ballots) give each token its section (a `]},` or `:{},` glue opens the next member
//      after a map), its null sub-section, its entry ordinal and its tag ordinal.  Each lane checks its
//      token against the compact grammar {"addSet":{E,...},"removeSet":{E,...},"nullAddGuid":[T,...],
//      "nullRemoveGuid":[T,...]}, E = "<name>":[T,...] (non-empty), T = "<36-char Guid D>", and writes its
//      entry (name hash, offset, length, side, position) or tag (reference, value) where the serial parse
//      would: the same slots of the same sparse regions, in the same order.
//
// Anything the chain does not prove (whitespace, members out of order or repeated, an unknown member, escapes,
// non-ASCII names, an empty tag set, an element named twice in one map, more than kOgBytes or kOgTok, or a
// malformed payload) marks the message slow; k_ow_parse then
// parses it serially (its flag array), so the fast path accepts a subset of what the serial parser accepts,
// with identical outputs, and never reports an error itself.  Writes are bounded by the message's own
// sparse regions, so a message that turns out slow overwrites nothing of another's.
#pragma once

constexpr uint32_t kOgBytes = 4096;            // LDS bytes per message: payload + its 16-B alignment offset
constexpr uint32_t kOgWin = kOgBytes / 16;     // windows per message
constexpr uint32_t kOgRounds = kOgBytes / 32 / 64;  // rounds of 32-byte windows (two 16-byte loads per lane)
constexpr uint32_t kOgTok = 192;               // string tokens per message (a compact 4 KB state has < 190)
constexpr uint32_t kOgTokRounds = kOgTok / 64;
constexpr int kOgWaves = kBlock / 64;          // messages per workgroup

struct OgShared {
    uint4 buf[kOgWaves][kOgWin + 1];           // +1 window: realigned reads near the end stay inside
    uint16_t q[kOgWaves][2 * kOgTok];          // quote positions (message-relative)
    unsigned long long nh[kOgWaves][kOgTok];   // element names: 64-bit FNV-1a with the map's side in bit 0
};

// glue codes: the bytes packed little-endian (no pattern holds a zero byte, so the length is implicit)
enum : uint32_t {
    kGlOpen = 0x7Bu,           // {      before "addSet"
    kGlMap = 0x7B3Au,          // :{     member -> first element name
    kGlArr = 0x5B3Au,          // :[     name -> first tag
    kGlNext = 0x2Cu,           // ,      tag -> tag
    kGlElem = 0x2C5Du,         // ],     last tag -> next element name (map) / "nullRemoveGuid" (null arrays)
    kGlEndMap = 0x2C7D5Du,     // ]},    last tag of a map -> next member
    kGlEmptyMap = 0x2C7D7B3Au, // :{},   member with an empty map -> next member
    kGlEmptyArr = 0x2C5D5B3Au, // :[],   "nullAddGuid" with no tags -> "nullRemoveGuid"
    kGlEndTag = 0x7D5Du,       // ]}     the last tag closes the message
    kGlEndEmpty = 0x7D5D5B3Au, // :[]}   "nullRemoveGuid" with no tags closes the message
};

__device__ __forceinline__ uint32_t og_glue(const uint8_t* lds, uint32_t a, int32_t p, int32_t q) {  // bytes [p, q) of the message
    const int32_t n = q - p;
    if (n <= 0 || n > 4) return 0;
    uint32_t X[1];
    jgw::lds_words<1>(lds, a + (uint32_t)p, X);
    return n == 4 ? X[0] : X[0] & ((1u << (8 * n)) - 1u);
}

__device__ __forceinline__ bool og_name_is(const uint8_t* c, uint32_t p, uint32_t n, const char* lit, uint32_t ln) {
    if (n != ln) return false;
    bool ok = true;
    for (uint32_t i = 0; i < ln; ++i) ok &= c[p + i] == (uint8_t)lit[i];
    return ok;
}

// The 36-character "D" form at LDS byte q (GuidSink's value, C# byte order); false unless every digit is hex
// and the four dashes sit at 8, 13, 18, 23.
__device__ __forceinline__ bool og_guid(const uint8_t* lds, uint32_t q, Tag16& t) {
    uint32_t X[9];
    jgw::lds_words<9>(lds, q, X);
    return jgw::guid_d(X, t.lo, t.hi);
}

__device__ __forceinline__ uint32_t og_prefix_le(unsigned long long ballot, uint32_t lane) {  // set bits at lanes <= lane
    return (uint32_t)__popcll(ballot & (lane == 63 ? ~0ull : (2ull << lane) - 1ull));
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void k_ow_group(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                                                     const uint32_t* __restrict__ mset, uint64_t m0, uint64_t m1, Sparse S, uint64_t kmask, uint64_t salt,
                                                     unsigned long long* __restrict__ ne, unsigned long long* __restrict__ nt,
                                                     uint32_t* __restrict__ na, unsigned long long* __restrict__ err, uint8_t* __restrict__ slow) {
    __shared__ OgShared sh;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t m = m0 + (uint64_t)blockIdx.x * kOgWaves + wv;
    if (m >= m1) return;  // wave-uniform: one message per wave, no workgroup barrier below
    const uint32_t set = mset[m];
    if (set == jg::kSkipIdx) {  // another kind's message in a node wave (csrc/node.hip)
        if (lane == 0) {
            ne[m] = nt[m] = 0;
            na[m] = 0;
            err[m] = kNone;
            slow[m] = 0;
        }
        return;
    }
    const uint64_t b = off[m], len = off[m + 1] - b;
    const uint32_t a = (uint32_t)(b & 15);
    if (len + a > kOgBytes || len < 2) {
        if (lane == 0) slow[m] = 1;
        return;
    }
    const uint32_t L = (uint32_t)len, span = a + L;
    uint8_t* lds = reinterpret_cast<uint8_t*>(sh.buf[wv]);
    uint16_t* qp = sh.q[wv];

    // phase 1: windows into LDS; quotes numbered; bytes the fast path does not take.  32-byte windows: the
    // ORSetWorkload state (~1.2 KB) is one round of the wave (16-byte windows took two, each paying the wave
    // scan, the range masks and the token loop's set-up)
    uint4 v[kOgRounds][2];
    const uint8_t* src = bytes + (b & ~15ull);
#pragma unroll
    for (uint32_t u = 0; u < kOgRounds; ++u) {
        const uint32_t w = u * 64 + lane;
        v[u][0] = 32 * w < span ? *reinterpret_cast<const uint4*>(src + (uint64_t)w * 32) : make_uint4(0, 0, 0, 0);
        v[u][1] = 32 * w + 16 < span ? *reinterpret_cast<const uint4*>(src + (uint64_t)w * 32 + 16) : make_uint4(0, 0, 0, 0);
    }
    uint32_t nq = 0;
    bool rej = false;
#pragma unroll
    for (uint32_t u = 0; u < kOgRounds; ++u) {
        if (u * 64 * 32 >= span) break;  // wave-uniform
        const uint32_t w = u * 64 + lane;
        sh.buf[wv][2 * w] = v[u][0];
        sh.buf[wv][2 * w + 1] = v[u][1];
        uint32_t qm = 0, bm = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t x[4] = {v[u][h].x, v[u][h].y, v[u][h].z, v[u][h].w};
            uint32_t badb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)  // backslash, control or non-ASCII
                badb[i] = (x[i] | jgw::le_bytes(x[i] & 0x7F7F7F7Fu, 0x1F) | jgw::zero_bytes(x[i] ^ 0x5C5C5C5Cu)) & 0x80808080u;
            qm |= jgw::quote_mask16(v[u][h]) << (16 * h);
            bm |= jgw::flags16(badb[0], badb[1], badb[2], badb[3]) << (16 * h);
        }
        // bytes of this window inside the message: span positions [a, a + L)
        const int lo = max((int)a - (int)(32 * w), 0), hi = min((int)span - (int)(32 * w), 32);
        const uint32_t width = (uint32_t)(hi - lo);
        const uint32_t in = hi > lo ? (width >= 32 ? ~0u : (1u << width) - 1u) << lo : 0u;
        qm &= in;
        rej |= __ballot((bm & in) != 0) != 0;
        const uint32_t cnt = __popc(qm);
        const uint32_t incl = jgw::wave_incl_scan(cnt);  // every lane of the wave is here (wave-uniform loop)
        uint32_t k = nq + incl - cnt;
        while (qm) {
            const int j = __ffs(qm) - 1;
            qm &= qm - 1;
            if (k < 2 * kOgTok) qp[k] = (uint16_t)(32 * w + j - a);
            ++k;
        }
        nq += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    const uint32_t ntok = nq >> 1;
    if (rej || (nq & 1) || ntok == 0 || ntok > kOgTok) {  // wave-uniform
        if (lane == 0) slow[m] = 1;
        return;
    }
    jgw::wave_sync();

    // phase 2: tokens dealt over the lanes; roles from the glue, ordinals from ballots
    const uint64_t es = (b + kEntryDiv - 1) / kEntryDiv, ts = (b + kTagDiv - 1) / kTagDiv;
    const uint64_t ecap = (off[m + 1] + kEntryDiv - 1) / kEntryDiv - es, tcap = (off[m + 1] + kTagDiv - 1) / kTagDiv - ts;
    const uint8_t* c = lds + a;
    uint32_t c_sec = 0, c_nsub = 0, c_ent = 0, c_add = 0, c_tag = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t r = 0; r < kOgTokRounds; ++r) {
        if (r * 64 >= ntok) break;  // wave-uniform
        const uint32_t k = r * 64 + lane;
        const bool has = k < ntok;
        int32_t s = 0, e = 0;
        uint32_t gb = 0, ga = 0;
        if (has) {
            s = qp[2 * k];
            e = qp[2 * k + 1];
            const int32_t pe = k ? (int32_t)qp[2 * k - 1] + 1 : 0;
            const int32_t ns = k + 1 < ntok ? (int32_t)qp[2 * k + 2] : (int32_t)L;
            gb = og_glue(lds, a, pe, s);
            ga = og_glue(lds, a, e + 1, ns);
        }
        const bool brk = has && (gb == kGlEndMap || gb == kGlEmptyMap);
        const uint32_t sec = c_sec + og_prefix_le(__ballot(brk), lane);
        const bool nbrk = has && sec == 2 && (gb == kGlElem || gb == kGlEmptyArr);
        const uint32_t nsub = c_nsub + og_prefix_le(__ballot(nbrk), lane);
        const bool isname = has && sec < 2 && (gb == kGlMap || gb == kGlElem);
        const unsigned long long bname = __ballot(isname), badd = __ballot(isname && sec == 0);
        const uint32_t ent = c_ent + og_prefix_le(bname, lane);  // names so far, this one included
        const bool isval = has && (gb == kGlArr || gb == kGlNext);
        const unsigned long long bval = __ballot(isval);
        const uint32_t tag = c_tag + og_prefix_le(bval, lane) - (isval ? 1u : 0u);
        if (has) {
            const uint32_t n = (uint32_t)(e - s - 1);
            const bool last = k + 1 == ntok;
            bool ok;
            if (last && ga != kGlEndTag && ga != kGlEndEmpty) {
                ok = false;
            } else if (k == 0) {
                ok = gb == kGlOpen && s == 1 && og_name_is(c, 2, n, "addSet", 6) && (ga == kGlMap || ga == kGlEmptyMap);
            } else if (sec > 2 || gb == kGlOpen) {
                ok = false;
            } else if (brk) {  // the member after a map
                ok = sec == 1 ? og_name_is(c, s + 1, n, "removeSet", 9) && (ga == kGlMap || ga == kGlEmptyMap)
                              : og_name_is(c, s + 1, n, "nullAddGuid", 11) && (ga == kGlArr || ga == kGlEmptyArr);
            } else if (isname) {  // an element: a non-empty tag array follows
                ok = ga == kGlArr;
                const uint32_t q = ent - 1;
                if (ok && q < ecap) {
                    unsigned long long h = kFnvBasis;
                    for (uint32_t i = 0; i < n; ++i) h = (h ^ c[s + 1 + i]) * kFnvPrime;
                    uint32_t X[2];
                    jgw::lds_words<2>(lds, a + (uint32_t)s + 1, X);
                    const unsigned long long pf = ((unsigned long long)X[1] << 32 | X[0]) & (n >= 8 ? ~0ull : (1ull << (8 * n)) - 1ull);
                    S.key[es + q] = name_key(set, h, salt) & kmask;
                    S.noff[es + q] = b + (uint64_t)s + 1;
                    S.pfx[es + q] = pf;
                    S.meta[es + q] = n | sec << 31;
                    S.pos[es + q] = (uint32_t)s;
                    S.set[es + q] = set;
                    sh.nh[wv][q] = (h & ~1ull) | sec;  // q < ntok <= kOgTok
                }
            } else if (nbrk) {  // "nullRemoveGuid"
                ok = nsub == 1 && og_name_is(c, s + 1, n, "nullRemoveGuid", 14) && (ga == kGlArr || (last && ga == kGlEndEmpty));
            } else if (isval) {
                Tag16 g;
                ok = n == 36 && og_guid(lds, a + (uint32_t)s + 1, g);
                if (sec < 2) ok &= ga == kGlNext || ga == kGlElem || ga == kGlEndMap;
                else if (nsub == 0) ok &= ga == kGlNext || ga == kGlElem;
                else ok &= ga == kGlNext || (last && ga == kGlEndTag);
                if (ok && tag < tcap) {
                    const bool null = sec == 2;
                    const uint32_t side = null ? nsub : sec, cur = ent ? ent - 1 : 0;
                    S.tref[ts + tag] = (unsigned long long)null << 63 | (unsigned long long)side << 62 | cur;
                    S.tval[ts + tag] = g;
                }
            } else {
                ok = false;
            }
            bad |= !ok;
        }
        c_sec += (uint32_t)__popcll(__ballot(brk));
        c_nsub += (uint32_t)__popcll(__ballot(nbrk));
        c_ent += (uint32_t)__popcll(bname);
        c_add += (uint32_t)__popcll(badd);
        c_tag += (uint32_t)__popcll(bval);
    }
    // an element named twice in one map: System.Text.Json keeps its LAST tag set at its FIRST place (oracle/json.hpp),
    // which the serial parse reproduces, so the message leaves the fast path here (names compared by their 64-bit
    // hashes in LDS; two different names sharing one only cost the slow path)
    if (__ballot(bad) == 0 && c_ent > 1) {  // wave-uniform
        jgw::wave_sync();
        bool dup = false;
        for (uint32_t q = lane; q < c_ent; q += 64) {
            const unsigned long long x = sh.nh[wv][q];
            for (uint32_t p = 0; p < q; ++p) dup |= sh.nh[wv][p] == x;
        }
        bad |= dup;
    }
    const bool fast = __ballot(bad) == 0;
    if (lane == 0) {
        slow[m] = fast ? 0 : 1;
        if (fast) {
            ne[m] = c_ent;
            nt[m] = c_tag;
            na[m] = c_add;  // removeSet never precedes addSet here
            err[m] = kNone;
        }
    }
}

// JANUS_ORSET_PARSE=group (tests): no serial fall-back — a message the group parse did not prove compact is
// rejected at its first byte, so a test of compact payloads shows that every one of them took the fast path.
__global__ void k_ow_reject_slow(const uint8_t* __restrict__ slow, uint64_t m0, uint64_t m1, unsigned long long* __restrict__ ne,
                                 unsigned long long* __restrict__ nt, uint32_t* __restrict__ na, unsigned long long* __restrict__ err) {
    const uint64_t m = m0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (m >= m1 || !slow[m]) return;
    ne[m] = nt[m] = 0;
    na[m] = 0;
    err[m] = kKindInval;
}
