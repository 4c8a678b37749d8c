// orset_tables.hpp — the OR-Set wave's string and record tables, filled chunk by chunk (included by
// orset_wire.hip only).
//
// A wave's commit needs, for every element string of every set, the first entry that names it (its id is
// issued in first-insertion order, ORSet.cs:255-279 / the Dictionaries' order), and, for every distinct tag
// record, its first occurrence (the arrival ordinal: HashSet<Guid>.UnionWith keeps a tag where it first
// entered).  Sorting the wave's entries and de-duplicating its records after the last chunk made the
// commit a ~2.3 ms tail behind the uploads on the ORSetWorkload wave (200k states, 4.6M entries, 4.6M tag
// references, ~0.4M distinct records).  Here three small kernels run after each chunk's parse, while the
// next chunk is still being gathered and uploaded:
//
//   k_ow_strings   one wave per message, one lane per entry: the (set, string) goes into an open-addressing
//                  table (exact byte compare on a hash match; slot = the string's id for this wave), the
//                  slot keeps the smallest canonical entry index (atomicMin; entry slots are ordered like
//                  commit order).  Both parsers hand over each (map, element) of a message once — System.Text.Json
//                  keeps a repeated key's last value at its first place, which the serial parse reproduces and the
//                  group parse leaves to it (round 6; the tables used to reject the repeat in LDS).
//   k_ow_rkeys     each tag reference's record identity without its tag: (string slot, side), or
//                  (set, side) for a null tag set.
//   k_ow_rins      each tag reference into the record table (exact compare of identity + tag), the slot
//                  keeping the smallest tag index = the record's arrival ordinal.
//                  Both: kMsgsPerWave messages per wave, their references dealt over the lanes.
//
// The commit then resolves only the distinct strings against the element table and sorts only the
// distinct records.  A table that runs out of probes (more distinct strings / records than it was sized
// for, or tests narrowing the hashes) raises the overflow word, and the wave falls back to the sort-based check and commit (k_ow_compact ... k_ow_dedup), which
// reads the same sparse regions.  Messages past the commit limit are in the tables too; the commit keeps
// the strings and records whose first occurrence lies before the limit (entry / tag slots are ordered
// like messages).
#pragma once

constexpr uint32_t kNoSid = 0xFFFFFFFFu;
constexpr uint32_t kUnresolved = 0xFFFFFFFEu;  // sid_id of a string not looked up at claim time (ids stay below it)
constexpr uint32_t kProbeCap = 256;  // probes before a table insert gives up (the wave falls back)
constexpr int kTabWaves = kBlock / 64;

// The slots a table's inserts claimed, appended as they are claimed, so the commit walks these instead of the
// whole table: kLists sub-lists of sub_cap entries (list j = the appending wave's message index % kLists, count n[j]) —
// one counter took every wave's append and serialised the insert kernels (360 us per 32k-state chunk).
constexpr uint32_t kLists = 16;
constexpr uint32_t kCountStride = 32;  // counters 256 B apart: atomics on one L2 line serialise
// One slot per table entry: a probe's word and the field every probe that hits then updates share one line
// (round 3 kept them in separate arrays: two scattered lines per entry / tag reference).
// The string slot (32 B) also carries the string's fingerprint — set, length, first 8 bytes — so a probe that
// hits a string claimed by an EARLIER chunk's launch compares against its own slot instead of the first
// inserter's entry arrays (round 4: four scattered lines per hit, 2.37 GB of traffic for a 245 MB ORSetWorkload
// wave).  The claimant writes the fingerprint with plain stores; the kernel boundary between
// chunks makes it visible everywhere.  A string claimed in the SAME launch (first inserter's entry slot at or
// past the chunk's first entry) is compared through the entry arrays as before: publishing the fingerprint
// within a launch needs an agent-scope release / acquire, which on this chip writes back / invalidates the
// XCD's whole L2 — measured 12.7x slower (k_ow_strings 538 -> 6855 us per wave, profiles/r05/orset_fp).
// Strings of <= 8 bytes (the ORSetWorkload's) are decided by the slot alone; longer ones read the tail bytes
// through the first inserter.
// Cleared per wave to {0, ~0, kLenUnset | 0, 0, 0} (k_str_clear); record slots to {0, ~0, 0} (k_tab_clear).
constexpr uint32_t kLenUnset = 0xFFFFFFFFu;
struct alignas(32) StrSlot {
    unsigned long long word;  // (key >> 32) << 32 | (entry slot + 1) of the string's first inserter; 0 = empty
    uint32_t first;           // smallest canonical entry index naming the string
    uint32_t len;             // the string's length (kLenUnset until claimed)
    unsigned long long pfx;   // the string's first 8 bytes (zero past its end)
    uint32_t set;             // the message's set
    uint32_t id0;             // the id k_ow_strings looked up at claim time (kNoName new, kUnresolved not looked up)
};
struct alignas(16) RecSlot {
    unsigned long long word;  // (hash >> 32) << 32 | (tag slot + 1) of the record's first inserter; 0 = empty
    uint32_t mint;            // smallest tag slot holding the record (arrival ordinal)
    uint32_t key;             // side << 31 | set, written by the claimant (the commit's bucket, without the string chain)
};
static_assert(sizeof(StrSlot) == 32 && sizeof(RecSlot) == 16, "a 32-byte string slot, a 16-byte record slot");

struct StrTab {
    StrSlot* slot;
    uint64_t mask;
    uint32_t* list;
    unsigned long long* n;
    uint64_t sub_cap;
};
struct RecTab {
    RecSlot* slot;
    uint64_t mask;
    uint32_t* list;
    unsigned long long* n;
    uint64_t sub_cap;
};

__global__ void k_tab_clear(uint4* __restrict__ slots, uint64_t n) {  // {word 0, ~0, 0}: empty, no first / mint yet
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        slots[i] = make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
}
__global__ void k_str_clear(uint4* __restrict__ slots, uint64_t n) {  // n 32-byte slots: empty, no first, fingerprint unset
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n; i += (uint64_t)gridDim.x * blockDim.x)
        slots[i] = (i & 1) ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(0u, 0u, 0xFFFFFFFFu, kLenUnset);
}

// Lanes that claimed a slot append it to their workgroup's sub-list: one atomic per wave (claims are a few
// per message).  A full sub-list raises the overflow word (the wave takes the sort path).
// spread: the sub-list is spread % kLists — the caller's message index (and round), so a wave's claims land in
// all sub-lists however few workgroups a chunk has (by workgroup, a 30-message chunk of 4-message waves filled
// two of the sixteen).
__device__ __forceinline__ void list_append(bool fresh, uint32_t slot, uint32_t* list, unsigned long long* n, uint64_t sub_cap,
                                            unsigned long long* overflow, uint64_t spread) {
    const unsigned long long b = __ballot(fresh);
    if (!b) return;
    const uint32_t lane = threadIdx.x & 63, j = (uint32_t)(spread % kLists);
    const int leader = __ffsll((long long)b) - 1;
    unsigned long long base = 0;
    if ((int)lane == leader) base = atomicAdd(n + j * kCountStride, (unsigned long long)__popcll(b));
    base = __shfl(base, leader);
    const unsigned long long at = base + __popcll(b & ((1ull << lane) - 1ull));
    if (!fresh) return;
    if (at < sub_cap) list[j * sub_cap + at] = slot;
    else *overflow = 1;
}

// The sub-lists packed back to back (offs[j] = where sub-list j starts; offs[kLists] = the total), grid-stride
// (the check queues it before the total is known on the host).
__global__ void k_list_pack(const uint32_t* __restrict__ list, uint64_t sub_cap, const unsigned long long* __restrict__ offs,
                            uint32_t* __restrict__ out) {
    const uint64_t total = offs[kLists];
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < total; i += (uint64_t)gridDim.x * kBlock) {
        uint32_t j = 0;
        while (offs[j + 1] <= i) ++j;
        out[i] = list[j * sub_cap + (i - offs[j])];
    }
}

// Both tables' sub-list offsets from their counters on the device (each count clamped to its sub-list: an
// overflowed table's counts run past it, and that wave never commits from the tables).
__global__ void k_list_offs(const unsigned long long* __restrict__ ns, uint64_t s_cap, const unsigned long long* __restrict__ nr, uint64_t r_cap,
                            unsigned long long* __restrict__ offs, unsigned long long* __restrict__ scatter_bad) {
    if (threadIdx.x == 2) *scatter_bad = 0;  // k_cb_scatter_claimed's bound flag, queued after this launch
    if (threadIdx.x >= 2) return;
    const unsigned long long* n = threadIdx.x ? nr : ns;
    const uint64_t cap = threadIdx.x ? r_cap : s_cap;
    unsigned long long* o = offs + threadIdx.x * (kLists + 1);
    unsigned long long run = 0;
    for (uint32_t j = 0; j < kLists; ++j) {
        o[j] = run;
        run += min((unsigned long long)cap, n[j * kCountStride]);
    }
    o[kLists] = run;
}

// A place in the bucket of `cell` (the key's counter) for every active lane, from one atomic per RUN of
// consecutive active lanes with the same key, all of the wave's in flight together (one round trip).  The lists
// hold each message's claims back to back (one wave per message appends them together) and a message is one
// set, so a wave's 64 items are a few runs: ~8x fewer atomics than one per lane, and a hot set costs one per
// wave.  Device-scope atomics execute at the memory side (MI355X_MICROARCH "Global float atomics"); the round-3
// fold took every distinct key of a wave in turn, a chain of up to 64 dependent ballot + atomic rounds.
__device__ __forceinline__ uint32_t bucket_add(bool active, uint32_t key, uint32_t* cell) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long act = __ballot(active);
    if (!act) return kDead;  // wave-uniform
    const uint32_t prev = (uint32_t)__shfl_up((int)key, 1);
    const bool head = active && (lane == 0 || !((act >> (lane - 1)) & 1) || prev != key);
    const unsigned long long heads = __ballot(head);
    const unsigned long long breaks = heads | ~act;  // a run ends before the next head or inactive lane
    const unsigned long long above = lane == 63 ? 0ull : breaks & (~0ull << (lane + 1));
    const uint32_t end = above ? (uint32_t)(__ffsll((long long)above) - 1) : 64u;
    uint32_t r = 0;
    if (head) r = atomicAdd(cell, end - lane);
    const unsigned long long hm = heads & (lane == 63 ? ~0ull : (2ull << lane) - 1ull);
    const uint32_t h = hm ? 63u - (uint32_t)__clzll(hm) : lane;  // this lane's run head (an inactive lane: itself)
    const uint32_t base = (uint32_t)__shfl((int)r, (int)h);
    return active ? base + (lane - h) : kDead;
}

// The bytes of each run of bucket_add (same runs: consecutive active lanes with one key) added to the key's
// byte counter by the run's head, no return: an inclusive wave scan of the lengths, the head adds the scan at
// the run's last lane minus the scan before it.  Lengths that could overflow the 32-bit scan (>= 2^25 each):
// one add per lane.  Every lane of the wave calls it.
__device__ __forceinline__ void run_bytes(bool active, uint32_t key, unsigned long long* cell, uint32_t len) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long act = __ballot(active);
    if (!act) return;  // wave-uniform
    const uint32_t v = active ? len : 0u;
    if (__ballot(v >= (1u << 25))) {  // wave-uniform
        if (active) atomicAdd(cell, (unsigned long long)len);
        return;
    }
    const uint32_t incl = jgw::wave_incl_scan(v);
    const uint32_t prev = (uint32_t)__shfl_up((int)key, 1);
    const bool head = active && (lane == 0 || !((act >> (lane - 1)) & 1) || prev != key);
    const unsigned long long breaks = __ballot(head) | ~act;
    const unsigned long long above = lane == 63 ? 0ull : breaks & (~0ull << (lane + 1));
    const uint32_t end = above ? (uint32_t)(__ffsll((long long)above) - 1) : 64u;
    const uint32_t at_end = (uint32_t)__shfl((int)incl, (int)(end - 1));
    if (head) atomicAdd(cell, (unsigned long long)(at_end - (incl - v)));
}

// The commit's per-set bucket counts taken at claim time (orset_commit.hpp): a claimant of a NEW string (not in
// the element table) takes its place in its set's bucket and adds its bytes; a claimant of a record takes its
// place in its (side, set) bucket.  place[slot] = {place or kDead, set | side << 31}.  A claim the counts cannot
// hold (a set at or past cap, a string not looked up) raises *uncounted and the commit counts from the lists
// (k_cb_count); so does a commit with a limit (claims past it are counted here).
inline constexpr uint64_t cb_al(uint64_t b) { return (b + 255) & ~255ull; }
// the four count arrays of cap + 1 entries: new strings, records (two sides) per set, then the strings' bytes
inline constexpr uint64_t cb_counts_bytes(uint64_t cap) { return 3 * cb_al((cap + 1) * 4) + cb_al((cap + 1) * 8); }
// places and bucket orders for every entry the two tables' lists can hold (orset_wire.hip buckets_of)
inline constexpr uint64_t cb_items_bytes(uint64_t st_cap, uint64_t rt_cap) {
    return 3 * cb_al((st_cap / 8) * kLists * 4 + 4) + 4 * cb_al((rt_cap / 8) * kLists * 4 + 4);
}
struct Claims {
    uint32_t* scnt;              // [cap + 1] new strings per set
    unsigned long long* sbytes;  // [cap + 1] their bytes
    uint32_t* rcnt[2];           // [cap + 1] records per set, per side
    uint2* splace;               // [string slots]
    uint2* rplace;               // [record slots]
    unsigned long long* uncounted;
    uint32_t cap;
};

__device__ __forceinline__ bool same_string(const Sparse& S, const uint8_t* bytes, uint64_t a, uint32_t set_a, unsigned long long key_a,
                                            uint32_t len_a, unsigned long long pfx_a, uint64_t noff_a, uint64_t b) {
    if (S.set[b] != set_a || S.key[b] != key_a || (S.meta[b] & 0x7FFFFFFFu) != len_a || S.pfx[b] != pfx_a) return false;
    return len_a <= 8 || same_bytes(bytes + S.noff[b] + 8, bytes + noff_a + 8, len_a - 8);
}

// kMsgsPerWave consecutive messages per wave for k_ow_rkeys / k_ow_rins, their tag references dealt over the
// 64 lanes in rounds: one message per wave left most lanes idle (≈23 references per ORSetWorkload state).
// Measured (round 4, one box): k_ow_rkeys 99 -> 69 us per wave, k_ow_rins 329 -> 317; the same for
// k_ow_strings was 7 % SLOWER (549 -> 589 us: its per-entry probe and string compare are a longer dependent
// chain, so packing its lanes only lengthens each wave) and it keeps one message per wave.
constexpr int kMsgsPerWave = 4;
// (round 5, the probe one load per slot: 2 and 4 messages per wave of k_ow_strings measured 491 and 522 us per wave
// against 505 at one — within noise either way, so it keeps one message per wave and its simpler duplicate check)

// The wave's messages [mb, mb + M) of [m0, m1): lane j < M holds message j's item count (0 for another
// kind's message or past m1) and its exclusive prefix; the total is wave-uniform.  Every shuffle reads lanes
// 0..M-1, so the callers run their item rounds with all 64 lanes active (a lane past the total idles).
template <int M>
struct WaveMsgs {
    uint32_t cnt = 0, pre = 0, total = 0;
    // the message of item q (< total): the last j whose prefix is <= q (a message without items shares its
    // prefix with the next one and never owns an item)
    __device__ __forceinline__ uint32_t owner(uint32_t q) const {
        uint32_t j = 0;
#pragma unroll
        for (int x = 1; x < M; ++x)
            if (q >= (uint32_t)__shfl((int)pre, x, 64)) j = (uint32_t)x;
        return j;
    }
    __device__ __forceinline__ void scan(uint32_t lane) {
        uint32_t incl = lane < (uint32_t)M ? cnt : 0u;
#pragma unroll
        for (int d = 1; d < M; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        total = (uint32_t)__shfl((int)incl, M - 1, 64);
        pre = incl - cnt;
    }
};
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, (int)src, 64) | (uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64) << 32;
}

// The lane that claims a string's slot also looks the string up in the store's element table (N: committed
// names, unchanged until the wave commits) and leaves the answer in sid_id[slot] (an id, kNoName for a new
// string, kUnresolved when the table or the set's generation word does not exist yet): the commit's
// per-string lookup — a chain of dependent random loads, 141 us behind the last upload of the ORSetWorkload
// wave — runs here, under the next chunk's upload.
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) void k_ow_strings(Sparse S, const uint64_t* __restrict__ off, const uint32_t* __restrict__ mset,
                                                       const uint8_t* __restrict__ bytes, const unsigned long long* __restrict__ ne,
                                                       const uint32_t* __restrict__ na, uint64_t m0, uint64_t m1, StrTab T,
                                                       unsigned long long* __restrict__ err, unsigned long long* __restrict__ overflow,
                                                       Names N, uint32_t set_lim, uint32_t* __restrict__ sid_id, Claims C) {
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t es_chunk = (off[m0] + kEntryDiv - 1) / kEntryDiv;  // entry slots from here on: this launch's
    const uint64_t m = m0 + (uint64_t)blockIdx.x * kTabWaves + wv;
    if (m >= m1) return;  // one message per wave: no workgroup barrier below
    const uint32_t set = mset[m];
    if (set == jg::kSkipIdx) return;
    const uint32_t cnt = (uint32_t)ne[m];
    if (cnt == 0) return;
    const uint64_t es = (off[m] + kEntryDiv - 1) / kEntryDiv;
    const uint32_t n_add = na[m] & 0x7FFFFFFFu, n_rem = cnt - n_add;
    const bool rem_first = (na[m] >> 31) != 0;
    bool over = false;
    for (uint32_t q0 = 0; q0 < cnt; q0 += 64) {  // wave-uniform bounds: list_append's ballot needs every lane
        const uint32_t q = q0 + lane;
        bool fresh = false, is_new = false;
        uint32_t sid = kNoSid, new_len = 0;
        if (q < cnt) {
        const uint64_t slot = es + q;
        const unsigned long long key = S.key[slot], pfx = S.pfx[slot];
        const uint32_t meta = S.meta[slot], len = meta & 0x7FFFFFFFu;
        const uint64_t noff = S.noff[slot];
        const unsigned long long word = (key >> 32) << 32 | (slot + 1);
        uint64_t p = key & T.mask;
        uint32_t first_seen = 0xFFFFFFFFu;  // the slot's `first` as the probe loaded it (it only decreases)
        for (uint32_t probe = 0; probe < kProbeCap; ++probe, p = (p + 1) & T.mask) {
            StrSlot* e = T.slot + p;
            // the whole 32-byte slot in one pair of loads: word, first, length | prefix, set, id (one dependent
            // memory level per probe instead of three: word, then the fingerprint, then `first` for the atomicMin)
            const uint4 h0 = reinterpret_cast<const uint4*>(e)[0], h1 = reinterpret_cast<const uint4*>(e)[1];
            unsigned long long w = (unsigned long long)h0.x | (unsigned long long)h0.y << 32;
            first_seen = h0.z;
            if (w == 0) {
                w = atomicCAS(&e->word, 0ull, word);
                if (w == 0) {
                    sid = (uint32_t)p;
                    fresh = true;
                    const uint32_t id0 = set < set_lim ? tab_find(N, key, set, bytes + noff, len) : kUnresolved;
                    sid_id[sid] = id0;
                    e->len = len;  // the fingerprint, read by the later chunks' launches
                    e->pfx = pfx;
                    e->set = set;
                    e->id0 = id0;
                    is_new = id0 == kNoName;
                    new_len = len;
                    if (id0 == kUnresolved) *C.uncounted = 1;
                    break;
                }
            }
            if ((w >> 32) != (key >> 32)) continue;
            const uint64_t b = (w & 0xFFFFFFFFull) - 1;
            // claimed in this launch: through the first inserter's entry (the loaded fingerprint may predate the
            // claim); by an earlier launch: the fingerprint, visible since that launch ended
            const bool same = b >= es_chunk ? same_string(S, bytes, slot, set, key, len, pfx, noff, b)
                                            : h0.w == len && h1.z == set && ((unsigned long long)h1.x | (unsigned long long)h1.y << 32) == pfx &&
                                                  (len <= 8 || same_bytes(bytes + S.noff[b] + 8, bytes + noff + 8, len - 8));
            if (same) {
                sid = (uint32_t)p;
                break;
            }
        }
        if (sid == kNoSid) {
            over = true;
        } else {
            const uint32_t c = (uint32_t)es + (!rem_first ? q : (q < n_rem ? n_add + q : q - n_rem));  // canonical: addSet first
            if (first_seen > c) atomicMin(&T.slot[sid].first, c);  // a stale `first` is only larger: the filter holds
        }
        S.sid[slot] = sid;
        }
        list_append(fresh, sid, T.list, T.n, T.sub_cap, overflow, m + q0 / 64);
        // the claim counted (one message per wave: every lane's set is `set`)
        const unsigned long long nb = __ballot(is_new);
        if (nb) {  // wave-uniform
            const int leader = __ffsll((long long)nb) - 1;
            unsigned long long bytes_sum = new_len;
            for (int o = 32; o > 0; o >>= 1) bytes_sum += __shfl_xor(bytes_sum, o);
            uint32_t base = 0;
            if ((int)lane == leader) {
                if (set < C.cap) {
                    base = atomicAdd(C.scnt + set, (uint32_t)__popcll(nb));
                    atomicAdd(C.sbytes + set, bytes_sum);
                } else {
                    *C.uncounted = 1;
                }
            }
            base = (uint32_t)__shfl((int)base, leader);
            if (is_new) C.splace[sid] = make_uint2(base + (uint32_t)__popcll(nb & ((1ull << lane) - 1ull)), set);
        }
        if (fresh && !is_new) C.splace[sid] = make_uint2(kDead, set);
    }
    if (__ballot(over) != 0 && lane == 0) *overflow = 1;
}

__global__ __launch_bounds__(kBlock) void k_ow_rkeys(Sparse S, const uint64_t* __restrict__ off, const uint32_t* __restrict__ mset,
                                                     const unsigned long long* __restrict__ nt, uint64_t m0, uint64_t m1) {
    constexpr int M = kMsgsPerWave;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t mb = m0 + ((uint64_t)blockIdx.x * kTabWaves + wv) * M;
    if (mb >= m1) return;  // wave-uniform
    WaveMsgs<M> W;
    uint32_t set = jg::kSkipIdx;
    uint64_t es = 0, ts = 0;
    if (lane < (uint32_t)M && mb + lane < m1) {
        set = mset[mb + lane];
        if (set != jg::kSkipIdx) {
            W.cnt = (uint32_t)nt[mb + lane];
            es = (off[mb + lane] + kEntryDiv - 1) / kEntryDiv;
            ts = (off[mb + lane] + kTagDiv - 1) / kTagDiv;
        }
    }
    W.scan(lane);
    for (uint32_t q0 = 0; q0 < W.total; q0 += 64) {  // wave-uniform rounds: the shuffles read lanes 0..M-1, which must be active
        const uint32_t q = q0 + lane;
        const uint32_t j = W.owner(q < W.total ? q : 0);
        const uint32_t qj = q - (uint32_t)__shfl((int)W.pre, (int)j, 64), sj = (uint32_t)__shfl((int)set, (int)j, 64);
        const uint64_t t = shfl64(ts, j) + qj, e0 = shfl64(es, j);
        if (q >= W.total) continue;
        const unsigned long long r = S.tref[t];
        const unsigned long long side = r >> 62 & 1;
        unsigned long long id;
        if (r >> 63) {
            id = 1ull << 63 | (unsigned long long)sj << 1 | side;
        } else {
            const uint32_t sid = S.sid[e0 + (uint32_t)r];
            id = sid == kNoSid ? kNone : ((unsigned long long)sid << 1 | side);
        }
        S.trk[t] = id;
    }
}

__global__ __launch_bounds__(kBlock) void k_ow_rins(Sparse S, const uint64_t* __restrict__ off, const uint32_t* __restrict__ mset,
                                                    const unsigned long long* __restrict__ nt, uint64_t m0, uint64_t m1, RecTab T,
                                                    unsigned long long* __restrict__ overflow, Claims C) {
    constexpr int M = kMsgsPerWave;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t mb = m0 + ((uint64_t)blockIdx.x * kTabWaves + wv) * M;
    if (mb >= m1) return;  // wave-uniform
    WaveMsgs<M> W;
    uint32_t set = jg::kSkipIdx;
    uint64_t ts = 0;
    if (lane < (uint32_t)M && mb + lane < m1) {
        set = mset[mb + lane];
        if (set != jg::kSkipIdx) {
            W.cnt = (uint32_t)nt[mb + lane];
            ts = (off[mb + lane] + kTagDiv - 1) / kTagDiv;
        }
    }
    W.scan(lane);
    bool over = false;
    for (uint32_t q0 = 0; q0 < W.total; q0 += 64) {  // wave-uniform bounds: list_append's ballot needs every lane
        const uint32_t q = q0 + lane;
        const uint32_t j = W.owner(q < W.total ? q : 0);
        const uint32_t sj = (uint32_t)__shfl((int)set, (int)j, 64);
        const uint64_t t = shfl64(ts, j) + (q - (uint32_t)__shfl((int)W.pre, (int)j, 64));
        const unsigned long long id = q < W.total ? S.trk[t] : kNone;
        bool fresh = false;
        uint64_t slot = ~0ull;
        uint32_t rkey = 0;
        if (id != kNone) {  // kNone: its string found no slot (the overflow word is up already), or past the wave's items
        const Tag16 g = S.tval[t];
        const uint64_t h = rec_hash(id, g, 0);
        const unsigned long long word = (h >> 32) << 32 | (t + 1);
        uint64_t p = h & T.mask;
        uint32_t mint_seen = 0xFFFFFFFFu;  // the slot's mint as the probe loaded it (it only decreases)
        for (uint32_t probe = 0; probe < kProbeCap; ++probe, p = (p + 1) & T.mask) {
            // most references repeat a record seen earlier in the wave: a plain load settles those (word and
            // mint in one 16-byte load: the atomicMin's filter needs no second trip)
            const uint4 hs = *reinterpret_cast<const uint4*>(T.slot + p);
            unsigned long long w = (unsigned long long)hs.x | (unsigned long long)hs.y << 32;
            mint_seen = hs.z;
            if (w == 0) {
                w = atomicCAS(&T.slot[p].word, 0ull, word);
                if (w == 0) {
                    slot = p;
                    fresh = true;
                    rkey = (uint32_t)(id & 1) << 31 | sj;  // the record's set is its message's
                    T.slot[slot].key = rkey;
                    break;
                }
            }
            if ((w >> 32) != (h >> 32)) continue;
            const uint64_t u = (w & 0xFFFFFFFFull) - 1;
            const Tag16 o = S.tval[u];
            if (S.trk[u] == id && o.lo == g.lo && o.hi == g.hi) {
                slot = p;
                break;
            }
        }
        if (slot == ~0ull) over = true;
        else if (mint_seen > (uint32_t)t) atomicMin(&T.slot[slot].mint, (uint32_t)t);  // a stale mint is only larger
        }
        list_append(fresh, (uint32_t)slot, T.list, T.n, T.sub_cap, overflow, mb / M + q0 / 64);
        // the claim counted in its (side, set) bucket
        const bool counted = fresh && sj < C.cap;
        const uint32_t pos = bucket_add(counted, rkey, C.rcnt[rkey >> 31] + (rkey & 0x7FFFFFFFu));
        if (counted) C.rplace[slot] = make_uint2(pos, rkey);
        else if (fresh) *C.uncounted = 1;
    }
    if (__ballot(over) != 0 && lane == 0) *overflow = 1;
}

// ---- commit from the tables ----------------------------------------------------------------------------
struct RecLive {  // list entry i: a record of side `side` whose first occurrence lies before the commit limit
    const uint32_t* list;
    const RecSlot* slot;
    const unsigned long long* trk;
    uint32_t lim, side;
    __host__ __device__ bool operator()(const uint32_t& i) const {
        const RecSlot& e = slot[list[i]];
        return e.mint < lim && (uint32_t)(trk[(e.word & 0xFFFFFFFFull) - 1] & 1) == side;
    }
};

// Each string of the table's list whose first entry lies before the limit, looked up in the set's element
// table: sid_id[sid] = its id, or a new string marked (set << 32 | first entry, to be sorted: ids go in
// first-insertion order per set).
__global__ void k_ow_sresolve(Sparse S, const uint8_t* __restrict__ bytes, StrTab T, uint64_t count, uint32_t lim, Names N,
                              uint32_t* __restrict__ sid_id, unsigned long long* __restrict__ newk) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const uint32_t sid = T.list[i];
    if (T.slot[sid].first >= lim) {
        newk[i] = kNone;
        return;
    }
    const uint64_t ref = (T.slot[sid].word & 0xFFFFFFFFull) - 1;
    const uint32_t set = S.set[ref];
    const uint32_t id = tab_find(N, S.key[ref], set, bytes + S.noff[ref], S.meta[ref] & 0x7FFFFFFFu);
    sid_id[sid] = id;
    newk[i] = id != kNoName ? kNone : ((unsigned long long)set << 32 | T.slot[sid].first);
}

// New strings sorted by (set, first entry): the r-th new string of a set takes next_id + r (k_ow_assign's
// rule, from the string slots).
// snk / snv: the wave's listed strings sorted by that key, the known ones (kNone) last; status[1] counts the
// new ones (the caller learns it at its next read, no sync here).
__global__ void k_ow_sassign(Sparse S, const uint8_t* __restrict__ bytes, StrTab T, const unsigned long long* __restrict__ snk,
                             const uint32_t* __restrict__ snv, uint64_t ns, uint64_t g0, Names N, uint32_t* __restrict__ sid_id,
                             unsigned long long* __restrict__ status) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= ns || snk[k] == kNone) return;
    if (k + 1 == ns || snk[k + 1] == kNone) status[1] = k + 1;  // the last new string: their count
    const uint32_t set = (uint32_t)(snk[k] >> 32);
    const uint64_t r = k - set_begin(snk, ns, set);
    const uint64_t id = (uint64_t)N.next_id[set] + r;
    if (id >= JG_NULL_ELEM - 1) atomicOr(status + 3, 1ull);
    const uint32_t sid = snv[k];
    const uint64_t ref = (T.slot[sid].word & 0xFFFFFFFFull) - 1;
    const uint32_t len = S.meta[ref] & 0x7FFFFFFFu;
    sid_id[sid] = (uint32_t)id;
    const uint64_t g = g0 + k;
    const unsigned long long p = atomicAdd(status + 2, (unsigned long long)len);
    const uint8_t* src = bytes + S.noff[ref];
    for (uint32_t q = 0; q < len; ++q) N.pool[p + q] = src[q];
    N.set[g] = set;
    N.id[g] = (uint32_t)id;
    N.gen[g] = N.set_gen[set];
    N.len[g] = len;
    N.off[g] = p;
    N.key[g] = S.key[ref];
    tab_insert(N, S.key[ref], (uint32_t)g);
    itab_insert(N, set, (uint32_t)id, (uint32_t)g);
}

// One side's live records (their table slots, compacted): store keys, tags, and the slot (its mint is the ord).
__global__ void k_ow_rgather(Sparse S, StrTab ST, RecTab RT, const uint32_t* __restrict__ sid_id, const uint32_t* __restrict__ idx,
                             const unsigned long long* __restrict__ count, unsigned long long* __restrict__ dk, Tag16* __restrict__ dt,
                             uint32_t* __restrict__ ds) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= *count) return;
    const uint32_t slot = RT.list[idx[j]];
    const uint64_t u = (RT.slot[slot].word & 0xFFFFFFFFull) - 1;
    const unsigned long long id = S.trk[u];
    unsigned long long key;
    if (id >> 63) {
        key = ((id >> 1) & 0xFFFFFFFFull) << 32 | JG_NULL_ELEM;
    } else {
        const uint32_t sid = (uint32_t)(id >> 1);
        const uint64_t ref = (ST.slot[sid].word & 0xFFFFFFFFull) - 1;
        key = (unsigned long long)S.set[ref] << 32 | sid_id[sid];
    }
    dk[j] = key;
    dt[j] = S.tval[u];
    ds[j] = slot;
}

// next_id of every set that took new strings (the sorted list's last new string of each set); kNone = known.
__global__ void k_ow_snext_ids(const unsigned long long* __restrict__ snk, uint64_t ns, Names N) {
    const uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= ns || snk[k] == kNone) return;
    const uint32_t set = (uint32_t)(snk[k] >> 32);
    if (k + 1 < ns && snk[k + 1] != kNone && (uint32_t)(snk[k + 1] >> 32) == set) return;  // not the set's last new string
    N.next_id[set] += (uint32_t)(k + 1 - set_begin(snk, ns, set));
}
