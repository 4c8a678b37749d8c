// orset_commit.hpp — the OR-Set wave commit from the tables, by set buckets (included by orset_wire.hip
// after orset_tables.hpp).
//
// A committed wave (ORSet.Merge of every state before the cut, ORSet.cs:253-283) needs two orders:
//   strings  the wave's new element strings get ids per set in first-insertion order (the add/remove
//            Dictionaries' order, :255-279): sorted by (set, first entry);
//   records  the wave's distinct tag records become a stream sorted by (set, element id, tag) that the
//            union merges into the store.
// Both orders are "by set, then a few hundred items of one set".  The round-3 commit sorted each list with a
// device-wide radix sort (rocprim's merge sort at these sizes: ~20 launches each, ~0.75 ms of launches, syncs
// and passes behind the last upload of the ORSetWorkload wave).  Here:
//   (claims)      when the whole wave commits, the tables' claimants already counted (Claims, orset_tables.hpp) and
//                 k_cb_scatter_claimed replaces k_cb_count + k_cb_scatter;
//   k_cb_count    one lane per listed string / record: known strings resolved against the element table,
//                 new strings (and their bytes) and live records counted per set (one atomic per run of a
//                 wave's items with one set, all in flight together) with their place in the set's bucket (the
//                 string's set and length, the record's side and set, stored beside the slots at claim time);
//   k_cb_scan     exclusive sums of the per-set counts and of the new strings' bytes, totals and the largest
//                 bucket — read back in the commit's one host sync;
//   k_cb_scatter  every item into its bucket;
//   k_cb_strings  one workgroup per set: the bucket sorted by first entry in LDS (a rank count, bitonic past
//                 256), ids next_id + rank, names appended in (set, first entry) order with their bytes placed by
//                 a prefix of lengths;
//   k_cb_records  one workgroup per (side, set): the bucket sorted by (element id, tag) in LDS, written straight
//                 into the dense stream the union reads (position = bucket offset + rank).
// A bucket larger than the LDS sort holds (kCbMax) sends the wave to the radix path (commit_tables' own).
#pragma once

constexpr uint32_t kCbMax = 2048;  // items of one set / (side, set) the LDS sorts hold
constexpr int kCbBlock = 256;      // the largest workgroup of k_cb_strings / k_cb_records
// Both kernels are launched with LDS for the wave's LARGEST bucket (P = its power of two, read back with the
// totals) and min(256, max(64, P)) threads: the ORSetWorkload's buckets hold tens to a few hundred items, and
// arrays sized for kCbMax (28 / 52 KB per workgroup) left 5 / 3 workgroups per CU for 2000 / 4000 of them.
__host__ __device__ constexpr size_t cb_strings_lds(uint32_t P) { return (size_t)P * 30 + 64; }
__host__ __device__ constexpr size_t cb_records_lds(uint32_t P) { return (size_t)P * 26 + 64; }

struct Buckets {
    uint32_t* scnt;              // [n_sets + 1] new strings per set -> exclusive offsets
    unsigned long long* sbytes;  // [n_sets + 1] their bytes -> exclusive byte offsets
    uint32_t* rcnt[2];           // [n_sets + 1] live records per set, per side -> exclusive offsets
    uint32_t* spos;              // [ns] place of listed string i in its set's bucket (kDead: known / past the limit)
    uint32_t* sset;              // [ns] its set
    uint32_t* rpos;              // [nrec] place of listed record j in its (side, set) bucket (kDead: past the limit)
    uint32_t* rset;              // [nrec] side << 31 | set
    uint32_t* sitem;             // [new strings] their string slots in bucket order
    uint32_t* ritem[2];          // [live records of the side] their record slots in bucket order
    uint32_t n_sets;
};

__global__ __launch_bounds__(kBlock) void k_cb_count(Sparse S, const uint8_t* __restrict__ bytes, StrTab T, RecTab R, uint64_t ns, uint64_t nrec,
                                                     uint32_t s_lim, uint32_t t_lim, Names N, uint32_t* __restrict__ sid_id, Buckets B) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    // a workgroup's lanes are all strings or all records up to the boundary wave (ns need not be a multiple of 64:
    // both adds run in every wave, each with its own lanes active)
    bool s_new = false, r_live = false;
    uint32_t s_set = 0, s_len = 0, r_key = 0;
    if (i < ns) {
        const uint32_t sid = T.list[i];
        const StrSlot& se = T.slot[sid];  // set, length, id looked up when the chunk's k_ow_strings claimed the slot
        const uint4 mt = make_uint4(se.set, se.len, se.id0, 0u);
        if (T.slot[sid].first < s_lim) {
            uint32_t id = mt.z;
            if (id == kUnresolved) {
                const uint64_t ref = (T.slot[sid].word & 0xFFFFFFFFull) - 1;
                id = tab_find(N, S.key[ref], mt.x, bytes + S.noff[ref], mt.y);
                if (id != kNoName) sid_id[sid] = id;
            }
            if (id == kNoName) {
                s_new = true;
                s_set = mt.x;
                s_len = mt.y;
            }
        }
    } else if (i - ns < nrec) {
        const uint32_t slot = R.list[i - ns];
        if (R.slot[slot].mint < t_lim) {
            r_live = true;
            r_key = R.slot[slot].key;
        }
    }
    const uint32_t sp = bucket_add(s_new, s_set, B.scnt + s_set);
    run_bytes(s_new, s_set, B.sbytes + s_set, s_len);
    const uint32_t rp = bucket_add(r_live, r_key, B.rcnt[r_key >> 31] + (r_key & 0x7FFFFFFFu));
    if (i < ns) {
        B.spos[i] = s_new ? sp : kDead;
        B.sset[i] = s_set;
    } else if (i - ns < nrec) {
        B.rpos[i - ns] = r_live ? rp : kDead;
        B.rset[i - ns] = r_key;
    }
}

// Exclusive sums of the four per-set arrays in place (n + 1 entries each, the last one 0 before: the total
// after), one workgroup per array, tiles of 1024 x 4 with a carried prefix; status[k] = total, status[4 + k]
// = the largest entry.
constexpr int kScanThreads = 1024, kScanItems = 4;
template <class T> __device__ void scan_array(T* a, uint64_t n, unsigned long long* total, unsigned long long* maxv) {
    __shared__ unsigned long long part[kScanThreads];
    __shared__ unsigned long long carry_s;
    const uint32_t t = threadIdx.x;
    if (t == 0) carry_s = 0;
    unsigned long long mx = 0;
    __syncthreads();
    for (uint64_t base = 0; base < n; base += (uint64_t)kScanThreads * kScanItems) {
        unsigned long long v[kScanItems], s = 0;
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t x = base + (uint64_t)t * kScanItems + q;
            v[q] = x < n ? (unsigned long long)a[x] : 0ull;
            mx = v[q] > mx ? v[q] : mx;
            s += v[q];
        }
        part[t] = s;
        __syncthreads();
        for (int o = 1; o < kScanThreads; o <<= 1) {  // inclusive Hillis-Steele over the thread sums
            const unsigned long long y = t >= (uint32_t)o ? part[t - o] : 0ull;
            __syncthreads();
            part[t] += y;
            __syncthreads();
        }
        unsigned long long run = carry_s + (t ? part[t - 1] : 0ull);
        for (int q = 0; q < kScanItems; ++q) {
            const uint64_t x = base + (uint64_t)t * kScanItems + q;
            if (x < n) a[x] = (T)run;
            run += v[q];
        }
        __syncthreads();
        if (t == kScanThreads - 1) carry_s += part[t];
        __syncthreads();
    }
    // the largest entry (a block max through the same LDS)
    part[t] = mx;
    __syncthreads();
    for (int o = kScanThreads / 2; o > 0; o >>= 1) {
        if (t < (uint32_t)o && part[t + o] > part[t]) part[t] = part[t + o];
        __syncthreads();
    }
    if (t == 0) {
        *total = carry_s;
        *maxv = part[0];
    }
}

__global__ __launch_bounds__(kScanThreads) void k_cb_scan(Buckets B, uint64_t n, unsigned long long* __restrict__ status) {
    switch (blockIdx.x) {
        case 0: scan_array(B.scnt, n, status + 0, status + 4); break;
        case 1: scan_array(B.sbytes, n, status + 1, status + 5); break;
        case 2: scan_array(B.rcnt[0], n, status + 2, status + 6); break;
        default: scan_array(B.rcnt[1], n, status + 3, status + 7); break;
    }
}

__global__ __launch_bounds__(kBlock) void k_cb_scatter(uint64_t ns, uint64_t nrec, const StrTab T, const RecTab R, Buckets B) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < ns) {
        const uint32_t p = B.spos[i];
        if (p != kDead) B.sitem[B.scnt[B.sset[i]] + p] = T.list[i];
    } else if (i - ns < nrec) {
        const uint64_t j = i - ns;
        const uint32_t p = B.rpos[j];
        if (p != kDead) {
            const uint32_t k = B.rset[j], sd = k >> 31;
            B.ritem[sd][B.rcnt[sd][k & 0x7FFFFFFFu] + p] = R.list[j];
        }
    }
}

// The same scatter from the places the tables' claimants took (k_ow_strings / k_ow_rins, `Claims`): a commit
// of the whole wave whose claims all counted reads one 8-byte place per listed item instead of k_cb_count's
// pass over the slots.  Grid-stride over the packed lists (offs: both tables' sub-list offsets, on the device).
// The check queues it before its one read (spec_commit_prep), so it runs before anyone knows whether the wave's
// claims all counted: it leaves without writing when a claim went uncounted or a table overflowed (places may then
// be stale, or name sets past the count arrays) — such a wave never commits from the claims.
//
// Round 5's fault (gpurun_out/r05/cb10): the first version of this speculative launch stored through
// bucket arrays carved from a block the commit had sized for the previous wave's items (or not yet allocated), so
// its stores ran past the block.  The block is now sized by tables_begin for the tables' capacities and the check
// refuses to queue the launch otherwise.  Past the guard, a listed slot outside its table, a place naming a set past
// the count arrays, or a bucket position past the arrays can only mean the tables are inconsistent: such an item is
// not written, and `bad` (zeroed by k_list_offs, read with the check's words) fails the wave's check with JG_EHIP —
// before anything of it commits — instead of committing a bucket with a stale slot.
__global__ __launch_bounds__(kBlock) void k_cb_scatter_claimed(const unsigned long long* __restrict__ offs, const StrTab T, const RecTab R,
                                                               Claims C, Buckets B, const unsigned long long* __restrict__ overflow,
                                                               unsigned long long* __restrict__ bad) {
    if (*overflow != 0 || *C.uncounted != 0) return;
    const uint64_t ns = offs[kLists], nrec = offs[2 * kLists + 1];
    const uint64_t cap_s = kLists * T.sub_cap, cap_r = kLists * R.sub_cap;  // the bucket arrays' capacities
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < ns + nrec; i += (uint64_t)gridDim.x * kBlock) {
        if (i < ns) {
            const uint32_t sid = T.list[i];
            if (sid > T.mask) { atomicOr(bad, 1ull); continue; }
            const uint2 pl = C.splace[sid];
            if (pl.x == kDead) continue;  // a name the element table already holds: no new id, no bucket place
            const uint64_t at = pl.y < C.cap ? (uint64_t)B.scnt[pl.y] + pl.x : ~0ull;
            if (at >= cap_s) { atomicOr(bad, 2ull); continue; }
            B.sitem[at] = sid;
        } else {
            const uint32_t slot = R.list[i - ns];
            if (slot > R.mask) { atomicOr(bad, 4ull); continue; }
            const uint2 pl = C.rplace[slot];
            const uint32_t sd = pl.y >> 31, set = pl.y & 0x7FFFFFFFu;
            const uint64_t at = set < C.cap ? (uint64_t)B.rcnt[sd][set] + pl.x : ~0ull;
            if (at >= cap_r) { atomicOr(bad, 8ull); continue; }
            B.ritem[sd][at] = slot;
        }
    }
}

// Bitonic sort of P (a power of two, <= kCbMax) slots by less(a, b) over an LDS permutation.
template <class Less> __device__ void lds_bitonic(uint16_t* perm, uint32_t P, Less less) {
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < P / 2; x += blockDim.x) {
                const uint32_t a = 2 * j * (x / j) + (x % j), b = a + j;
                const bool up = (a & k) == 0;
                const uint16_t pa = perm[a], pb = perm[b];
                if (less(pb, pa) == up) {
                    perm[a] = pb;
                    perm[b] = pa;
                }
            }
            __syncthreads();
        }
}

// The same permutation by counting for a bucket of at most one item per thread: item r's rank is the number of
// items before it in the order (the order is total: ties broken by index).  A ~200-item bucket takes ~200 LDS
// broadcast reads per thread instead of bitonic's 36 passes with a workgroup barrier each.
template <class Less> __device__ void lds_rank_sort(uint16_t* perm, uint32_t cnt, Less less) {
    const uint32_t r = threadIdx.x;
    if (r < cnt) {
        uint32_t rank = 0;
        for (uint32_t j = 0; j < cnt; ++j) rank += less((uint16_t)j, (uint16_t)r) ? 1u : 0u;
        perm[rank] = (uint16_t)r;
    }
    __syncthreads();
}

__host__ __device__ __forceinline__ uint32_t pow2_ge(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// One workgroup per set: its new strings by first entry; ids next_id + rank; names g0 + bucket offset + rank
// with their bytes at pool0 + the set's byte offset + the prefix of lengths in rank order.  Everything a
// string's name needs (its first entry, length, first inserter's name offset and key) is gathered into LDS
// before the sort, and the set's counters with it, so the write phase waits on memory only for the bytes and
// the two table inserts (a chain of ~13 dependent loads became ~8).
__global__ __launch_bounds__(kCbBlock) void k_cb_strings(Sparse S, const uint8_t* __restrict__ bytes, StrTab T, Buckets B, uint64_t g0,
                                                         uint64_t pool0, Names N, uint32_t* __restrict__ sid_id,
                                                         unsigned long long* __restrict__ status) {
    const uint32_t s = blockIdx.x;
    const uint32_t o0 = B.scnt[s], cnt = B.scnt[s + 1] - o0;
    if (cnt == 0) return;
    const uint64_t pbase = pool0 + B.sbytes[s];
    const uint32_t next = N.next_id[s], gen = N.set_gen[s];
    const uint32_t P = pow2_ge(cnt), NT = blockDim.x;
    extern __shared__ __align__(16) unsigned char cb_lds[];  // cb_strings_lds(the launch's largest P)
    __shared__ unsigned long long wsum[kCbBlock / 64];
    unsigned long long* noff = reinterpret_cast<unsigned long long*>(cb_lds);
    unsigned long long* skey = noff + P;
    uint32_t* key = reinterpret_cast<uint32_t*>(skey + P);
    uint32_t* item = key + P;
    uint32_t* lens = item + P;
    uint16_t* perm = reinterpret_cast<uint16_t*>(lens + P);
    for (uint32_t r = threadIdx.x; r < P; r += NT) {
        if (r < cnt) {
            const uint32_t sid = B.sitem[o0 + r];
            const StrSlot& e = T.slot[sid];
            const unsigned long long word = e.word;
            const uint32_t first = e.first, len = e.len;
            const uint64_t ref = (word & 0xFFFFFFFFull) - 1;
            item[r] = sid;
            key[r] = first;
            lens[r] = len;
            noff[r] = S.noff[ref];
            skey[r] = S.key[ref];
        }
        perm[r] = (uint16_t)r;
    }
    __syncthreads();
    const auto by_first = [&](uint16_t a, uint16_t b) {
        const uint32_t ka = a < cnt ? key[a] : 0xFFFFFFFFu, kb = b < cnt ? key[b] : 0xFFFFFFFFu;
        return ka != kb ? ka < kb : a < b;  // pads (index >= cnt) last
    };
    if (cnt <= NT) lds_rank_sort(perm, cnt, by_first);
    else lds_bitonic(perm, P, by_first);
    // exclusive prefix of the lengths in rank order (each thread a contiguous run, then the thread sums)
    const uint32_t per = (cnt + NT - 1) / NT, r0 = min(cnt, threadIdx.x * per), r1 = min(cnt, r0 + per);
    unsigned long long mine = 0;
    for (uint32_t r = r0; r < r1; ++r) mine += lens[perm[r]];
    unsigned long long incl = mine;  // inclusive scan over the threads: wave scan, then the wave totals
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o);
        if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    unsigned long long before = incl - mine;
    for (uint32_t q = 0; q < wv; ++q) before += wsum[q];
    for (uint32_t r = r0; r < r1; ++r) {
        const uint32_t x = perm[r];
        const uint32_t sid = item[x], len = lens[x];
        const unsigned long long k = skey[x];
        const uint64_t id = (uint64_t)next + r;
        if (id >= JG_NULL_ELEM - 1) atomicOr(status + 8, 1ull);
        sid_id[sid] = (uint32_t)id;
        const uint64_t g = g0 + o0 + r, p = pbase + before;
        const uint8_t* src = bytes + noff[x];
        for (uint32_t q = 0; q < len; ++q) N.pool[p + q] = src[q];
        before += len;
        N.set[g] = s;
        N.id[g] = (uint32_t)id;
        N.gen[g] = gen;
        N.len[g] = len;
        N.off[g] = p;
        N.key[g] = k;
        tab_insert(N, k, (uint32_t)g);
        itab_insert(N, s, (uint32_t)id, (uint32_t)g);
    }
    __syncthreads();
    if (threadIdx.x == 0) N.next_id[s] = next + cnt;
}

// One workgroup per (set, side): its live records by (element id, tag.lo, tag.hi) into the side's dense stream
// at the bucket's offset; ord = the record's arrival ordinal (its first tag slot).
__global__ __launch_bounds__(kCbBlock) void k_cb_records(Sparse S, StrTab T, RecTab R, Buckets B, const uint32_t* __restrict__ sid_id,
                                                         unsigned long long* __restrict__ k0, Tag16* __restrict__ t0, uint32_t* __restrict__ o0_,
                                                         unsigned long long* __restrict__ k1, Tag16* __restrict__ t1, uint32_t* __restrict__ o1_) {
    const uint32_t s = blockIdx.x, sd = blockIdx.y;
    const uint32_t* off = B.rcnt[sd];
    const uint32_t o0 = off[s], cnt = off[s + 1] - o0;
    if (cnt == 0) return;
    const uint32_t P = pow2_ge(cnt), NT = blockDim.x;
    extern __shared__ __align__(16) unsigned char cb_lds[];  // cb_records_lds(the launch's largest P)
    unsigned long long* lo = reinterpret_cast<unsigned long long*>(cb_lds);
    unsigned long long* hi = lo + P;
    uint32_t* elem = reinterpret_cast<uint32_t*>(hi + P);
    uint32_t* mint = elem + P;
    uint16_t* perm = reinterpret_cast<uint16_t*>(mint + P);
    const uint32_t* items = B.ritem[sd];
    for (uint32_t r = threadIdx.x; r < P; r += NT) {
        if (r < cnt) {
            const uint32_t slot = items[o0 + r];
            const uint64_t u = (R.slot[slot].word & 0xFFFFFFFFull) - 1;
            const unsigned long long id = S.trk[u];
            elem[r] = (id >> 63) ? JG_NULL_ELEM : sid_id[(uint32_t)(id >> 1)];
            const Tag16 g = S.tval[u];
            lo[r] = g.lo;
            hi[r] = g.hi;
            mint[r] = R.slot[slot].mint;
        }
        perm[r] = (uint16_t)r;
    }
    __syncthreads();
    const auto by_record = [&](uint16_t a, uint16_t b) {
        const bool pa = a >= cnt, pb = b >= cnt;  // pads last
        if (pa || pb) return !pa && pb ? true : (pa && pb ? a < b : false);
        if (elem[a] != elem[b]) return elem[a] < elem[b];
        if (lo[a] != lo[b]) return lo[a] < lo[b];
        if (hi[a] != hi[b]) return hi[a] < hi[b];
        return a < b;  // (never equal: the records are distinct) a total order for the rank count
    };
    lds_bitonic(perm, P, by_record);  // (a rank count over three-field keys measured slower here: 108 vs 64 us per wave)
    unsigned long long* ok = sd ? k1 : k0;
    Tag16* ot = sd ? t1 : t0;
    uint32_t* oo = sd ? o1_ : o0_;
    for (uint32_t r = threadIdx.x; r < cnt; r += NT) {
        const uint32_t x = perm[r];
        ok[o0 + r] = (unsigned long long)s << 32 | elem[x];
        ot[o0 + r] = Tag16{lo[x], hi[x]};
        oo[o0 + r] = mint[x];
    }
}
