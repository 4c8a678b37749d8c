// oracle/capi.cpp — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
//
// extern "C" bridge so pytest (ctypes) and bench.py's cpu_baseline leg can drive the oracle on
// the same dense / record layouts the GPU engine uses.  Every bridge routes the data through the
// dictionary-faithful objects of oracle.hpp; nothing here re-implements merge arithmetic on
// arrays.  Also holds the host copy of the synthetic-workload generators (BASELINE.md §2,
// SURVEY.md §8d D2/D3), which the HIP engine re-states on the device in synth.hip.
#include <chrono>
#include <cstring>
#include <limits>
#include <thread>

#include "json.hpp"
#include "oracle.hpp"

using namespace oracle;

namespace {

constexpr uint32_t kNullElem = 0xFFFFFFFFu;  // elem id of C# null (ORSet.cs:136-140)

// key = set << 32 | elem; tag = {t0, t1} (16 opaque bytes); ord = arrival ordinal (jg_tagrec.ord:
// tags of one (set, elem) enumerate in ascending (ord, tag); remove-Dictionary elements by their
// smallest ord, ties by elem; add-Dictionary elements by elem id)
struct Rec { uint64_t key, t0, t1, ord; };

// Column c of key k is replica Guid {k+1, c+1}: unique per (key, replica) like the reference's
// per-instance Guid.NewGuid() (PNCounters.cs:75).
inline Guid col_guid(uint64_t k, uint32_t c) { Guid g; g.lo = k + 1; g.hi = (uint64_t)c + 1; return g; }

template <class T> inline T absent_sentinel() { return std::numeric_limits<T>::min(); }

template <class T>
void load_local(PNCounter<T>& pc, uint64_t k, uint32_t R, const T* P, const T* N) {
    for (uint32_t c = 0; c < R; ++c) pc.mutP()[col_guid(k, c)] = P[k * R + c];
    for (uint32_t c = 0; c < R; ++c) pc.mutN()[col_guid(k, c)] = N[k * R + c];
}

template <class T>
PNCounterMsg<T> row_msg(uint64_t k, uint32_t R, const T* P, const T* N) {
    PNCounterMsg<T> m;
    for (uint32_t c = 0; c < R; ++c) if (P[c] != absent_sentinel<T>()) m.pVector[col_guid(k, c)] = P[c];
    for (uint32_t c = 0; c < R; ++c) if (N[c] != absent_sentinel<T>()) m.nVector[col_guid(k, c)] = N[c];
    return m;
}

template <class T>
int pnc_merge(uint64_t n_keys, uint32_t R, T* AP, T* AN, uint64_t n_rows, const uint32_t* key_idx, const T* BP, const T* BN) {
    std::unordered_map<uint64_t, PNCounter<T>> live;
    for (uint64_t m = 0; m < n_rows; ++m) {
        uint64_t k = key_idx ? key_idx[m] : m;
        if (k >= n_keys) return -1;
        auto it = live.find(k);
        if (it == live.end()) {
            it = live.emplace(k, PNCounter<T>(Guid{k + 1, 0})).first;
            it->second.mutP().Clear(); it->second.mutN().Clear();  // dense rows carry every column
            load_local(it->second, k, R, AP, AN);
        }
        it->second.Merge(row_msg<T>(k, R, BP + m * R, BN + m * R));
    }
    for (auto& kv : live) {
        uint64_t k = kv.first;
        for (uint32_t c = 0; c < R; ++c) { kv.second.P().TryGetValue(col_guid(k, c), AP[k * R + c]); kv.second.N().TryGetValue(col_guid(k, c), AN[k * R + c]); }
    }
    return 0;
}

template <class T>
int pnc_values(uint64_t n_keys, uint32_t R, const T* P, const T* N, uint64_t n_q, const uint32_t* key_idx, int64_t* out, uint8_t* ovf) {
    for (uint64_t q = 0; q < n_q; ++q) {
        uint64_t k = key_idx ? key_idx[q] : q;
        if (k >= n_keys) return -1;
        PNCounter<T> pc(Guid{k + 1, 0});
        pc.mutP().Clear(); pc.mutN().Clear();
        load_local(pc, k, R, P, N);
        try { out[q] = (int64_t)pc.Get(); ovf[q] = 0; }
        catch (const OverflowException&) { out[q] = 0; ovf[q] = 1; }
    }
    return 0;
}

// ---- OR-Set record <-> object bridge ----------------------------------------------------------
inline Elem elem_of(uint32_t e) { return e == kNullElem ? Elem() : Elem(std::to_string(e)); }
inline uint32_t elem_id(const std::string& s) { return (uint32_t)std::stoul(s); }
inline Guid tag_of(const Rec& r) { Guid g; g.lo = r.t0; g.hi = r.t1; return g; }

// ORSet objects from records: each set's add Dictionary filled in ascending elem id, its remove
// Dictionary in ascending (smallest ord, elem), every HashSet in ascending (ord, tag) — the order the
// engine's records encode (jg_tagrec.ord).
void build_sets(std::map<uint32_t, ORSet>& sets, const Rec* A, uint64_t nA, const Rec* Rm, uint64_t nR) {
    auto tag_order = [](const Rec& a, const Rec& b) {
        return a.key != b.key ? a.key < b.key : a.ord != b.ord ? a.ord < b.ord : a.t0 != b.t0 ? a.t0 < b.t0 : a.t1 < b.t1;
    };
    std::vector<Rec> add(A, A + nA), rem(Rm, Rm + nR);
    std::sort(add.begin(), add.end(), tag_order);  // by (set, elem): ascending id, then HashSet order
    for (const Rec& r : add) sets[(uint32_t)(r.key >> 32)].AddTag(elem_of((uint32_t)r.key), tag_of(r));
    std::sort(rem.begin(), rem.end(), tag_order);
    std::unordered_map<uint64_t, uint64_t> first;  // key -> smallest ord
    for (const Rec& r : rem) {
        auto it = first.find(r.key);
        if (it == first.end()) first.emplace(r.key, r.ord);
    }
    std::stable_sort(rem.begin(), rem.end(), [&](const Rec& a, const Rec& b) {
        const uint32_t sa = (uint32_t)(a.key >> 32), sb = (uint32_t)(b.key >> 32);
        if (sa != sb) return sa < sb;
        const uint64_t fa = first.at(a.key), fb = first.at(b.key);
        return fa != fb ? fa < fb : (uint32_t)a.key < (uint32_t)b.key;
    });
    for (const Rec& r : rem) {
        ORSet& o = sets[(uint32_t)(r.key >> 32)];
        const uint32_t e = (uint32_t)r.key;
        if (e == kNullElem) o.mutNullRem().insert(tag_of(r));
        else o.mutRemoveSet()[std::to_string(e)].insert(tag_of(r));
    }
}

// Records of ORSet objects, sorted by (key, t0, t1); ord = the record's position in its set's
// enumeration (Dictionary entries in order, each HashSet in order, then the null set).
void export_sets(const std::map<uint32_t, ORSet>& sets, std::vector<Rec>& add, std::vector<Rec>& rem) {
    for (const auto& kv : sets) {
        uint64_t s = (uint64_t)kv.first << 32;
        uint64_t oa = 0, orr = 0;
        for (const auto& e : kv.second.addSet()) for (const auto& g : e.second) add.push_back(Rec{s | elem_id(e.first), g.lo, g.hi, oa++});
        for (const auto& e : kv.second.removeSet()) for (const auto& g : e.second) rem.push_back(Rec{s | elem_id(e.first), g.lo, g.hi, orr++});
        for (const auto& g : kv.second.nullAdd()) add.push_back(Rec{s | kNullElem, g.lo, g.hi, oa++});
        for (const auto& g : kv.second.nullRem()) rem.push_back(Rec{s | kNullElem, g.lo, g.hi, orr++});
    }
    auto lt = [](const Rec& a, const Rec& b) { return a.key != b.key ? a.key < b.key : a.t0 != b.t0 ? a.t0 < b.t0 : a.t1 < b.t1; };
    std::sort(add.begin(), add.end(), lt);
    std::sort(rem.begin(), rem.end(), lt);
}

// ---- synthetic generators (host copy; device copy in janus-crdt_amd/csrc/synth.hip) ------------
inline uint64_t synth_hash(uint64_t seed, uint64_t idx) { return mix64(seed + (idx + 1) * 0x9E3779B97F4A7C15ull); }

inline int64_t synth_pnc_cell(uint64_t seed, uint32_t which, uint64_t key, uint32_t col, uint32_t R, uint32_t elem_bytes) {
    uint64_t idx = ((key * R + col) << 2) | which;
    uint64_t h = synth_hash(seed, idx);
    if (h % 100 < 30) {  // unseen replica: 0 locally, absent in a received message
        if (which < 2) return 0;
        return elem_bytes == 4 ? (int64_t)INT32_MIN : INT64_MIN;
    }
    return (int64_t)((h >> 33) % 2147483647ull);
}

inline Rec synth_orset_rec(uint64_t seed, uint64_t g, uint32_t u, uint32_t elems_per_set) {
    uint64_t h1 = mix64(seed ^ mix64(g * 256 + u + 1));
    uint64_t h2 = mix64(h1 + 0x9E3779B97F4A7C15ull);
    Rec r;
    r.key = ((g / elems_per_set) << 32) | (g % elems_per_set);
    r.t0 = ((uint64_t)u << 56) | (h1 >> 8);
    r.t1 = h2;
    r.ord = 0;  // set by the caller: the record's index in its stream (synth.hip)
    return r;
}

template <class T> double median_of(std::vector<T> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : (double)v[v.size() / 2]; }

}  // namespace

extern "C" {

int orc_version(void) { return 1; }

// ---- synthetic workloads ----------------------------------------------------------------------
// which: 0 = local P, 1 = local N, 2 = received P, 3 = received N.  Rows [key0, key0+n_keys).
void orc_synth_pnc_rows(uint64_t seed, uint32_t which, uint64_t key0, uint64_t n_keys, uint32_t R, uint32_t elem_bytes, void* out) {
    for (uint64_t k = 0; k < n_keys; ++k)
        for (uint32_t c = 0; c < R; ++c) {
            int64_t v = synth_pnc_cell(seed, which, key0 + k, c, R, elem_bytes);
            if (elem_bytes == 4) ((int32_t*)out)[k * R + c] = (int32_t)v;
            else ((int64_t*)out)[k * R + c] = v;
        }
}

// Records [first, first+n) of a stream holding `per_group` tags u in [u0, u0+per_group) for every
// (set, elem) group in order; group g = set * elems_per_set + elem.
void orc_synth_orset(uint64_t seed, uint64_t first, uint64_t n, uint32_t elems_per_set, uint32_t per_group, uint32_t u0, Rec* out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t r = first + i;
        out[i] = synth_orset_rec(seed, r / per_group, u0 + (uint32_t)(r % per_group), elems_per_set);
        out[i].ord = r;
    }
}

// ---- PN-Counter bridges (elem_bytes 4 = reference int, 8 = long variant) ----------------------
// Merge received rows (ABSENT = INT_MIN of the width marks an entry missing from the message)
// into the dense local store [n_keys x R], in row order, through PNCounter::Merge.
int orc_pnc_merge_dense(uint64_t n_keys, uint32_t R, uint32_t elem_bytes, void* AP, void* AN, uint64_t n_rows,
                        const uint32_t* key_idx, const void* BP, const void* BN) {
    if (elem_bytes == 4) return pnc_merge<int32_t>(n_keys, R, (int32_t*)AP, (int32_t*)AN, n_rows, key_idx, (const int32_t*)BP, (const int32_t*)BN);
    if (elem_bytes == 8) return pnc_merge<int64_t>(n_keys, R, (int64_t*)AP, (int64_t*)AN, n_rows, key_idx, (const int64_t*)BP, (const int64_t*)BN);
    return -2;
}

// PNCounter.Get per queried key (column order = dictionary order): value, or ovf=1 where the
// checked LINQ Sum throws OverflowException.
int orc_pnc_values_dense(uint64_t n_keys, uint32_t R, uint32_t elem_bytes, const void* P, const void* N, uint64_t n_q,
                         const uint32_t* key_idx, int64_t* out, uint8_t* ovf) {
    if (elem_bytes == 4) return pnc_values<int32_t>(n_keys, R, (const int32_t*)P, (const int32_t*)N, n_q, key_idx, out, ovf);
    if (elem_bytes == 8) return pnc_values<int64_t>(n_keys, R, (const int64_t*)P, (const int64_t*)N, n_q, key_idx, out, ovf);
    return -2;
}

// Increment / Decrement on replica column `col` of `key`, in op order (PNCounters.cs:97-112,
// unchecked '+=').  Each op runs on a PNCounter whose own replica is that column.
int orc_pnc_apply_ops_dense(uint64_t n_keys, uint32_t R, uint32_t elem_bytes, void* P, void* N, uint64_t n_ops,
                            const uint32_t* key, const uint32_t* col, const int64_t* delta, const uint8_t* is_n) {
    for (uint64_t i = 0; i < n_ops; ++i) {
        if (key[i] >= n_keys || col[i] >= R) return -1;
        uint64_t at = (uint64_t)key[i] * R + col[i];
        if (elem_bytes == 4) {
            PNCounter<int32_t> pc(col_guid(key[i], col[i]));
            int32_t* arr = is_n[i] ? (int32_t*)N : (int32_t*)P;
            (is_n[i] ? pc.mutN() : pc.mutP())[pc.replicaIdx()] = arr[at];
            if (is_n[i]) pc.Decrement((int32_t)delta[i]); else pc.Increment((int32_t)delta[i]);
            (is_n[i] ? pc.N() : pc.P()).TryGetValue(pc.replicaIdx(), arr[at]);
        } else if (elem_bytes == 8) {
            PNCounter<int64_t> pc(col_guid(key[i], col[i]));
            int64_t* arr = is_n[i] ? (int64_t*)N : (int64_t*)P;
            (is_n[i] ? pc.mutN() : pc.mutP())[pc.replicaIdx()] = arr[at];
            if (is_n[i]) pc.Decrement(delta[i]); else pc.Increment(delta[i]);
            (is_n[i] ? pc.N() : pc.P()).TryGetValue(pc.replicaIdx(), arr[at]);
        } else return -2;
    }
    return 0;
}

// ---- OR-Set bridges ---------------------------------------------------------------------------
// Local state (La adds, Lr tombstones) merged with received (Ra, Rr) through ORSet::Merge per set,
// exported canonically (sorted by key, t0, t1).  out arrays need room for nLa+nRa / nLr+nRr.
int orc_orset_merge(const Rec* La, uint64_t nLa, const Rec* Lr, uint64_t nLr, const Rec* Ra, uint64_t nRa,
                    const Rec* Rr, uint64_t nRr, Rec* out_a, uint64_t* n_out_a, Rec* out_r, uint64_t* n_out_r) {
    std::map<uint32_t, ORSet> local, recv;
    build_sets(local, La, nLa, Lr, nLr);
    build_sets(recv, Ra, nRa, Rr, nRr);
    for (const auto& kv : recv) local[kv.first].Merge(kv.second.GetLastSynchronizedUpdate());
    std::vector<Rec> a, r;
    export_sets(local, a, r);
    std::copy(a.begin(), a.end(), out_a); *n_out_a = a.size();
    std::copy(r.begin(), r.end(), out_r); *n_out_r = r.size();
    return 0;
}

// ORSet.Contains(elem) of `set` for each query (elem 0xFFFFFFFF = null).
int orc_orset_contains(const Rec* A, uint64_t nA, const Rec* Rm, uint64_t nR, uint64_t n_q, const uint32_t* set,
                       const uint32_t* elem, uint8_t* out) {
    std::map<uint32_t, ORSet> sets;
    build_sets(sets, A, nA, Rm, nR);
    for (uint64_t q = 0; q < n_q; ++q) {
        auto it = sets.find(set[q]);
        out[q] = (it != sets.end() && it->second.Contains(elem_of(elem[q]))) ? 1 : 0;
    }
    return 0;
}

// ORSet.Add / Remove / Clear applied in op order (op 1 Add with the given tag, 2 Remove, 3 Clear)
// to the state (A adds, Rm tombstones) through ORSet objects; exports the new state canonically and
// each op's bool result.  out arrays need room for nA + n_ops / nR + (all tags that could be
// tombstoned: nA + n_ops).
int orc_orset_apply_ops(const Rec* A, uint64_t nA, const Rec* Rm, uint64_t nR, uint64_t n_ops, const uint32_t* set, const uint32_t* elem,
                        const uint8_t* op, const uint64_t* tag_lo, const uint64_t* tag_hi, uint8_t* result, Rec* out_a, uint64_t* n_out_a,
                        Rec* out_r, uint64_t* n_out_r) {
    std::map<uint32_t, ORSet> sets;
    build_sets(sets, A, nA, Rm, nR);
    for (uint64_t i = 0; i < n_ops; ++i) {
        ORSet& o = sets[set[i]];
        const Elem e = elem_of(elem[i]);
        if (op[i] == 1) result[i] = o.AddTag(e, Guid{tag_lo[i], tag_hi[i]}) ? 1 : 0;
        else if (op[i] == 2) result[i] = o.Remove(e) ? 1 : 0;
        else if (op[i] == 3) { o.Clear(); result[i] = 1; }
        else return -1;
    }
    std::vector<Rec> a, r;
    export_sets(sets, a, r);
    std::copy(a.begin(), a.end(), out_a); *n_out_a = a.size();
    std::copy(r.begin(), r.end(), out_r); *n_out_r = r.size();
    return 0;
}

// ORSet.LookupAll() of one set, in the reference's order (the state is built from canonical
// records, so insertion order = ascending elem id).  Returns the count; out needs room for it.
int64_t orc_orset_lookup_all(const Rec* A, uint64_t nA, const Rec* Rm, uint64_t nR, uint32_t set, uint32_t* out, uint64_t cap) {
    std::map<uint32_t, ORSet> sets;
    build_sets(sets, A, nA, Rm, nR);
    auto it = sets.find(set);
    if (it == sets.end()) return 0;
    auto v = it->second.LookupAll();
    if (v.size() > cap) return -1;
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i] ? elem_id(*v[i]) : kNullElem;
    return (int64_t)v.size();
}

// ---- CPU baseline (bench.py cpu_baseline, kind "port") --------------------------------------
constexpr int kWarmups = 3;  // untimed passes before the timed ones (3 warm-ups, median of >= 10)

// PNCounter.Merge over pre-decoded messages for keys [0, n_keys) of the synthetic C2 workload,
// with `threads` workers splitting the keys (1 = the reference's serialized apply task,
// SafeCRDTManager.cs:115-117).  Returns the median seconds of `reps` passes; one pass merges
// n_keys x R cells (P and N).
double orc_bench_pnc_merge(uint64_t n_keys, uint32_t R, uint64_t seed, int threads, int reps) {
    std::vector<PNCounter<int64_t>> local;
    std::vector<PNCounterMsg<int64_t>> msgs;
    local.reserve(n_keys); msgs.reserve(n_keys);
    std::vector<int64_t> a_p(R), a_n(R), b_p(R), b_n(R);
    for (uint64_t k = 0; k < n_keys; ++k) {
        orc_synth_pnc_rows(seed, 0, k, 1, R, 8, a_p.data());
        orc_synth_pnc_rows(seed, 1, k, 1, R, 8, a_n.data());
        orc_synth_pnc_rows(seed, 2, k, 1, R, 8, b_p.data());
        orc_synth_pnc_rows(seed, 3, k, 1, R, 8, b_n.data());
        local.emplace_back(Guid{k + 1, 0});
        local.back().mutP().Clear(); local.back().mutN().Clear();
        for (uint32_t c = 0; c < R; ++c) local.back().mutP()[col_guid(k, c)] = a_p[c];
        for (uint32_t c = 0; c < R; ++c) local.back().mutN()[col_guid(k, c)] = a_n[c];
        msgs.push_back(row_msg<int64_t>(k, R, b_p.data(), b_n.data()));
    }
    if (threads < 1) threads = 1;
    std::vector<double> times;
    for (int rep = -kWarmups; rep < reps; ++rep) {  // 3 warm-ups, then the median of reps
        auto t0 = std::chrono::steady_clock::now();
        auto work = [&](uint64_t lo, uint64_t hi) { for (uint64_t k = lo; k < hi; ++k) local[k].Merge(msgs[k]); };
        if (threads == 1) work(0, n_keys);
        else {
            std::vector<std::thread> ts;
            for (int t = 0; t < threads; ++t) ts.emplace_back(work, n_keys * t / threads, n_keys * (t + 1) / threads);
            for (auto& t : ts) t.join();
        }
        if (rep >= 0) times.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return median_of(times);
}

// ORSet.Merge per set over the synthetic C3 shape for sets [0, n_sets): local adds u in
// [0,a), received adds u in [a-ov, 2a-ov), tombstones likewise with (t, tov).  Returns the median
// seconds of `reps` passes; one pass consumes n_sets*E*(2a+2t) records.  The local objects are
// re-copied (untimed) before every pass so each pass is a first merge.
double orc_bench_orset_merge(uint64_t n_sets, uint32_t E, uint32_t a, uint32_t ov, uint32_t t, uint32_t tov, uint64_t seed, int threads, int reps) {
    const uint64_t G = n_sets * E;
    std::vector<Rec> la(G * a), lr(G * t), ra(G * a), rr(G * t);
    orc_synth_orset(seed, 0, G * a, E, a, 0, la.data());
    orc_synth_orset(seed, 0, G * t, E, t, 0, lr.data());
    orc_synth_orset(seed, 0, G * a, E, a, a - ov, ra.data());
    orc_synth_orset(seed, 0, G * t, E, t, t - tov, rr.data());
    std::map<uint32_t, ORSet> lmap, rmap;
    build_sets(lmap, la.data(), la.size(), lr.data(), lr.size());
    build_sets(rmap, ra.data(), ra.size(), rr.data(), rr.size());
    std::vector<ORSet> base; std::vector<ORSetMsg> msgs;
    for (auto& kv : lmap) base.push_back(kv.second);
    for (auto& kv : rmap) msgs.push_back(kv.second.GetLastSynchronizedUpdate());
    if (threads < 1) threads = 1;
    std::vector<double> times;
    for (int rep = -kWarmups; rep < reps; ++rep) {
        std::vector<ORSet> local = base;
        auto t0 = std::chrono::steady_clock::now();
        auto work = [&](size_t lo, size_t hi) { for (size_t s = lo; s < hi; ++s) local[s].Merge(msgs[s]); };
        if (threads == 1) work(0, local.size());
        else {
            std::vector<std::thread> ts;
            for (int th = 0; th < threads; ++th) ts.emplace_back(work, local.size() * th / threads, local.size() * (th + 1) / threads);
            for (auto& x : ts) x.join();
        }
        if (rep >= 0) times.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return median_of(times);
}

// ---- state-message wire codec (oracle/json.hpp) ------------------------------
// Encode one PNCounterMsg whose pVector and nVector hold the n Guids (lo[i], hi[i]) in order with
// values pv[i] / nv[i] (int64 storage; eb = 4 or 8 is the C# width).  Returns the length, or -1 if
// cap is too small.
int64_t orc_json_encode_pnc(uint64_t n, const uint64_t* lo, const uint64_t* hi, const int64_t* pv, const int64_t* nv, uint32_t eb,
                            char* out, uint64_t cap) {
    std::string s;
    if (eb == 4) {
        PNCounterMsg<int32_t> m;
        for (uint64_t i = 0; i < n; ++i) { m.pVector[Guid{lo[i], hi[i]}] = (int32_t)pv[i]; m.nVector[Guid{lo[i], hi[i]}] = (int32_t)nv[i]; }
        s = json::EncodePNC(m);
    } else {
        PNCounterMsg<int64_t> m;
        for (uint64_t i = 0; i < n; ++i) { m.pVector[Guid{lo[i], hi[i]}] = pv[i]; m.nVector[Guid{lo[i], hi[i]}] = nv[i]; }
        s = json::EncodePNC(m);
    }
    if (s.size() > cap) return -1;
    std::memcpy(out, s.data(), s.size());
    return (int64_t)s.size();
}

// ORSetMsg<string>.Decode (ORSet.cs:56-63) of one payload, flattened for tests in ORSet.Merge's walk
// order (ORSet.cs:255-282): addSet entries in Dictionary order, removeSet entries, then the null add and
// null remove sets, each as [u8 side][u8 is_null][u32 name_len][name bytes][u32 n_tags][n_tags x (u64 lo,
// u64 hi)].  Returns the bytes written (or needed, if cap is short: nothing is written), -1 if Decode
// throws (JsonException).
int64_t orc_json_decode_orset(const char* bytes, uint64_t len, uint8_t* out, uint64_t cap) {
    ORSetMsg m;
    try {
        m = json::DecodeORSet(std::string_view(bytes, len));
    } catch (const json::JsonException&) {
        return -1;
    }
    std::string o;
    auto u32 = [&](uint32_t v) { o.append(reinterpret_cast<const char*>(&v), 4); };
    auto entry = [&](uint8_t side, uint8_t is_null, const std::string& name, const GuidSet& tags) {
        o.push_back((char)side);
        o.push_back((char)is_null);
        u32((uint32_t)name.size());
        o += name;
        u32((uint32_t)tags.size());
        for (const Guid& g : tags) {
            o.append(reinterpret_cast<const char*>(&g.lo), 8);
            o.append(reinterpret_cast<const char*>(&g.hi), 8);
        }
    };
    for (const auto& kv : m.addSet) entry(0, 0, kv.first, kv.second);
    for (const auto& kv : m.removeSet) entry(1, 0, kv.first, kv.second);
    entry(0, 1, std::string(), m.nullAddGuid);
    entry(1, 1, std::string(), m.nullRemoveGuid);
    if (o.size() <= cap) std::memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

// 1 if the payload is accepted by PNCounterMsg.Decode at width eb (the wire contract), else 0.
int orc_json_accepts_pnc(const char* bytes, uint64_t len, uint32_t eb) {
    try {
        if (eb == 4) json::DecodePNC<int32_t>(std::string_view(bytes, len));
        else json::DecodePNC<int64_t>(std::string_view(bytes, len));
        return 1;
    } catch (const json::JsonException&) {
        return 0;
    }
}

// The stable-apply loop over encoded states (SafeCRDT.ApplyUpdateStable -> Decode -> Merge, in
// commit order, SafeCRDTManager.cs:122-146) on a dense store with a replica table: row k holds the
// Guids cols[k*R + c] (c < ncols[k]) with values P/N[k*R + c], i.e. a PNCounter whose P and N
// dictionaries enumerate those Guids in column order.  Messages are applied in order until the first
// one Decode rejects (the reference's loop stops at the throwing message): *bad = its index, or
// UINT64_MAX.  The touched rows are written back (P, N, cols, ncols; columns = P's enumeration order).
// Returns 0, or -2 if a row would hold more than R replicas (the engine's capacity limit, not a
// reference behaviour) — *bad is then that message.
}  // extern "C"

namespace {
template <class T>
int json_apply(uint64_t n_keys, uint32_t R, T* P, T* N, uint64_t* cols, uint32_t* ncols, uint64_t n, const uint32_t* key_idx,
               const uint64_t* off, const char* bytes, uint64_t* bad) {
    std::unordered_map<uint64_t, PNCounter<T>> live;
    *bad = UINT64_MAX;
    auto obj = [&](uint64_t k) -> PNCounter<T>& {
        auto it = live.find(k);
        if (it != live.end()) return it->second;
        it = live.emplace(k, PNCounter<T>(Guid{~0ull, ~0ull})).first;
        it->second.mutP().Clear(); it->second.mutN().Clear();
        for (uint32_t c = 0; c < ncols[k]; ++c) {
            const Guid g{cols[2 * (k * R + c)], cols[2 * (k * R + c) + 1]};
            it->second.mutP()[g] = P[k * R + c];
            it->second.mutN()[g] = N[k * R + c];
        }
        return it->second;
    };
    int rc = 0;
    for (uint64_t m = 0; m < n; ++m) {
        const uint64_t k = key_idx[m];
        if (k >= n_keys) return -1;
        PNCounterMsg<T> msg;
        try {
            msg = json::DecodePNC<T>(std::string_view(bytes + off[m], off[m + 1] - off[m]));
        } catch (const json::JsonException&) {
            *bad = m;
            break;
        }
        PNCounter<T>& pc = obj(k);
        pc.ApplySynchronizedUpdate(msg);
        if (pc.P().size() > R || pc.N().size() > R) { *bad = m; rc = -2; break; }
    }
    for (auto& kv : live) {
        const uint64_t k = kv.first;
        uint32_t c = 0;
        for (const auto& e : kv.second.P()) {
            if (c >= R) break;
            cols[2 * (k * R + c)] = e.first.lo;
            cols[2 * (k * R + c) + 1] = e.first.hi;
            P[k * R + c] = e.second;
            T v = 0;
            kv.second.N().TryGetValue(e.first, v);
            N[k * R + c] = v;
            ++c;
        }
        ncols[k] = c;
    }
    return rc;
}
}  // namespace

extern "C" {

int orc_pnc_apply_json(uint64_t n_keys, uint32_t R, uint32_t eb, void* P, void* N, uint64_t* cols, uint32_t* ncols, uint64_t n,
                       const uint32_t* key_idx, const uint64_t* off, const char* bytes, uint64_t* bad) {
    if (eb == 4) return json_apply<int32_t>(n_keys, R, (int32_t*)P, (int32_t*)N, cols, ncols, n, key_idx, off, bytes, bad);
    return json_apply<int64_t>(n_keys, R, (int64_t*)P, (int64_t*)N, cols, ncols, n, key_idx, off, bytes, bad);
}

}  // extern "C"

// ---- UpdateMessage.ComputeDigest (digest.hpp; DAGUpdateMessage.cs:32-55) -----------------------
#include "digest.hpp"

extern "C" {

// SHA256 of n payloads: payload i = bytes[off[i], off[i+1]); out = n * 32 bytes.
void orc_sha256_batch(uint64_t n, const uint64_t* off, const uint8_t* bytes, uint8_t* out) {
    for (uint64_t i = 0; i < n; ++i) sha256(bytes + off[i], off[i + 1] - off[i], out + 32 * i);
}

// n_updates UpdateMessages over n payloads (update u = payloads [first[u], first[u+1])); is_null may be
// NULL; msg_digest (n * 32, optional) and digest (n_updates * 32).
void orc_update_digests(uint64_t n, const uint64_t* off, const uint8_t* bytes, const uint8_t* is_null, uint64_t n_updates,
                        const uint64_t* first, uint8_t* msg_digest, uint8_t* digest) {
    std::vector<const uint8_t*> ptr(n);
    std::vector<uint64_t> len(n);
    for (uint64_t i = 0; i < n; ++i) { ptr[i] = bytes + off[i]; len[i] = off[i + 1] - off[i]; }
    for (uint64_t u = 0; u < n_updates; ++u) {
        uint64_t a = first[u], c = first[u + 1] - a;
        update_digest(c, ptr.data() + a, len.data() + a, is_null ? is_null + a : nullptr, digest + 32 * u,
                      msg_digest ? msg_digest + 32 * a : nullptr);
    }
}

// CPU baseline: seconds for orc_update_digests over the same inputs (median of reps, 1 thread).
double orc_bench_update_digests(uint64_t n, const uint64_t* off, const uint8_t* bytes, uint64_t n_updates, const uint64_t* first, int reps) {
    std::vector<uint8_t> out(32 * (n_updates ? n_updates : 1));
    std::vector<double> t;
    for (int r = -kWarmups; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        orc_update_digests(n, off, bytes, nullptr, n_updates, first, nullptr, out.data());
        if (r >= 0) t.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return median_of(t);
}

}  // extern "C"
