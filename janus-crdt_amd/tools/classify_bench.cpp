// classify_bench.cpp — dev tool (CPU only): the apply loop's classify pass (uid lookup + safe-update
// claim per message, GpuStableStore::apply_msgs) on a C5-shaped wave, to see where its ~100 ns per
// message per worker goes.  Same data structures as host/janus_host.hpp (restated here: they are
// private there).  Build: g++ -O3 -std=c++17 -pthread classify_bench.cpp -o classify_bench
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

struct Guid { uint64_t lo, hi; bool operator==(const Guid& o) const { return lo == o.lo && hi == o.hi; } };
static size_t ghash(const Guid& g) {
    uint64_t x = g.lo ^ (g.hi * 0x9E3779B97F4A7C15ull);
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
    return (size_t)x;
}
struct NP { Guid uid; int type = 1; uint64_t seq = 0; std::string message; };
struct alignas(32) USlot { Guid key; uint32_t type = 0, idx = 0; uint8_t used = 0; };
struct TSlot { std::atomic<uint64_t> key{0}; uint64_t val = 0; };
static size_t sslot(uint64_t x) { x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; return (size_t)x; }

template <class T> T* big(size_t n, bool huge) {
    void* p = nullptr;
    const size_t bytes = (n * sizeof(T) + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
    if (posix_memalign(&p, 2u << 20, bytes)) std::abort();
    if (huge) madvise(p, bytes, MADV_HUGEPAGE);
    std::memset(p, 0, bytes);
    return static_cast<T*>(p);
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 8;
    const bool huge = argc > 2 && std::atoi(argv[2]);
    const size_t accounts = 1000000, n = 1000000;
    std::mt19937_64 rng(1);
    std::vector<Guid> uid(accounts);
    for (auto& g : uid) g = Guid{rng(), rng()};
    const size_t us = 1u << 21, ts = 1u << 21;  // load <= 0.5 / 0.25 like the product tables
    USlot* ut = big<USlot>(us, huge);
    TSlot* tt = big<TSlot>(ts, huge);
    for (size_t k = 0; k < accounts; ++k)
        for (size_t i = ghash(uid[k]) & (us - 1);; i = (i + 1) & (us - 1))
            if (!ut[i].used) { ut[i].used = 1; ut[i].key = uid[k]; ut[i].idx = (uint32_t)k; break; }
    // the wave: 1000 UpdateMessages of 1000 NetworkProtocols (payload ~357 B), half of them safe
    std::vector<std::vector<NP>> blocks(1000);
    std::vector<const NP*> msgs;
    uint64_t seq = 1;
    for (auto& b : blocks) {
        b.resize(1000);
        for (auto& m : b) {
            m.uid = uid[rng() % accounts];
            m.seq = seq++;
            m.message.assign(340 + rng() % 36, 'x');
        }
    }
    for (auto& b : blocks) for (auto& m : b) msgs.push_back(&m);
    std::vector<uint32_t> cls(n);
    auto fill_tracker = [&] {
        for (size_t i = 0; i < ts; ++i) tt[i].key.store(0, std::memory_order_relaxed);
        for (const NP* m : msgs)
            if (m->seq & 1)
                for (size_t i = sslot(m->seq) & (ts - 1);; i = (i + 1) & (ts - 1))
                    if (!tt[i].key.load(std::memory_order_relaxed)) { tt[i].key.store(m->seq); tt[i].val = m->seq * 3; break; }
    };
    auto find = [&](const Guid& g) -> const USlot* {
        for (size_t i = ghash(g) & (us - 1);; i = (i + 1) & (us - 1)) {
            if (!ut[i].used) return nullptr;
            if (ut[i].key == g) return &ut[i];
        }
    };
    auto claim = [&](uint64_t s, uint64_t* o) -> bool {
        for (size_t i = sslot(s) & (ts - 1);; i = (i + 1) & (ts - 1)) {
            uint64_t k = tt[i].key.load(std::memory_order_acquire);
            if (k == 0) return false;
            if (k != s) continue;
            const uint64_t v = tt[i].val;
            if (!tt[i].key.compare_exchange_strong(k, ~0ull, std::memory_order_acq_rel)) return false;
            *o = v;
            return true;
        }
    };
    // mode bits: 1 uid lookup, 2 claim, 4 prefetch; pf = distance
    auto run = [&](int mode, size_t pf, bool relaxed_claim) {
        fill_tracker();
        std::atomic<uint64_t> claimed{0};
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                const size_t b = n * t / T, e = n * (t + 1) / T;
                uint64_t c = 0;
                for (size_t i = b; i < e; ++i) {
                    if (mode & 4) {
                        if (i + 2 * pf < e) __builtin_prefetch(msgs[i + 2 * pf]);
                        if (i + pf < e) {
                            if (mode & 1) __builtin_prefetch(&ut[ghash(msgs[i + pf]->uid) & (us - 1)]);
                            if (mode & 2) __builtin_prefetch(&tt[sslot(msgs[i + pf]->seq) & (ts - 1)], 1);
                        }
                    }
                    const NP& m = *msgs[i];
                    uint32_t cl = (uint32_t)m.message.size();
                    if (mode & 1) { const USlot* s = find(m.uid); cl = s ? s->idx : ~0u; }
                    cls[i] = cl;
                    uint64_t o;
                    if (mode & 2) {
                        if (relaxed_claim) {  // load + plain store instead of the CAS (single-owner sweep)
                            for (size_t j = sslot(m.seq) & (ts - 1);; j = (j + 1) & (ts - 1)) {
                                const uint64_t k = tt[j].key.load(std::memory_order_relaxed);
                                if (k == 0) break;
                                if (k != m.seq) continue;
                                o = tt[j].val;
                                tt[j].key.store(~0ull, std::memory_order_relaxed);
                                c += o != 0;
                                break;
                            }
                        } else if (claim(m.seq, &o)) ++c;
                    }
                }
                claimed += c;
            });
        for (auto& x : th) x.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return std::make_pair(s, claimed.load());
    };
    // classify (uid + claim, pf 8) then gather into one staging buffer (the product's two passes), vs one
    // pass that classifies and copies each payload into a per-worker buffer, then a streaming copy of the
    // per-worker buffers into the staging buffer at their prefix offsets
    std::vector<char> stage(400u << 20);
    std::vector<std::vector<char>> priv(T, std::vector<char>(64u << 20));
    auto gather = [&](bool fused) {
        fill_tracker();
        std::vector<size_t> bytes(T + 1, 0);
        const auto t0 = std::chrono::steady_clock::now();
        auto pass1 = [&](int t) {
            const size_t b = n * t / T, e = n * (t + 1) / T;
            size_t o = 0;
            for (size_t i = b; i < e; ++i) {
                if (i + 16 < e) __builtin_prefetch(msgs[i + 16]);
                if (i + 8 < e) {
                    __builtin_prefetch(&ut[ghash(msgs[i + 8]->uid) & (us - 1)]);
                    __builtin_prefetch(&tt[sslot(msgs[i + 8]->seq) & (ts - 1)], 1);
                    if (fused) __builtin_prefetch(msgs[i + 8]->message.data());
                }
                const NP& m = *msgs[i];
                const USlot* sl = find(m.uid);
                cls[i] = sl ? sl->idx : ~0u;
                uint64_t og;
                claim(m.seq, &og);
                if (fused) { std::memcpy(priv[t].data() + o, m.message.data(), m.message.size()); }
                o += m.message.size();
            }
            bytes[t + 1] = o;
        };
        auto pass2 = [&](int t) {
            size_t at = 0;
            for (int u = 0; u < t; ++u) at += bytes[u + 1];
            if (fused) { std::memcpy(stage.data() + at, priv[t].data(), bytes[t + 1]); return; }
            const size_t b = n * t / T, e = n * (t + 1) / T;
            for (size_t i = b; i < e; ++i) {
                if (i + 8 < e) __builtin_prefetch(msgs[i + 8]->message.data());
                const std::string& p = msgs[i]->message;
                std::memcpy(stage.data() + at, p.data(), p.size());
                at += p.size();
            }
        };
        double t1s = 0;
        for (int ph = 0; ph < 2; ++ph) {
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back([&, t, ph] { ph == 0 ? pass1(t) : pass2(t); });
            for (auto& x : th) x.join();
            if (ph == 0) t1s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%-30s %7.2f ms (pass 1 %.2f, pass 2 %.2f)\n", fused ? "fused classify+gather" : "classify, then gather", s * 1e3, t1s * 1e3,
                    (s - t1s) * 1e3);
    };
    for (int rep = 0; rep < 3; ++rep) { gather(false); gather(true); }
    if (argc > 3) return 0;
    struct V { const char* name; int mode; size_t pf; bool relaxed; };
    const V vs[] = {{"read NP only", 0, 8, false},        {"uid, no prefetch", 1, 8, false},    {"uid, pf 8", 5, 8, false},
                    {"uid+claim, no prefetch", 3, 8, false}, {"uid+claim, pf 8 (product)", 7, 8, false},
                    {"uid+claim, pf 16", 7, 16, false},   {"uid+claim, pf 4", 7, 4, false},    {"uid+claim pf 8, plain store", 7, 8, true},
                    {"claim only, pf 8", 6, 8, false}};
    std::printf("T=%d huge=%d\n", T, (int)huge);
    for (int rep = 0; rep < 2; ++rep)
        for (const V& v : vs) {
            const auto r = run(v.mode, v.pf, v.relaxed);
            std::printf("%-30s %7.2f ms  %6.1f ns/msg/thread  claimed %llu\n", v.name, r.first * 1e3, r.first * 1e9 * T / n,
                        (unsigned long long)r.second);
        }
    return 0;
}
