// test_tracker.cpp — CPU unit test of janus::SafeUpdateTracker (host/tracker.cpp), the safe-update
// notification map of SafeCRDTManager (SafeCRDTManager.cs:33, TryAdd / ContainsKey / TryRemove), checked
// against std::unordered_map: ring hits, seqs whose ring slot is taken (table), ring growth, table
// growth, copies, and concurrent takes (every tracked seq claimed exactly once, duplicates included).
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

#include "janus_host.hpp"

namespace {
std::atomic<int> fails{0};
void check(bool ok, const char* what) {
    if (!ok) {
        std::printf("FAIL %s\n", what);
        ++fails;
    }
}

bool same(const janus::SafeUpdateTracker& t, const std::unordered_map<uint64_t, uint64_t>& m) {
    auto it = t.items();
    if (it.size() != m.size()) return false;
    for (const auto& [k, v] : it) {
        auto f = m.find(k);
        if (f == m.end() || f->second != v) return false;
    }
    return true;
}
}  // namespace

int main() {
    constexpr uint64_t kRing = uint64_t(1) << 20;  // SafeUpdateTracker's first ring size
    {   // sequential seqs, random removals, reference map
        janus::SafeUpdateTracker t;
        std::unordered_map<uint64_t, uint64_t> m;
        std::mt19937_64 rng(7);
        check(!t.add(0, 1), "seq 0 is not a message");
        for (uint64_t s = 1; s <= 200000; ++s) {
            if (rng() % 2) {
                check(t.add(s, s * 3 + 1), "add new");
                m[s] = s * 3 + 1;
            }
        }
        const bool had2 = m.count(2) == 1;
        check(t.add(2, 9) != had2, "add of a present seq fails, of an absent one succeeds");
        if (!had2) m[2] = 9;
        for (uint64_t s = 1; s <= 200000; s += 3) {
            uint64_t o = 0;
            const bool took = t.take(s, &o);
            check(took == (m.count(s) == 1), "take matches the map");
            if (took) check(o == m[s], "take returns the origin"), m.erase(s);
            check(!t.contains(s), "taken seq is gone");
        }
        check(same(t, m), "items after takes");
        check(t.size() == m.size(), "size after takes");
    }
    {   // seqs one ring apart share a slot: the second goes to the table; both found, both taken
        janus::SafeUpdateTracker t;
        check(t.add(5, 50) && t.add(5 + kRing, 51) && t.add(5 + 2 * kRing, 52), "colliding adds");
        check(t.contains(5) && t.contains(5 + kRing) && t.contains(5 + 2 * kRing), "colliding contains");
        check(!t.add(5 + kRing, 1), "colliding add present");
        uint64_t o = 0;
        check(t.take(5, &o) && o == 50, "take ring entry");
        check(!t.add(5 + kRing, 1), "table entry still present after its ring slot emptied");
        check(t.take(5 + kRing, &o) && o == 51, "take table entry");
        check(t.take(5 + 2 * kRing, &o) && o == 52, "take second table entry");
        check(t.size() == 0 && t.items().empty(), "empty after takes");
        check(t.add(5 + kRing, 7) && t.contains(5 + kRing), "re-add after take");
    }
    {   // a live span wider than the ring: the table fills, the ring doubles, nothing is lost
        janus::SafeUpdateTracker t;
        std::unordered_map<uint64_t, uint64_t> m;
        for (uint64_t s = 1; s <= 3 * kRing; s += 2) {
            t.add(s, s ^ 0x55);
            m[s] = s ^ 0x55;
        }
        check(same(t, m), "items after ring growth");
        check(t.size() == m.size(), "size after ring growth");
        size_t claimed = 0;
        for (uint64_t s = 1; s <= 3 * kRing; s += 4) {
            uint64_t o;
            if (t.claim(s, &o)) ++claimed, m.erase(s);
        }
        t.settle(claimed);
        check(same(t, m) && t.size() == m.size(), "claim + settle after growth");
        janus::SafeUpdateTracker c(t), d;
        d = t;
        check(same(c, m) && same(d, m), "copy and assignment");
    }
    {   // concurrent takes, every seq attempted by two threads: each claimed exactly once
        janus::SafeUpdateTracker t;
        constexpr uint64_t n = 400000;
        for (uint64_t s = 1; s <= n; ++s) t.add(s, s);
        std::vector<std::atomic<int>> hits(n + 1);
        for (auto& h : hits) h.store(0);
        std::vector<std::thread> th;
        for (int w = 0; w < 8; ++w)
            th.emplace_back([&, w] {
                for (uint64_t s = 1 + (w / 2); s <= n; s += 4) {  // workers 2k and 2k+1 race on the same seqs
                    uint64_t o;
                    if (t.claim(s, &o)) hits[s].fetch_add(1), check(o == s, "concurrent origin");
                }
            });
        for (auto& x : th) x.join();
        bool once = true;
        for (uint64_t s = 1; s <= n; ++s) once &= hits[s].load() == 1;
        check(once, "every seq claimed exactly once");
        check(t.items().empty(), "nothing left after the concurrent takes");
    }
    std::printf(fails ? "tracker: %d FAILED\n" : "tracker: all passed\n", fails.load());
    return fails ? 1 : 0;
}
