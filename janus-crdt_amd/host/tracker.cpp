// tracker.cpp — SafeUpdateTracker and the huge-page table storage (see janus_host.hpp).  Plain C++,
// no engine calls: also linked by the CPU unit test (host/test_tracker.cpp).
#include <sys/mman.h>

#include <cstdlib>
#include <new>

#include "janus_host.hpp"

namespace janus {

void* table_alloc(size_t bytes) {
    if (bytes < TableAlloc<char>::kHuge) return ::operator new(bytes, std::align_val_t(64));
    const size_t b = (bytes + TableAlloc<char>::kHuge - 1) & ~(TableAlloc<char>::kHuge - 1);
    void* p = std::aligned_alloc(TableAlloc<char>::kHuge, b);
    if (!p) throw std::bad_alloc();
    (void)madvise(p, b, MADV_HUGEPAGE);  // advisory: without THP support the table works the same
    return p;
}
void table_free(void* p, size_t bytes) {
    if (bytes < TableAlloc<char>::kHuge) ::operator delete(p, std::align_val_t(64));
    else std::free(p);
}

bool SafeUpdateTracker::add(uint64_t seq, uint64_t origin) {
    if (seq == 0 || seq == kTomb || contains(seq)) return false;
    if (ring_.empty()) {
        std::vector<Slot, TableAlloc<Slot>> fresh(kRing0);
        ring_.swap(fresh);
    }
    Slot& r = ring_[seq & (ring_.size() - 1)];
    if (r.key.load(std::memory_order_relaxed) == 0) {
        r.val = origin;
        r.key.store(seq, std::memory_order_release);
        n_.fetch_add(1, std::memory_order_relaxed);
        return true;
    }
    table_add(seq, origin);  // the ring slot holds another live seq
    if (++spill_ > ring_.size() / 16) grow_ring();
    return true;
}

bool SafeUpdateTracker::contains(uint64_t seq) const {
    if (seq == 0 || seq == kTomb) return false;
    if (!ring_.empty() && ring_[seq & (ring_.size() - 1)].key.load(std::memory_order_acquire) == seq) return true;
    return table_contains(seq);
}

bool SafeUpdateTracker::claim(uint64_t seq, uint64_t* origin) {
    if (seq == 0 || seq == kTomb) return false;
    if (!ring_.empty()) {
        Slot& r = ring_[seq & (ring_.size() - 1)];
        uint64_t k = r.key.load(std::memory_order_acquire);
        if (k == seq) {
            const uint64_t v = r.val;
            if (!r.key.compare_exchange_strong(k, 0, std::memory_order_acq_rel)) return false;  // another take won
            if (origin) *origin = v;
            return true;
        }
    }
    return used_ ? table_claim(seq, origin) : false;
}

bool SafeUpdateTracker::table_add(uint64_t seq, uint64_t origin) {
    if ((used_ + 1) * 2 > slots_.size()) grow();
    const size_t mask = slots_.size() - 1;
    for (size_t i = seq_slot(seq) & mask;; i = (i + 1) & mask) {
        const uint64_t k = slots_[i].key.load(std::memory_order_relaxed);
        if (k == seq) return false;
        if (k == 0) {
            slots_[i].val = origin;
            slots_[i].key.store(seq, std::memory_order_release);
            ++used_;
            n_.fetch_add(1, std::memory_order_relaxed);
            return true;
        }
    }
}

bool SafeUpdateTracker::table_contains(uint64_t seq) const {
    if (slots_.empty()) return false;
    const size_t mask = slots_.size() - 1;
    for (size_t i = seq_slot(seq) & mask;; i = (i + 1) & mask) {
        const uint64_t k = slots_[i].key.load(std::memory_order_acquire);
        if (k == seq) return true;
        if (k == 0) return false;
    }
}

bool SafeUpdateTracker::table_claim(uint64_t seq, uint64_t* origin) {
    if (slots_.empty()) return false;
    const size_t mask = slots_.size() - 1;
    for (size_t i = seq_slot(seq) & mask;; i = (i + 1) & mask) {
        uint64_t k = slots_[i].key.load(std::memory_order_acquire);
        if (k == 0) return false;
        if (k != seq) continue;
        const uint64_t v = slots_[i].val;
        if (!slots_[i].key.compare_exchange_strong(k, kTomb, std::memory_order_acq_rel)) return false;  // another take won
        if (origin) *origin = v;
        return true;
    }
}

std::vector<std::pair<uint64_t, uint64_t>> SafeUpdateTracker::items() const {
    std::vector<std::pair<uint64_t, uint64_t>> out;
    for (const Slot& s : ring_) {
        const uint64_t k = s.key.load(std::memory_order_acquire);
        if (k != 0) out.emplace_back(k, s.val);
    }
    for (const Slot& s : slots_) {
        const uint64_t k = s.key.load(std::memory_order_acquire);
        if (k != 0 && k != kTomb) out.emplace_back(k, s.val);
    }
    return out;
}

void SafeUpdateTracker::grow() {  // rehash the table's live entries (tombstones dropped), single-threaded
    std::vector<std::pair<uint64_t, uint64_t>> live;
    for (const Slot& s : slots_) {
        const uint64_t k = s.key.load(std::memory_order_acquire);
        if (k != 0 && k != kTomb) live.emplace_back(k, s.val);
    }
    size_t cap = 1024;
    while (cap < 4 * (live.size() + 1)) cap <<= 1;
    std::vector<Slot, TableAlloc<Slot>> fresh(cap);
    slots_.swap(fresh);
    used_ = 0;
    n_.fetch_sub(live.size(), std::memory_order_relaxed);  // table_add counts them again
    for (const auto& kv : live) table_add(kv.first, kv.second);
}

void SafeUpdateTracker::grow_ring() {  // twice the ring; every live entry placed again, single-threaded
    const std::vector<std::pair<uint64_t, uint64_t>> live = items();
    const size_t pending = n_.load(std::memory_order_relaxed) - live.size();  // claimed, not settled yet
    const size_t cap = ring_.size() * 2;
    clear();
    n_.store(pending, std::memory_order_relaxed);
    std::vector<Slot, TableAlloc<Slot>> fresh(cap);
    ring_.swap(fresh);
    for (const auto& kv : live) {
        Slot& r = ring_[kv.first & (cap - 1)];
        if (r.key.load(std::memory_order_relaxed) == 0) {
            r.val = kv.second;
            r.key.store(kv.first, std::memory_order_relaxed);
            n_.fetch_add(1, std::memory_order_relaxed);
        } else {
            table_add(kv.first, kv.second);
            ++spill_;
        }
    }
}

}  // namespace janus
