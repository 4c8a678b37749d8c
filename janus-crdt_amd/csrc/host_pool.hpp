// host_pool.hpp — the library's host workers (csrc/node.hip): the committed-wave gather of payloads into
// pinned staging runs here, on the caller's thread plus host_threads() - 1 persistent workers.
#pragma once

#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace jg {

// Workers: JANUS_HOST_THREADS, else min(16, hardware threads, the cgroup CPU quota).  A process over its
// cgroup quota (cpu.max "quota period": the GPU box grants 16 CPUs of time on a 256-CPU host) is
// throttled as a whole, so the pool never asks for more CPUs than the quota holds.
inline int host_threads() {
    if (const char* e = std::getenv("JANUS_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return v;
    }
    unsigned cap = std::thread::hardware_concurrency();
    cap = std::min(cap ? cap : 1u, 16u);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (std::fscanf(f, "%31s %llu", q, &period) == 2 && std::strcmp(q, "max") != 0 && period) {
            const unsigned long long cpus = std::strtoull(q, nullptr, 10) / period;
            if (cpus >= 1) cap = std::min<unsigned>(cap, (unsigned)cpus);
        }
        std::fclose(f);
    }
    return (int)std::max(1u, cap);
}

// Persistent workers (creating threads per phase cost ~0.3 ms a phase).  run(fn) calls fn(t) for every
// worker t in [0, n), t = 0 on the caller, and returns when all are done.
class WorkerPool {
  public:
    explicit WorkerPool(int n) : n_(n) {
        for (int t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    WorkerPool(const WorkerPool&) = delete;
    WorkerPool& operator=(const WorkerPool&) = delete;
    int size() const { return n_; }
    void run(const std::function<void(int)>& fn) {
        if (n_ == 1) { fn(0); return; }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            pending_ = n_ - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
                job = job_;
            }
            (*job)(t);
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

// Tasks q in [0, ntask) dealt from a shared counter over the pool (a static split made every phase wait
// for its slowest worker on a shared host); inline when `par` is false.
template <class F> void deal(WorkerPool& pool, bool par, size_t ntask, F&& fn) {
    std::atomic<size_t> next{0};
    auto body = [&](int t) {
        for (size_t q; (q = next.fetch_add(1, std::memory_order_relaxed)) < ntask;) fn(q, t);
    };
    if (par && pool.size() > 1 && ntask > 1) pool.run(body);
    else body(0);
}

// One task's contiguous output range in pinned staging, written with non-temporal stores in whole 64-B
// lines: the staging is read once by the H2D copy engine, so a line written through the cache would cost
// a read for ownership first.  The range's first and last partial lines (shared with the neighbouring
// tasks' ranges) use ordinary stores.
class LineStream {
  public:
    LineStream(char* base, size_t pos) : base_(base), pos_(pos) {}
    void put(const char* src, size_t n) {
        if (head_) {  // up to the range's first line boundary: ordinary stores
            const size_t c = std::min(n, (64 - (pos_ & 63)) & 63);
            std::memcpy(base_ + pos_, src, c);
            pos_ += c, src += c, n -= c;
            if ((pos_ & 63) == 0) head_ = false;
            if (head_ || n == 0) return;
        }
        if (fill_) {
            const size_t c = std::min(n, 64 - fill_);
            std::memcpy(line_ + fill_, src, c);
            fill_ += c, pos_ += c, src += c, n -= c;
            if (fill_ < 64) return;
            stream(base_ + pos_ - 64, line_);
            fill_ = 0;
        }
        for (; n >= 64; pos_ += 64, src += 64, n -= 64) stream(base_ + pos_, src);
        std::memcpy(line_, src, n);
        fill_ = n, pos_ += n;
    }
    void finish() {  // the range's last partial line, then order the streamed lines before the join
        if (fill_) std::memcpy(base_ + pos_ - fill_, line_, fill_);
        _mm_sfence();
    }

  private:
    static void stream(char* dst, const char* src) {
        for (int k = 0; k < 4; ++k)
            _mm_stream_si128(reinterpret_cast<__m128i*>(dst) + k, _mm_loadu_si128(reinterpret_cast<const __m128i*>(src) + k));
    }
    char* base_;
    size_t pos_;
    bool head_ = true;
    size_t fill_ = 0;
    alignas(64) char line_[64];
};

}  // namespace jg
