// stage_bw.cpp — host gather bandwidth into pinned staging, by allocation flavour (tuning tool).
// Gathers 1M scattered ~357-byte strings (the C5 wave's payloads) into one staging buffer with T threads,
// then times the H2D of the buffer.  Build: hipcc -O3 -std=c++17 stage_bw.cpp -o stage_bw -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 16;
    const size_t n = 1000000;
    std::mt19937_64 rng(1);
    std::vector<std::string> msgs(n);
    size_t total = 0;
    for (auto& m : msgs) {
        m.assign(340 + rng() % 36, 'x');
        total += m.size();
    }
    std::vector<size_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + msgs[i].size();
    void* dev = nullptr;
    if (hipMalloc(&dev, total) != hipSuccess) return 1;
    hipStream_t st;
    (void)hipStreamCreate(&st);
    struct Kind { const char* name; unsigned flags; int mode; };  // mode 0 hipHostMalloc, 1 malloc+register, 2 plain malloc
    Kind kinds[] = {{"hipHostMallocDefault", hipHostMallocDefault, 0},
                    {"hipHostMallocNonCoherent", hipHostMallocNonCoherent, 0},
                    {"hipHostMallocCoherent", hipHostMallocCoherent, 0},
                    {"hipHostMallocWriteCombined", hipHostMallocWriteCombined, 0},
                    {"malloc+hipHostRegister", 0, 1},
                    {"malloc (pageable)", 0, 2}};
    for (const Kind& k : kinds) {
        char* buf = nullptr;
        if (k.mode == 0) { if (hipHostMalloc((void**)&buf, total, k.flags) != hipSuccess) { std::printf("%s: alloc failed\n", k.name); continue; } }
        else {
            buf = static_cast<char*>(std::aligned_alloc(4096, (total + 4095) & ~size_t(4095)));
            std::memset(buf, 0, total);
            if (k.mode == 1 && hipHostRegister(buf, total, hipHostRegisterDefault) != hipSuccess) { std::printf("%s: register failed\n", k.name); continue; }
        }
        double best_g = 1e9, best_h = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            const double t0 = now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    const size_t b = n * t / T, e = n * (t + 1) / T;
                    for (size_t i = b; i < e; ++i) std::memcpy(buf + off[i], msgs[i].data(), msgs[i].size());
                });
            for (auto& x : th) x.join();
            const double t1 = now();
            (void)hipMemcpyAsync(dev, buf, total, hipMemcpyHostToDevice, st);
            (void)hipStreamSynchronize(st);
            const double t2 = now();
            best_g = std::min(best_g, t1 - t0);
            best_h = std::min(best_h, t2 - t1);
        }
        std::printf("%-28s gather %6.2f ms = %6.1f GB/s   H2D %6.2f ms = %6.1f GB/s   (%d threads, %.0f MB)\n", k.name, best_g * 1e3,
                    total / best_g / 1e9, best_h * 1e3, total / best_h / 1e9, T, total / 1e6);
        if (k.mode == 0) (void)hipHostFree(buf);
        else { if (k.mode == 1) (void)hipHostUnregister(buf); std::free(buf); }
    }
    return 0;
}
