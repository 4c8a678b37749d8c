// tune_h2d.hip — dev tool: host -> device upload rate of the apply loop's chunk shape (48 MB from
// page-locked host memory into HBM), by engine: one hipMemcpyAsync per chunk on one stream, the chunk
// split over 2 / 4 streams, and a copy kernel reading the page-locked buffer directly (zero-copy, 16-B
// loads over the host link).  Run it with HSA_ENABLE_SDMA=0 too to see the blit-kernel path.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o build/tune_h2d tools/tune_h2d.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {  // four 16-B loads in flight per lane
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a; dst[i + stride] = b; dst[i + 2 * stride] = c; dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t chunk = 48ull << 20, n_chunks = 8, total = chunk * n_chunks;  // 384 MB per "wave"
    char* h;
    CK(hipHostMalloc(&h, total, hipHostMallocDefault));
    std::memset(h, 1, total);
    char* d;
    CK(hipMalloc(&d, total));
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int cus = 256;
    { hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0)); cus = p.multiProcessorCount; }
    auto run = [&](const char* name, int mode) {
        std::vector<double> t;
        for (int r = 0; r < 7; ++r) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            for (size_t c = 0; c < n_chunks; ++c) {
                char* dd = d + c * chunk;
                const char* hh = h + c * chunk;
                if (mode == 1) CK(hipMemcpyAsync(dd, hh, chunk, hipMemcpyHostToDevice, st[0]));
                else if (mode == 2 || mode == 4) {
                    const size_t part = chunk / mode;
                    for (int k = 0; k < mode; ++k) CK(hipMemcpyAsync(dd + k * part, hh + k * part, part, hipMemcpyHostToDevice, st[k]));
                } else if (mode == 10 || mode == 11 || mode == 12) {
                    const unsigned g = (unsigned)(mode == 10 ? cus : mode == 11 ? 2 * cus : 8 * cus);
                    hipLaunchKernelGGL(k_pull, dim3(g), dim3(256), 0, st[0], reinterpret_cast<const uint4*>(hh), reinterpret_cast<uint4*>(dd), chunk / 16);
                }
            }
            CK(hipDeviceSynchronize());
            t.push_back(now() - t0);
        }
        std::sort(t.begin(), t.end());
        std::printf("%-34s median %.3f ms = %.1f GB/s  (min %.3f ms)\n", name, t[3] * 1e3, total / t[3] / 1e9, t[0] * 1e3);
    };
    run("hipMemcpyAsync, 1 stream", 1);
    run("hipMemcpyAsync, 2 streams", 2);
    run("hipMemcpyAsync, 4 streams", 4);
    run("pull kernel, 1 WG/CU", 10);
    run("pull kernel, 2 WG/CU", 11);
    run("pull kernel, 8 WG/CU", 12);
    run("hipMemcpyAsync, 1 stream (again)", 1);
    return 0;
}
