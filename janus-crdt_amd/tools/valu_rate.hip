// valu_rate.hip — issue rate of the 32-bit integer VALU instructions the SHA-256 kernels are made of
// (v_alignbit_b32, v_bitop3_b32, v_add3_u32, v_add_u32) against v_fma_f32, on gfx950.  Each lane runs 8
// independent chains of one instruction (so dependency latency is hidden by the other chains and by the
// other waves); 8 waves per SIMD.  Reports wave-instructions per cycle per SIMD at the measured clock-free
// rate (events) and the assumed 2.4 GHz: 0.5 = one wave64 instruction every 2 cycles, 0.25 = every 4.
// Used to price csrc/digest.hip's roofline (bench.py SHA_VALU_PER_BLOCK / VALU_LANE_OPS).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../csrc/sha256_device.hpp"

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

constexpr int kIters = 4096;  // loop trips; 8 chains x 8 unrolled steps per trip
constexpr int kSteps = 8;

template <int Op>
__device__ __forceinline__ uint32_t step(uint32_t x, uint32_t y, uint32_t z) {
    if constexpr (Op == 0) return __builtin_amdgcn_alignbit(x, y, 7);
    else if constexpr (Op == 1) return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
    else if constexpr (Op == 2) return x + y + z;  // v_add3_u32
    else if constexpr (Op == 3) return x + y;      // v_add_u32
    else {
        float r;  // one v_fma_f32 (inline: the compiler would pack pairs into v_pk_fma_f32)
        asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(__uint_as_float(x)), "v"(__uint_as_float(y)), "v"(__uint_as_float(z)));
        return __float_as_uint(r);
    }
}

template <int Op>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = seed + threadIdx.x * 8 + k;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int s = 0; s < kSteps; ++s) {  // 8 independent instructions per step, each mixing two chains
            uint32_t n[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) n[k] = step<Op>(c[k], c[(k + 1) & 7], c[(k + 3) & 7]);
#pragma unroll
            for (int k = 0; k < 8; ++k) c[k] = n[k];
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= c[k];
    if (r == 0x12345678u) out[blockIdx.x] = r;  // keeps the chains live
}

template <int Op>
void run(const char* name, uint32_t* d, int n_cu) {
    const int blocks = n_cu * 8;  // 8 x 256-thread workgroups per CU = 8 waves per SIMD
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_rate<Op>, dim3(blocks), dim3(256), 0, 0, d, 1u);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_rate<Op>, dim3(blocks), dim3(256), 0, 0, d, 2u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double wave_insts = (double)blocks * 4 * kIters * kSteps * 8;  // 4 waves per block
    const double per_simd_per_cycle = wave_insts / (n_cu * 4.0) / (ms * 1e-3 * 2.4e9);
    std::printf("%-16s %8.3f ms  %.3f wave-instructions per cycle per SIMD at 2.4 GHz (%.2f cycles each)\n", name, ms, per_simd_per_cycle,
                1.0 / per_simd_per_cycle);
}

// The issue ceiling of csrc/digest.hip's compression: every lane compresses kBlocks blocks held in registers
// (each block's words fed from the previous digest, so nothing hoists), no memory traffic; `wg_per_cu`
// 256-thread workgroups per CU = that many waves per SIMD.
constexpr int kBlocks = 256;
__global__ __launch_bounds__(256) void k_sha_ceiling(uint32_t* out, uint32_t seed) {
    uint32_t H[8], W[16];
    jgsha::sha_init(H);
#pragma unroll
    for (int k = 0; k < 16; ++k) W[k] = seed + threadIdx.x * 16 + k + blockIdx.x;
    for (int b = 0; b < kBlocks; ++b) {
        uint32_t X[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) X[k] = W[k] ^ H[k & 7];
        jgsha::compress(H, X);
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r ^= H[k];
    if (r == 0x12345678u) out[blockIdx.x] = r;
}

void run_sha(uint32_t* d, int n_cu, int wg_per_cu) {
    const int blocks = n_cu * wg_per_cu;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_sha_ceiling, dim3(blocks), dim3(256), 0, 0, d, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(k_sha_ceiling, dim3(blocks), dim3(256), 0, 0, d, 2u);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double sha_blocks = (double)blocks * 256 * kBlocks;
    const double cyc = (ms * 1e-3 * 2.4e9) * (n_cu * 4.0) / (sha_blocks / 64.0);  // cycles per wave-block per SIMD
    std::printf("sha256 compress, %d waves/SIMD: %8.3f ms  %.2f Gblocks/s  (%.0f SIMD cycles per 64-lane block at 2.4 GHz)\n", wg_per_cu, ms,
                sha_blocks / (ms * 1e-3) / 1e9, cyc);
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    uint32_t* d = nullptr;
    CHECK(hipMalloc(&d, 1 << 20));
    std::printf("%s, %d CUs\n", p.gcnArchName, p.multiProcessorCount);
    run<0>("v_alignbit_b32", d, p.multiProcessorCount);
    run<1>("v_bitop3_b32", d, p.multiProcessorCount);
    run<2>("v_add3_u32", d, p.multiProcessorCount);
    run<3>("v_add_u32", d, p.multiProcessorCount);
    run<4>("v_fma_f32", d, p.multiProcessorCount);
    run_sha(d, p.multiProcessorCount, 4);  // k_sha_msgs' occupancy (120 VGPRs)
    run_sha(d, p.multiProcessorCount, 5);  // the most that fit (95 VGPRs)
    CHECK(hipFree(d));
    return 0;
}
