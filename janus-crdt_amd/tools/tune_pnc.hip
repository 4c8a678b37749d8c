// tune_pnc.hip — dev tool: interleaved A/B timing of PN-Counter dense-merge kernel variants on the
// C2 shape (10M keys x 64 replicas, int64), one process, hipEvents per launch, median of rounds.
// Build: hipcc -O3 --offload-arch=gfx950 -o tune_pnc tune_pnc.hip ; run on the GPU box.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

typedef long long v2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2 vmax(v2 a, v2 b) {
    v2 r;
    r.x = a.x > b.x ? a.x : b.x;
    r.y = a.y > b.y ? a.y : b.y;
    return r;
}

template <bool NT> __device__ __forceinline__ v2 ld(const v2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT> __device__ __forceinline__ void st(v2* p, v2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride, U vectors in flight per lane (the production kernel shape)
template <int U, bool NTL, bool NTS, int B>
__global__ __launch_bounds__(B) void k_stride(v2* AP, v2* AN, const v2* BP, const v2* BN, unsigned long long nv) {
    const unsigned long long stride = (unsigned long long)gridDim.x * B;
    unsigned long long i = (unsigned long long)blockIdx.x * B + threadIdx.x;
    for (; i + (U - 1) * stride < nv; i += U * stride) {
        v2 ap[U], an[U], bp[U], bn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ap[u] = ld<false>(AP + i + u * stride);
            bp[u] = ld<NTL>(BP + i + u * stride);
            an[u] = ld<false>(AN + i + u * stride);
            bn[u] = ld<NTL>(BN + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st<NTS>(AP + i + u * stride, vmax(ap[u], bp[u]));
            st<NTS>(AN + i + u * stride, vmax(an[u], bn[u]));
        }
    }
    for (; i < nv; i += stride) {
        AP[i] = vmax(AP[i], BP[i]);
        AN[i] = vmax(AN[i], BN[i]);
    }
}

// block-contiguous chunks: block b owns [b*C, (b+1)*C) vectors, C = B*U*ITER
template <int U, bool NTL, bool NTS, int B>
__global__ __launch_bounds__(B) void k_chunk(v2* AP, v2* AN, const v2* BP, const v2* BN, unsigned long long nv, unsigned long long per_block) {
    const unsigned long long beg = (unsigned long long)blockIdx.x * per_block;
    const unsigned long long end = beg + per_block < nv ? beg + per_block : nv;
    unsigned long long i = beg + threadIdx.x;
    for (; i + (U - 1) * B < end; i += U * B) {
        v2 ap[U], an[U], bp[U], bn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ap[u] = ld<false>(AP + i + u * B);
            bp[u] = ld<NTL>(BP + i + u * B);
            an[u] = ld<false>(AN + i + u * B);
            bn[u] = ld<NTL>(BN + i + u * B);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st<NTS>(AP + i + u * B, vmax(ap[u], bp[u]));
            st<NTS>(AN + i + u * B, vmax(an[u], bn[u]));
        }
    }
    for (; i < end; i += B) {
        AP[i] = vmax(AP[i], BP[i]);
        AN[i] = vmax(AN[i], BN[i]);
    }
}

// reference point: plain float4-style copy of the same byte volume (read 4 arrays... write 2)
template <int B>
__global__ __launch_bounds__(B) void k_copy(v2* dst, const v2* src, unsigned long long nv) {
    const unsigned long long stride = (unsigned long long)gridDim.x * B;
    for (unsigned long long i = (unsigned long long)blockIdx.x * B + threadIdx.x; i < nv; i += stride) dst[i] = src[i];
}

struct Variant {
    const char* name;
    void (*launch)(v2*, v2*, const v2*, const v2*, unsigned long long, hipStream_t, int);
};

int num_cus;

template <int U, bool NTL, bool NTS, int B, int PER_CU>
void L_stride(v2* a, v2* b, const v2* c, const v2* d, unsigned long long nv, hipStream_t s, int) {
    unsigned g = num_cus * PER_CU;
    hipLaunchKernelGGL((k_stride<U, NTL, NTS, B>), dim3(g), dim3(B), 0, s, a, b, c, d, nv);
}
template <int U, bool NTL, bool NTS, int B, int ITER>
void L_chunk(v2* a, v2* b, const v2* c, const v2* d, unsigned long long nv, hipStream_t s, int) {
    unsigned long long per = (unsigned long long)B * U * ITER;
    unsigned g = (unsigned)((nv + per - 1) / per);
    hipLaunchKernelGGL((k_chunk<U, NTL, NTS, B>), dim3(g), dim3(B), 0, s, a, b, c, d, nv, per);
}

int main(int argc, char** argv) {
    const unsigned long long n_cells = 10000000ull * 64, nv = n_cells / 2;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    num_cus = prop.multiProcessorCount;
    v2 *AP, *AN, *BP, *BN;
    CK(hipMalloc(&AP, nv * 16)); CK(hipMalloc(&AN, nv * 16)); CK(hipMalloc(&BP, nv * 16)); CK(hipMalloc(&BN, nv * 16));
    CK(hipMemset(AP, 1, nv * 16)); CK(hipMemset(AN, 2, nv * 16)); CK(hipMemset(BP, 3, nv * 16)); CK(hipMemset(BN, 0, nv * 16));
    std::vector<Variant> vs = {
        {"stride U4 B256 g16/CU (prod r1)", L_stride<4, false, false, 256, 16>},
        {"chunk U4 B256 it4 nt both", L_chunk<4, true, true, 256, 4>},
        {"chunk U1 B256 it1 nt both", L_chunk<1, true, true, 256, 1>},
        {"chunk U1 B256 it1 plain", L_chunk<1, false, false, 256, 1>},
        {"chunk U1 B256 it1 ntload", L_chunk<1, true, false, 256, 1>},
        {"chunk U1 B256 it1 ntstore", L_chunk<1, false, true, 256, 1>},
        {"chunk U2 B256 it1 nt both", L_chunk<2, true, true, 256, 1>},
        {"chunk U1 B512 it1 nt both", L_chunk<1, true, true, 512, 1>},
        {"chunk U1 B128 it1 nt both", L_chunk<1, true, true, 128, 1>},
        {"chunk U1 B1024 it1 nt both", L_chunk<1, true, true, 1024, 1>},
        {"chunk U1 B256 it2 nt both", L_chunk<1, true, true, 256, 2>},
        {"chunk U2 B256 it2 nt both", L_chunk<2, true, true, 256, 2>},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    std::vector<std::vector<float>> t(vs.size());
    for (auto& v : vs) v.launch(AP, AN, BP, BN, nv, s, 0);  // warm
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r)
        for (size_t k = 0; k < vs.size(); ++k) {
            CK(hipEventRecord(e0, s));
            vs[k].launch(AP, AN, BP, BN, nv, s, 0);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            t[k].push_back(ms);
        }
    // copy reference: 3 x (read 16B write 16B) ~ same 48 B/cell? no: report copy GB/s separately
    std::vector<float> tc;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL((k_copy<256>), dim3(num_cus * 16), dim3(256), 0, s, AP, BP, nv);
        hipLaunchKernelGGL((k_copy<256>), dim3(num_cus * 16), dim3(256), 0, s, AN, BN, nv);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        tc.push_back(ms);
    }
    const double bytes = (double)n_cells * 48;
    for (size_t k = 0; k < vs.size(); ++k) {
        auto v = t[k]; std::sort(v.begin(), v.end());
        std::printf("%-40s median %.3f ms  min %.3f  -> %.0f GB/s (%.1f%% of 8 TB/s)\n", vs[k].name, v[v.size() / 2], v[0],
                    bytes / (v[v.size() / 2] * 1e-3) / 1e9, 100.0 * bytes / (v[v.size() / 2] * 1e-3) / 8e12);
    }
    std::sort(tc.begin(), tc.end());
    const double cb = (double)nv * 16 * 4;
    std::printf("%-40s median %.3f ms -> %.0f GB/s (copy of 2 x 5.12 GB)\n", "reference copy", tc[tc.size() / 2], cb / (tc[tc.size() / 2] * 1e-3) / 1e9);
    return 0;
}
