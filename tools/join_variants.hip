// Standalone micro-benchmark of OR-join streaming variants at the bench size
// (3 x 2^32 16-byte cells = 192 GiB resident).  Not part of liblaspj: it explores
// launch shapes and cache policies for k_or16 before one is adopted there.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/join_variants tools/join_variants.hip
//   run:   tools/join_variants [log2_cells=32] [steps=6]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <bool NT>
__device__ __forceinline__ u64x2 ld(const u64x2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u64x2* p, u64x2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__global__ void k_fill(u64x2* p, uint64_t n, u64 seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        u64 x = (i + seed) * 0x9E3779B97F4A7C15ull;
        x ^= x >> 31;
        p[i] = u64x2{x, x & (x >> 7)};
    }
}

// grid-stride, U cells per lane in flight, optional XCD swizzle of the block index
template <int U, bool NTL, bool NTS, bool SWZ, int B>
__global__ __launch_bounds__(B) void k_gs(u64x2* d, const u64x2* a, const u64x2* b, uint64_t n) {
    uint64_t blk = blockIdx.x;
    if constexpr (SWZ) {
        // dispatch is round-robin over 8 XCDs: make XCD x own a contiguous 1/8 of each sweep
        uint64_t per = gridDim.x / 8;
        blk = (blk % 8) * per + blk / 8;
    }
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = blk * B + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u64x2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NTL>(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld<NTL>(b + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st<NTS>(d + i + u * stride, x[u] | y[u]);
    }
    for (; i < n; i += stride) st<NTS>(d + i, ld<NTL>(a + i) | ld<NTL>(b + i));
}

// each block owns one contiguous chunk; U consecutive block-widths per iteration
template <int U, int B>
__global__ __launch_bounds__(B) void k_chunk(u64x2* d, const u64x2* a, const u64x2* b,
                                             uint64_t n) {
    uint64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    chunk = (chunk + (uint64_t)U * B - 1) / ((uint64_t)U * B) * ((uint64_t)U * B);
    uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * B < hi; i += U * B) {
        u64x2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<true>(a + i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld<true>(b + i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st<true>(d + i + u * B, x[u] | y[u]);
    }
    for (; i < hi; i += B) st<true>(d + i, ld<true>(a + i) | ld<true>(b + i));
}

// 32 bytes per lane: two adjacent cells per lane per access pair
template <int U, int B>
__global__ __launch_bounds__(B) void k_pair(u64x2* d, const u64x2* a, const u64x2* b,
                                            uint64_t n) {
    const uint64_t np = n / 2;
    const uint64_t stride = (uint64_t)gridDim.x * B;
    uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x;
    for (; i + (U - 1) * stride < np; i += U * stride) {
        u64x2 x[2 * U], y[2 * U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[2 * u] = ld<true>(a + 2 * (i + u * stride));
            x[2 * u + 1] = ld<true>(a + 2 * (i + u * stride) + 1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            y[2 * u] = ld<true>(b + 2 * (i + u * stride));
            y[2 * u + 1] = ld<true>(b + 2 * (i + u * stride) + 1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st<true>(d + 2 * (i + u * stride), x[2 * u] | y[2 * u]);
            st<true>(d + 2 * (i + u * stride) + 1, x[2 * u + 1] | y[2 * u + 1]);
        }
    }
    for (; i < np; i += stride) {
        st<true>(d + 2 * i, ld<true>(a + 2 * i) | ld<true>(b + 2 * i));
        st<true>(d + 2 * i + 1, ld<true>(a + 2 * i + 1) | ld<true>(b + 2 * i + 1));
    }
}

typedef void (*Kern)(u64x2*, const u64x2*, const u64x2*, uint64_t);

struct Variant {
    const char* name;
    Kern k;
    int grid_per_cu;
    int block;
    bool inplace;
};

// skew mode: tools/join_variants <lg> <steps> skew <bytes>...: the current kernel with
// b offset by `bytes` and d by 2 x `bytes` from their allocations (HBM placement of the
// three streams relative to each other)
static int skew_mode(int lg, int steps, int argc, char** argv) {
    uint64_t n = 1ull << lg;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t pad = 64ull << 20;
    char *ra, *rb, *rd;
    CK(hipMalloc(&ra, n * 16 + pad));
    CK(hipMalloc(&rb, n * 16 + pad));
    CK(hipMalloc(&rd, n * 16 + 2 * pad));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int k = 4; k < argc; ++k) {
        const uint64_t sk = strtoull(argv[k], nullptr, 0);
        u64x2* a = (u64x2*)ra;
        u64x2* b = (u64x2*)(rb + sk);
        u64x2* d = (u64x2*)(rd + 2 * sk);
        hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, a, n, 1ull);
        hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, b, n, 2ull);
        auto kern = k_gs<2, true, true, false, 256>;
        hipLaunchKernelGGL(kern, dim3(cus * 64), dim3(256), 0, 0, d, a, b, n);
        CK(hipEventRecord(e0, 0));
        for (int s = 0; s < steps; ++s)
            hipLaunchKernelGGL(kern, dim3(cus * 64), dim3(256), 0, 0, d, a, b, n);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= steps;
        const double gbs = 48.0 * n / (ms * 1e-3) / 1e9;
        printf("skew %-10llu a=%p b=%p d=%p %8.3f ms %7.1f GB/s %.1f%%\n", (unsigned long long)sk,
               (void*)a, (void*)b, (void*)d, ms, gbs, gbs / 80.0);
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    int lg = argc > 1 ? atoi(argv[1]) : 32;
    int steps = argc > 2 ? atoi(argv[2]) : 6;
    if (argc > 3 && !strcmp(argv[3], "skew")) return skew_mode(lg, steps, argc, argv);
    uint64_t n = 1ull << lg;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    u64x2 *a, *b, *d;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&d, n * 16));
    hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, a, n, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, b, n, 2ull);
    hipLaunchKernelGGL(k_fill, dim3(cus * 16), dim3(256), 0, 0, d, n, 3ull);
    CK(hipDeviceSynchronize());
    Variant vs[] = {
        {"gs_u2_nt_256x64 (current)", k_gs<2, true, true, false, 256>, 64, 256, false},
        {"gs_u2_nt_256x64 inplace", k_gs<2, true, true, false, 256>, 64, 256, true},
        {"gs_u2_ntload_plainstore", k_gs<2, true, false, false, 256>, 64, 256, false},
        {"gs_u2_plainload_ntstore", k_gs<2, false, true, false, 256>, 64, 256, false},
        {"gs_u2_nt_swz", k_gs<2, true, true, true, 256>, 64, 256, false},
        {"gs_u4_nt_256x32", k_gs<4, true, true, false, 256>, 32, 256, false},
        {"gs_u1_nt_256x128", k_gs<1, true, true, false, 256>, 128, 256, false},
        {"gs_u2_nt_512x32", k_gs<2, true, true, false, 512>, 32, 512, false},
        {"gs_u2_nt_1024x16", k_gs<2, true, true, false, 1024>, 16, 1024, false},
        {"chunk_u2_256x64", k_chunk<2, 256>, 64, 256, false},
        {"chunk_u4_256x16", k_chunk<4, 256>, 16, 256, false},
        {"chunk_u2_256x8", k_chunk<2, 256>, 8, 256, false},
        {"pair_u1_256x64", k_pair<1, 256>, 64, 256, false},
        {"pair_u2_256x32", k_pair<2, 256>, 32, 256, false},
        {"gs_u2_nt_256x64 (current, again)", k_gs<2, true, true, false, 256>, 64, 256, false},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Variant& v : vs) {
        u64x2* dst = v.inplace ? a : d;
        int grid = cus * v.grid_per_cu;
        hipLaunchKernelGGL(v.k, dim3(grid), dim3(v.block), 0, 0, dst, a, b, n);
        CK(hipEventRecord(e0, 0));
        for (int s = 0; s < steps; ++s)
            hipLaunchKernelGGL(v.k, dim3(grid), dim3(v.block), 0, 0, dst, a, b, n);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= steps;
        double gbs = 48.0 * n / (ms * 1e-3) / 1e9;
        printf("%-36s %8.3f ms  %7.1f GB/s  %.1f%%\n", v.name, ms, gbs, gbs / 80.0);
        fflush(stdout);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(d));
    return 0;
}
