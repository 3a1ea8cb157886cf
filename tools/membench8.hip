// membench8.hip -- XCD-aware block order for the streaming encode shapes.
// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8).
//   map 0: logical block = b                 (default: a stripe's column chunks spread over all XCDs)
//   map 1: logical block = (b % 8) * (G / 8) + b / 8   (each XCD streams one contiguous eighth)
//   map 2: logical block = (b / 8) % C * ... chunk-major: chunk c of 8 consecutive stripes on one XCD
// Shapes: RS(10,4) and RS(8,14) with 1 MiB shards (4 KiB per shard per block) and
// RS(64,16) with 64 KiB shards (8 KiB per shard per block), nt loads/stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load((GlobalCU4*)p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, (GlobalU4*)p); }

template <int MAP>
__device__ __forceinline__ uint32_t logical(uint32_t b, uint32_t G, uint32_t chunks) {
    if constexpr (MAP == 1) {
        const uint32_t per = G / 8;  // G is a multiple of 8
        return (b % 8) * per + b / 8;
    } else if constexpr (MAP == 2) {
        // XCD x gets stripes x, x+8, ... ; within an XCD blocks walk a stripe's chunks in order
        const uint32_t x = b % 8, i = b / 8;
        const uint32_t s_local = i / chunks, c = i % chunks;
        return (s_local * 8 + x) * chunks + c;
    }
    return b;
}

// K data shards, M outputs, C 16-B columns per lane (block = 256 * C columns per shard)
template <int K, int M, int C, int MAP>
__global__ __launch_bounds__(256) void enc(const u32x4* __restrict__ data, u32x4* __restrict__ par, size_t pitch, uint32_t chunks) {
    const uint32_t L = logical<MAP>(blockIdx.x, gridDim.x, chunks);
    const size_t s = L / chunks;
    const uint32_t chunk = L % chunks;
    u32x4 acc[M][C];
#pragma unroll
    for (int t = 0; t < M; ++t)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[t][c] = u32x4{0u, 0u, 0u, (unsigned)t};
#pragma unroll 4
    for (int j = 0; j < K; ++j) {
        u32x4 x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = ld(data + (s * K + j) * pitch + (size_t(chunk) * C + c) * 256 + threadIdx.x);
#pragma unroll
        for (int t = 0; t < M; ++t)
#pragma unroll
            for (int c = 0; c < C; ++c) acc[t][c] ^= x[c] << ((t + j) & 7);
    }
#pragma unroll
    for (int t = 0; t < M; ++t)
#pragma unroll
        for (int c = 0; c < C; ++c) st(par + (s * M + t) * pitch + (size_t(chunk) * C + c) * 256 + threadIdx.x, acc[t][c]);
}

template <typename F> float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

template <int K, int M, int C> void shape(const char* name, size_t S, int stripes, u32x4* data, u32x4* par) {
    const size_t pitch = S / 16;
    const uint32_t chunks = S / 16 / (256 * C);
    const dim3 g(stripes * chunks);
    float t0 = timeit([&] { hipLaunchKernelGGL((enc<K, M, C, 0>), g, dim3(256), 0, 0, data, par, pitch, chunks); }, 3);
    float t1 = timeit([&] { hipLaunchKernelGGL((enc<K, M, C, 1>), g, dim3(256), 0, 0, data, par, pitch, chunks); }, 3);
    float t2 = timeit([&] { hipLaunchKernelGGL((enc<K, M, C, 2>), g, dim3(256), 0, 0, data, par, pitch, chunks); }, 3);
    const double bytes = double(stripes) * (K + M) * S;
    printf("%-22s default %7.1f  xcd-contiguous %7.1f  xcd-by-stripe %7.1f GB/s\n", name, bytes / t0 / 1e6, bytes / t1 / 1e6, bytes / t2 / 1e6);
}

int main() {
    u32x4 *data, *par;
    const size_t dbytes = size_t(4096) * 10 * (1 << 20), pbytes = size_t(4096) * 4 * (1 << 20);
    CK(hipMalloc(&data, dbytes));
    CK(hipMalloc(&par, pbytes));
    CK(hipMemset(data, 1, dbytes));
    for (int rep = 0; rep < 2; ++rep) {
        shape<10, 4, 1>("RS(10,4) 1 MiB", 1 << 20, 4096, data, par);          // 40 GiB data
        shape<64, 16, 2>("RS(64,16) 64 KiB", 1 << 16, 8192, data, par);      // 32 GiB data
        shape<8, 6, 1>("RS(8,14) 1 MiB", 1 << 20, 2048, data, par);          // 16 GiB data, 12 GiB parity
    }
    return 0;
}
