// membench.hip -- what HBM rate can a k-read / m-write stripe stream reach on
// MI355X?  Pure data movement (XOR, no GF tables) with the encode kernel's
// geometry, in several variants, plus copy / read-only / write-only anchors.
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT_LOAD, bool NT_STORE>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT_LOAD) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT_STORE>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT_STORE) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__global__ void copy_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) b[i] = a[i];
}
__global__ void read_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) acc ^= a[i];
    if (acc.x == 0x12345678u) b[0] = acc;
}
__global__ void write_k(u32x4* __restrict__ b, size_t n) {
    u32x4 v = {1, 2, 3, 4};
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) b[i] = v;
}

// stripe stream: block = (stripe, chunk); ITERS iterations of 256*U columns.
template <int K, int M, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void stripe_k(const u32x4* __restrict__ data, u32x4* __restrict__ par,
                                                size_t cols, int chunks, int iters) {
    const size_t s = blockIdx.x / chunks;
    const int chunk = blockIdx.x % chunks;
    const u32x4* d = data + s * K * cols;
    u32x4* p = par + s * M * cols;
    for (int it = 0; it < iters; ++it) {
        const size_t c0 = (size_t(chunk) * iters + it) * 256 * U + threadIdx.x;
        u32x4 x[K][U];
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) x[j][u] = ld<NTL, NTS>(d + j * cols + c0 + u * 256);
#pragma unroll
        for (int t = 0; t < M; ++t)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
                for (int j = 0; j < K; ++j) acc ^= (x[j][u] << ((t + j) & 7));
                st<NTS>(p + t * cols + c0 + u * 256, acc);
            }
    }
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const size_t S = 1 << 20;  // shard bytes
    const int stripes = argc > 1 ? atoi(argv[1]) : 2048;
    const int K = 10, M = 4;
    const size_t cols = S / 16;
    u32x4 *data, *par;
    CK(hipMalloc(&data, stripes * K * S));
    CK(hipMalloc(&par, stripes * M * S));
    CK(hipMemset(data, 1, stripes * K * S));
    CK(hipMemset(par, 0, stripes * M * S));
    const double enc_bytes = double(stripes) * (K + M) * S;
    const int reps = 5;

    const size_t n16 = stripes * K * S / 16 / 2;
    float ms = timeit([&] { copy_k<<<8192, 256>>>(data, data + n16, n16); }, reps);
    printf("copy            %7.1f GB/s\n", 2.0 * n16 * 16 / ms / 1e6);
    ms = timeit([&] { read_k<<<8192, 256>>>(data, par, 2 * n16); }, reps);
    printf("read-only       %7.1f GB/s\n", 2.0 * n16 * 16 / ms / 1e6);
    ms = timeit([&] { write_k<<<8192, 256>>>(data, 2 * n16); }, reps);
    printf("write-only      %7.1f GB/s\n", 2.0 * n16 * 16 / ms / 1e6);

#define RUN(U, NTL, NTS, ITERS)                                                              \
    {                                                                                        \
        const int chunks = int(cols / (256 * U * ITERS));                                    \
        ms = timeit([&] { stripe_k<K, M, U, NTL, NTS><<<stripes * chunks, 256>>>(data, par, cols, chunks, ITERS); }, reps); \
        printf("stripe U=%d ntl=%d nts=%d iters=%-3d %7.1f GB/s (%.3f ms)\n", U, NTL, NTS, ITERS, enc_bytes / ms / 1e6, ms); \
    }
    RUN(1, false, false, 16)
    RUN(1, false, false, 4)
    RUN(1, false, false, 64)
    RUN(1, false, false, 256)
    RUN(2, false, false, 8)
    RUN(1, true, false, 16)
    RUN(1, false, true, 16)
    RUN(1, true, true, 16)
    RUN(2, true, true, 8)
    RUN(1, false, false, 1)
    return 0;
}
