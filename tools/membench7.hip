// membench7.hip -- time-phased movement: can the RS(10,4) encode shape beat
// the mixed 10-read/4-write stream (6.0-6.2 TB/s, membench6) if every CU
// reads only in global "read windows" and writes only in "write windows"?
// Windows are absolute multiples of the period on s_memrealtime (the 100 MHz
// constant clock), so no barrier is needed.  Persistent blocks: per window a
// block loads U units (10 x 16 B per lane each), keeps the 4 x 16 B outputs
// per unit in registers, waits for the write window and stores them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load((GlobalCU4*)p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, (GlobalU4*)p); }

constexpr int K = 10, M = 4;
const size_t S = 1 << 20;
const size_t PITCH = S / 16;
const int CHUNKS = S / 16 / 256;  // 4 KiB column chunks per shard

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void wait_until(uint64_t t) {
    while (now() < t) __builtin_amdgcn_s_sleep(2);
}

// Plain one-pass encode shape (one unit per block), for reference.
__global__ __launch_bounds__(256) void onepass(const u32x4* __restrict__ data, u32x4* __restrict__ par) {
    const size_t s = blockIdx.x / CHUNKS;
    const size_t col = size_t(blockIdx.x % CHUNKS) * 256 + threadIdx.x;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld(data + (s * K + j) * PITCH + col);
#pragma unroll
    for (int t = 0; t < M; ++t) {
        u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= (x[j] << ((t + j) & 7));
        st(par + (s * M + t) * PITCH + col, acc);
    }
}

template <int U>
__global__ __launch_bounds__(256) void phased(const u32x4* __restrict__ data, u32x4* __restrict__ par, uint32_t units,
                                              uint32_t period, uint32_t rwin) {
    // unit u = (stripe, chunk); block b takes units b*U .. b*U+U-1, then b + grid, ...
    uint64_t t = now();
    uint64_t base = (t / period + 1) * period;  // next window start (global)
    for (uint32_t u0 = blockIdx.x * U; u0 < units; u0 += gridDim.x * U) {
        wait_until(base);
        u32x4 out[U][M];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t uu = u0 + u < units ? u0 + u : units - 1;
            const size_t s = uu / CHUNKS;
            const size_t col = size_t(uu % CHUNKS) * 256 + threadIdx.x;
            u32x4 x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = ld(data + (s * K + j) * PITCH + col);
#pragma unroll
            for (int q = 0; q < M; ++q) {
                u32x4 acc = {0u, 0u, 0u, (unsigned)q};
#pragma unroll
                for (int j = 0; j < K; ++j) acc ^= (x[j] << ((q + j) & 7));
                out[u][q] = acc;
            }
        }
        wait_until(base + rwin);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u0 + u >= units) break;
            const uint32_t uu = u0 + u;
            const size_t s = uu / CHUNKS;
            const size_t col = size_t(uu % CHUNKS) * 256 + threadIdx.x;
#pragma unroll
            for (int q = 0; q < M; ++q) st(par + (s * M + q) * PITCH + col, out[u][q]);
        }
        base += period;
    }
}

int stripes = 4096;
u32x4 *data, *par;

template <typename F> float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}
double rate(float ms) { return double(stripes) * (K + M) * S / ms / 1e6; }

template <int U> void sweep(int blocks_per_cu, uint32_t period, uint32_t rwin) {
    const uint32_t units = stripes * CHUNKS;
    const int grid = 256 * blocks_per_cu;
    float ms = timeit([&] { hipLaunchKernelGGL(phased<U>, dim3(grid), dim3(256), 0, 0, data, par, units, period, rwin); }, 2);
    printf("phased U=%d blocks/CU=%d period=%u ticks read=%u: %8.3f ms %7.1f GB/s\n", U, blocks_per_cu, period, rwin, ms, rate(ms));
}

int main(int argc, char** argv) {
    if (argc > 1) stripes = atoi(argv[1]);
    CK(hipMalloc(&data, stripes * K * S));
    CK(hipMalloc(&par, stripes * M * S));
    CK(hipMemset(data, 1, stripes * K * S));
    CK(hipMemset(par, 0, stripes * M * S));
    float ms = timeit([&] { hipLaunchKernelGGL(onepass, dim3(stripes * CHUNKS), dim3(256), 0, 0, data, par); }, 3);
    printf("one-pass: %8.3f ms %7.1f GB/s\n", ms, rate(ms));
    // no phases (read window = period: writes right after the loads, like one-pass but persistent)
    sweep<4>(4, 1, 0);
    for (int bpc : {2, 4})
        for (uint32_t period : {600u, 1000u, 1600u, 2400u})
            for (double frac : {0.6, 0.7})
                sweep<4>(bpc, period, uint32_t(period * frac));
    for (uint32_t period : {1000u, 1600u, 2400u}) sweep<2>(4, period, uint32_t(period * 0.7));
    for (uint32_t period : {1600u, 2400u, 3200u}) sweep<8>(2, period, uint32_t(period * 0.7));
    ms = timeit([&] { hipLaunchKernelGGL(onepass, dim3(stripes * CHUNKS), dim3(256), 0, 0, data, par); }, 3);
    printf("one-pass: %8.3f ms %7.1f GB/s\n", ms, rate(ms));
    return 0;
}
