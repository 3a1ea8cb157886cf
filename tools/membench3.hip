// membench3.hip -- does the 1 MiB power-of-two shard stride cost bandwidth?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// K reads, M writes; shard j of stripe s at base + s*sstride + j*pitch (in 16B units)
template <int K, int M>
__global__ __launch_bounds__(256) void stripe_k(const u32x4* __restrict__ data, u32x4* __restrict__ par, size_t pitch, size_t dss, size_t pss, int chunks) {
    const size_t s = blockIdx.x / chunks;
    const int chunk = blockIdx.x % chunks;
    const size_t c = size_t(chunk) * 256 + threadIdx.x;
    const u32x4* d = data + s * dss;
    u32x4* p = par + s * pss;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = d[j * pitch + c];
    if (M == 0) {
        u32x4 acc = {0,0,0,0};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= x[j];
        if (acc.x == 0x1234567u) par[0] = acc;
    }
#pragma unroll
    for (int t = 0; t < M; ++t) {
        u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= (x[j] << ((t + j) & 7));
        p[t * pitch + c] = acc;
    }
}

template <typename F> float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int main(int argc, char** argv) {
    const size_t S = 1 << 20;
    const int stripes = argc > 1 ? atoi(argv[1]) : 4096;
    const size_t cols = S / 16;
    const size_t maxpitch = S + 64 * 1024;
    u32x4 *data, *par;
    CK(hipMalloc(&data, stripes * 10 * maxpitch + (1 << 24))); CK(hipMalloc(&par, stripes * 4 * maxpitch + (1 << 24)));
    CK(hipMemset(data, 1, stripes * 10 * maxpitch)); CK(hipMemset(par, 0, stripes * 4 * maxpitch));
    const int reps = 5;
    float ms;
    const int chunks = cols / 256;
    size_t pads[] = {0, 256, 1024, 4096, 8192, 65536, 4096 + 256};
    for (size_t pad : pads) {
        size_t pitch = (S + pad) / 16;
        ms = timeit([&]{ stripe_k<10, 4><<<stripes * chunks, 256>>>(data, par, pitch, 10 * pitch, 4 * pitch, chunks); }, reps);
        printf("10r4w pad=%-6zu %7.1f GB/s\n", pad, double(stripes) * 14 * S / ms / 1e6);
    }
    for (size_t pad : pads) {
        size_t pitch = (S + pad) / 16;
        ms = timeit([&]{ stripe_k<10, 0><<<stripes * chunks, 256>>>(data, par, pitch, 10 * pitch, 0, chunks); }, reps);
        printf("10r0w pad=%-6zu %7.1f GB/s\n", pad, double(stripes) * 10 * S / ms / 1e6);
    }
    for (size_t pad : pads) {
        size_t pitch = (S + pad) / 16;
        ms = timeit([&]{ stripe_k<1, 1><<<stripes * 10 * chunks, 256>>>(data, par, pitch, pitch, pitch, chunks); }, reps);
        printf("1r1w  pad=%-6zu %7.1f GB/s\n", pad, double(stripes) * 20 * S / ms / 1e6);
    }
    for (size_t pad : pads) {  // 2 reads 2 writes per block
        size_t pitch = (S + pad) / 16;
        ms = timeit([&]{ stripe_k<2, 2><<<stripes * 5 * chunks, 256>>>(data, par, pitch, 2 * pitch, 2 * pitch, chunks); }, reps);
        printf("2r2w  pad=%-6zu %7.1f GB/s\n", pad, double(stripes) * 20 * S / ms / 1e6);
    }
    return 0;
}
