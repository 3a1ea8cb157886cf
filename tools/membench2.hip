// membench2.hip -- access-pattern sweep for k-read/m-write stripe streams.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UN>
__global__ void copy_flat(const u32x4* __restrict__ a, u32x4* __restrict__ b) {
    size_t base = (size_t(blockIdx.x) * UN) * blockDim.x + threadIdx.x;
    u32x4 v[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) v[u] = a[base + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < UN; ++u) b[base + u * blockDim.x] = v[u];
}
template <int UN>
__global__ void read_flat(const u32x4* __restrict__ a, u32x4* __restrict__ b) {
    size_t base = (size_t(blockIdx.x) * UN) * blockDim.x + threadIdx.x;
    u32x4 acc = {0,0,0,0};
#pragma unroll
    for (int u = 0; u < UN; ++u) acc ^= a[base + u * blockDim.x];
    if (acc.x == 0x12345679u) b[0] = acc;
}

// one block per (stripe, chunk of CH columns); BT threads; each thread handles CH/BT columns
template <int K, int M, int BT, int CPT, bool XCD>
__global__ __launch_bounds__(BT) void stripe_k(const u32x4* __restrict__ data, u32x4* __restrict__ par, size_t cols, int chunks, int nblocks) {
    int bid = blockIdx.x;
    if (XCD) { // group 8 consecutive logical blocks onto one XCD: logical = (bid%8)*(nblocks/8) + bid/8
        bid = (bid % 8) * (nblocks / 8) + bid / 8;
    }
    const size_t s = bid / chunks;
    const int chunk = bid % chunks;
    const u32x4* d = data + s * K * cols;
    u32x4* p = par + s * M * cols;
    const size_t c0 = size_t(chunk) * BT * CPT + threadIdx.x;
#pragma unroll 1
    for (int it = 0; it < CPT; ++it) {
        const size_t c = c0 + it * BT;
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = d[j * cols + c];
#pragma unroll
        for (int t = 0; t < M; ++t) {
            u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
            for (int j = 0; j < K; ++j) acc ^= (x[j] << ((t + j) & 7));
            p[t * cols + c] = acc;
        }
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
    const int K = 10, M = 4;
    const size_t cols = S / 16;
    u32x4 *data, *par;
    CK(hipMalloc(&data, stripes * K * S)); CK(hipMalloc(&par, stripes * M * S));
    CK(hipMemset(data, 1, stripes * K * S)); CK(hipMemset(par, 0, stripes * M * S));
    const double enc = double(stripes) * (K + M) * S;
    const int reps = 5;
    const size_t n16 = stripes * K * S / 16 / 2;  // half-buffer elements
    float ms;
#define COPY(UN, BT) ms = timeit([&]{ copy_flat<UN><<<n16 / (UN * BT), BT>>>(data, data + n16); }, reps); printf("copy UN=%d BT=%d  %7.1f GB/s\n", UN, BT, 2.0*n16*16/ms/1e6);
    COPY(1, 256) COPY(4, 256) COPY(8, 256) COPY(1, 1024) COPY(4, 512)
#define READ(UN, BT) ms = timeit([&]{ read_flat<UN><<<2*n16 / (UN * BT), BT>>>(data, par); }, reps); printf("read UN=%d BT=%d  %7.1f GB/s\n", UN, BT, 2.0*n16*16/ms/1e6);
    READ(1, 256) READ(4, 256) READ(8, 256)
#define ST(BT, CPT, XCD) { int chunks = cols / (BT * CPT); int nb = stripes * chunks; ms = timeit([&]{ stripe_k<K, M, BT, CPT, XCD><<<nb, BT>>>(data, par, cols, chunks, nb); }, reps); printf("stripe BT=%-4d CPT=%-3d xcd=%d blocks=%-7d %7.1f GB/s\n", BT, CPT, XCD, nb, enc/ms/1e6); }
    ST(256, 1, false) ST(256, 2, false) ST(256, 4, false) ST(512, 1, false) ST(1024, 1, false) ST(128, 1, false) ST(64, 1, false) ST(64, 4, false)
    ST(256, 1, true) ST(256, 4, true) ST(64, 1, true)
    return 0;
}
