// pcie_small.hip -- how fast can a kernel pull a single message's chunk
// (256 KiB .. 1 MiB) out of pinned host memory, by grid shape?  Timed inside
// the kernel: every block records the device wall clock before its first
// load and after its last one arrived; the transfer time is the max end
// minus the min start (no launch or dispatch in it).  Shapes: threads per
// block x 16-byte loads in flight per lane (ILP), blocks = bytes / (threads
// x 16 x ILP).  Medians of 15 runs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int ILP>
__global__ void pull(const u32x4* __restrict__ src, u32x4* __restrict__ dst, unsigned long long* t, size_t per_block) {
    const size_t base = static_cast<size_t>(blockIdx.x) * per_block;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    u32x4 v[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) v[i] = __builtin_nontemporal_load(src + base + i * blockDim.x + threadIdx.x);
    u32x4 acc = v[0];
#pragma unroll
    for (int i = 1; i < ILP; ++i) acc ^= v[i];
    dst[base / ILP + threadIdx.x] = acc;
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = t1;
    }
}

template <int ILP>
double run(const u32x4* hsrc, u32x4* ddst, unsigned long long* dt, unsigned long long* ht, size_t bytes, int threads,
           double tick_us) {
    const size_t per_block = static_cast<size_t>(threads) * ILP;  // 16-byte units
    const int blocks = static_cast<int>(bytes / 16 / per_block);
    std::vector<double> r;
    for (int rep = 0; rep < 16; ++rep) {
        hipLaunchKernelGGL(pull<ILP>, dim3(blocks), dim3(threads), 0, 0, hsrc, ddst, dt, per_block);
        (void)hipMemcpy(ht, dt, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
        unsigned long long lo = ~0ull, hi = 0;
        for (int b = 0; b < blocks; ++b) {
            lo = std::min(lo, ht[2 * b]);
            hi = std::max(hi, ht[2 * b + 1]);
        }
        if (rep) r.push_back((hi - lo) * tick_us);
    }
    std::sort(r.begin(), r.end());
    return r[r.size() / 2];
}

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t N = size_t(1) << 20;
    void* h = nullptr;
    CK(hipHostMalloc(&h, N, hipHostMallocDefault));
    std::memset(h, 3, N);
    void* hd = nullptr;
    CK(hipHostGetDevicePointer(&hd, h, 0));
    void* d = nullptr;
    CK(hipMalloc(&d, N));
    unsigned long long *dt = nullptr, *ht = nullptr;
    CK(hipMalloc(&dt, sizeof(unsigned long long) * 2 * 65536));
    CK(hipHostMalloc(reinterpret_cast<void**>(&ht), sizeof(unsigned long long) * 2 * 65536, hipHostMallocDefault));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const double tick_us = 1e3 / khz;
    const u32x4* src = static_cast<const u32x4*>(hd);
    u32x4* dst = static_cast<u32x4*>(d);
    for (size_t bytes : {size_t(256) << 10, size_t(512) << 10, size_t(1) << 20}) {
        for (int threads : {64, 256}) {
            const double a = run<1>(src, dst, dt, ht, bytes, threads, tick_us);
            const double b = run<4>(src, dst, dt, ht, bytes, threads, tick_us);
            const double c = run<10>(src, dst, dt, ht, bytes, threads, tick_us);
            std::printf("%4zu KiB, %3d threads/block: ILP 1 %6.2f us (%5.1f GB/s, %5zu blocks) | ILP 4 %6.2f us (%5.1f GB/s) | ILP 10 %6.2f us (%5.1f GB/s, %4zu blocks)\n",
                        bytes >> 10, threads, a, bytes / a / 1e3, bytes / 16 / threads, b, bytes / b / 1e3, c,
                        bytes / c / 1e3, bytes / 16 / threads / 10);
        }
    }
    return 0;
}
