// pcie_rates.hip -- host<->device rates that bound the batched host-API
// calls (rs_encode_batch / rs_decode_batch: 64 config-1 messages = 64 MiB of
// survivors in, 25.6 MiB of parity out): copy-engine H2D / D2H of 16 MiB
// pinned chunks alone and both directions at once, against a kernel reading
// pinned host memory over PCIe (the engine's direct form) and writing it.
// Medians of 20 reps, GB/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <vector>

#define CK(x) do { if ((x) != hipSuccess) { std::printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

__global__ void read_host(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

template <class F>
static double med_ms(F f, hipStream_t s) {
    std::vector<double> t;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int r = 0; r < 21; ++r) {
        (void)hipEventRecord(a, s);
        f();
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t N = size_t(16) << 20;
    void *h1, *h2, *d1, *d2;
    CK(hipHostMalloc(&h1, N, hipHostMallocDefault));
    CK(hipHostMalloc(&h2, N, hipHostMallocDefault));
    CK(hipMalloc(&d1, N));
    CK(hipMalloc(&d2, N));
    memset(h1, 1, N);
    memset(h2, 2, N);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    void* hd1 = nullptr;
    CK(hipHostGetDevicePointer(&hd1, h1, 0));
    void* hd2 = nullptr;
    CK(hipHostGetDevicePointer(&hd2, h2, 0));
    auto gbs = [&](double ms, size_t bytes) { return bytes / ms / 1e6; };
    double ms = med_ms([&] { (void)hipMemcpyAsync(d1, h1, N, hipMemcpyHostToDevice, s1); }, s1);
    std::printf("copy engine H2D 16 MiB: %.1f GB/s\n", gbs(ms, N));
    ms = med_ms([&] { (void)hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s1); }, s1);
    std::printf("copy engine D2H 16 MiB: %.1f GB/s\n", gbs(ms, N));
    hipEvent_t e2;
    CK(hipEventCreate(&e2));
    ms = med_ms([&] {
        (void)hipMemcpyAsync(h2, d2, N, hipMemcpyDeviceToHost, s2);
        (void)hipEventRecord(e2, s2);
        (void)hipMemcpyAsync(d1, h1, N, hipMemcpyHostToDevice, s1);
        (void)hipStreamWaitEvent(s1, e2, 0);
    }, s1);
    std::printf("copy engine H2D + D2H 16 MiB each at once: %.1f GB/s each way\n", gbs(ms, N));
    for (int blocks : {64, 256, 1024, 4096}) {
        ms = med_ms([&] { hipLaunchKernelGGL(read_host, dim3(blocks), dim3(256), 0, s1, (const uint4*)hd1, (uint4*)d1, N / 16); }, s1);
        std::printf("kernel reads pinned host 16 MiB (%d blocks): %.1f GB/s\n", blocks, gbs(ms, N));
    }
    for (int blocks : {256, 1024}) {
        ms = med_ms([&] { hipLaunchKernelGGL(read_host, dim3(blocks), dim3(256), 0, s1, (const uint4*)d2, (uint4*)hd2, N / 16); }, s1);
        std::printf("kernel writes pinned host 16 MiB (%d blocks): %.1f GB/s\n", blocks, gbs(ms, N));
    }
    // A single config-1 chunk's sizes: one kernel reading 256 KiB .. 1 MiB of
    // pinned host memory (one 16-byte column per lane, as rs_matmul_kernel).
    for (size_t bytes : {size_t(256) << 10, size_t(512) << 10, size_t(1) << 20}) {
        const int blocks = static_cast<int>(bytes / 16 / 256);
        ms = med_ms([&] { hipLaunchKernelGGL(read_host, dim3(blocks), dim3(256), 0, s1, (const uint4*)hd1, (uint4*)d1, bytes / 16); }, s1);
        std::printf("kernel reads %zu KiB of pinned host (%d blocks): %.2f us, %.1f GB/s\n", bytes >> 10, blocks, ms * 1e3, gbs(ms, bytes));
    }
    ms = med_ms([&] {
        hipLaunchKernelGGL(read_host, dim3(1024), dim3(256), 0, s2, (const uint4*)d2, (uint4*)hd2, N / 16 * 4 / 10);
        (void)hipEventRecord(e2, s2);
        hipLaunchKernelGGL(read_host, dim3(1024), dim3(256), 0, s1, (const uint4*)hd1, (uint4*)d1, N / 16);
        (void)hipStreamWaitEvent(s1, e2, 0);
    }, s1);
    std::printf("kernel reads 16 MiB + another writes 6.4 MiB of pinned host at once: %.1f GB/s read\n", gbs(ms, N));
    return 0;
}
