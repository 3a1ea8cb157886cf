// membench11.hip -- does separating reads from writes in time raise the
// RS(10,4) encode's movement ceiling?
//
// The encode (10 reads + 4 writes of 1 MiB shards per stripe) runs at the
// chip's float4-copy rate (~6.2 TB/s) while 10 reads alone move ~6.9 TB/s
// (profiles/r05c/): the writes cost DRAM read/write turnaround that barely
// shrinks with their number.  This program asks whether the turnaround can be
// amortised by making the whole chip read for a window and then write for a
// window, using the SoC-wide constant clock (s_memrealtime, 100 MHz) as the
// phase reference -- no inter-block synchronisation, every wait ends when the
// clock reaches the next window.
//
//   plain       the encode's shape: one 4 KiB column chunk of one stripe per block,
//               10 nt loads, XOR, 4 nt stores (the shipped kernel's movement)
//   reads       the same 10 loads, stores suppressed (data-dependent, never taken)
//   writes      the 4 stores only
//   batch<B>    grid-stride over the pieces, B pieces per block per batch: B x 10
//               loads, then B x 4 stores (per-block bursts, no clock)
//   plain phased  plain, its loads started inside a read window of a clock period P
//               and its stores inside the write window after it
//   phased<B>   batch<B>, each batch's loads start inside a read window and its
//               stores inside the following write window of a clock period P
//               (read fraction f of P)
//
// GB/s = algorithmic bytes / kernel time (HIP events, mean of 3 launches after one).
// Usage: membench11 [stripes]   (default 6553)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load((GlobalCU4*)p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, (GlobalU4*)p); }

constexpr int K = 10, M = 4;
constexpr size_t S = size_t(1) << 20;
constexpr size_t PITCH = S / 16;         // u32x4 per shard
constexpr uint32_t CHUNKS = S / 16 / 256;  // 4 KiB pieces per shard

struct Args {
    const u32x4* data;
    u32x4* par;
    uint32_t npieces;
    uint32_t mode;     // 0 plain, 1 reads only, 2 writes only
    uint64_t pmask;    // period - 1 (ticks, power of two)
    uint64_t rwin;     // read window length (ticks)
};

__device__ __forceinline__ void piece_io(const Args& a, uint32_t q, u32x4 acc[M]) {
    const size_t s = q / CHUNKS, col = size_t(q % CHUNKS) * 256 + threadIdx.x;
#pragma unroll
    for (int t = 0; t < M; ++t) acc[t] = u32x4{0u, 0u, 0u, (unsigned)t};
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld(a.data + (s * K + j) * PITCH + col);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int t = 0; t < M; ++t) acc[t] ^= x[j] << ((t + j) & 7);
}

__device__ __forceinline__ void piece_store(const Args& a, uint32_t q, const u32x4 acc[M]) {
    const size_t s = q / CHUNKS, col = size_t(q % CHUNKS) * 256 + threadIdx.x;
#pragma unroll
    for (int t = 0; t < M; ++t) st(a.par + (s * M + t) * PITCH + col, acc[t]);
}

__device__ __forceinline__ void wait_window(uint64_t pmask, uint64_t lo, uint64_t hi) {
    for (;;) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime() & pmask;
        if (t >= lo && t < hi) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

__global__ __launch_bounds__(256) void plain(Args a) {
    const uint32_t q = blockIdx.x;
    u32x4 acc[M];
    if (a.mode == 3) {  // the encode's shape, loads in a read window, stores in a write window
        wait_window(a.pmask, 0, a.rwin);
        piece_io(a, q, acc);
        wait_window(a.pmask, a.rwin, a.pmask + 1);
        piece_store(a, q, acc);
        return;
    }
    if (a.mode == 2) {
#pragma unroll
        for (int t = 0; t < M; ++t) acc[t] = u32x4{q, 1u, 2u, (unsigned)t};
        piece_store(a, q, acc);
        return;
    }
    piece_io(a, q, acc);
    if (a.mode == 1) {
        if (acc[0].x == 0x9E3779B9u && acc[1].y == 0x7F4A7C15u) piece_store(a, q, acc);  // never
        return;
    }
    piece_store(a, q, acc);
}

__global__ void clockprobe(uint64_t* t) {
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

template <int B, bool kPhased>
__global__ __launch_bounds__(256) void batched(Args a) {
    for (uint32_t base = blockIdx.x * B; base < a.npieces; base += gridDim.x * B) {
        if (kPhased) wait_window(a.pmask, 0, a.rwin);
        u32x4 acc[B][M];
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (base + b < a.npieces) piece_io(a, base + b, acc[b]);
        if (kPhased) wait_window(a.pmask, a.rwin, a.pmask + 1);
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (base + b < a.npieces) piece_store(a, base + b, acc[b]);
    }
}

int main(int argc, char** argv) {
    const int stripes = argc > 1 ? atoi(argv[1]) : 6553;
    u32x4 *data, *par;
    CK(hipMalloc(&data, stripes * K * S));
    CK(hipMalloc(&par, stripes * M * S));
    CK(hipMemset(data, 1, stripes * K * S));
    CK(hipMemset(par, 2, stripes * M * S));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const uint32_t npieces = uint32_t(stripes) * CHUNKS;
    const double enc_bytes = double(stripes) * (K + M) * S;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](auto launch, double bytes, const char* name) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 3;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-44s %8.3f ms %8.1f GB/s\n", name, ms, bytes / ms / 1e6);
        fflush(stdout);
    };
    Args a{data, par, npieces, 0, 0, 0};
    char name[128];
    auto run_plain = [&](uint32_t mode, double bytes, const char* name) {
        Args b = a;
        b.mode = mode;
        time([&] { hipLaunchKernelGGL(plain, dim3(npieces), dim3(256), 0, 0, b); }, bytes, name);
    };
    auto run_batched = [&](auto kern, int B, bool phased, uint64_t period, double frac) {
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0));
        const uint32_t grid = uint32_t(prop.multiProcessorCount * per_cu);
        Args b = a;
        b.pmask = period ? period - 1 : 0;
        b.rwin = uint64_t(frac * double(period));
        if (phased)
            snprintf(name, sizeof name, "phased<%d> P=%.1fus f=%.2f (%u blk)", B, period / 100.0, frac, grid);
        else
            snprintf(name, sizeof name, "batch<%d> (%u blocks)", B, grid);
        time([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, b); }, enc_bytes, name);
    };
    {  // is the constant clock one clock for the chip?  blocks go to XCDs round-robin
        uint64_t* d_t;
        CK(hipMalloc(&d_t, 64 * sizeof(uint64_t)));
        hipLaunchKernelGGL(clockprobe, dim3(64), dim3(64), 0, 0, d_t);
        std::vector<uint64_t> t(64);
        CK(hipMemcpy(t.data(), d_t, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        uint64_t lo = t[0];
        for (uint64_t v : t) lo = v < lo ? v : lo;
        printf("clock probe (block start - earliest, ticks of 10 ns, block b on XCD b %% 8):");
        for (int b = 0; b < 64; ++b) printf("%s%llu", b % 8 ? " " : "\n  ", (unsigned long long)(t[b] - lo));
        printf("\n");
        CK(hipFree(d_t));
    }
    for (int rep = 0; rep < 2; ++rep) {
        run_plain(0, enc_bytes, "plain (encode shape)");
        run_plain(1, double(stripes) * K * S, "reads only (10 per stripe)");
        run_plain(2, double(stripes) * M * S, "writes only (4 per stripe)");
        for (uint64_t period : {32u, 64u, 128u, 256u, 512u})
            for (double f : {0.6, 0.7, 0.8}) {
                Args b = a;
                b.mode = 3;
                b.pmask = period - 1;
                b.rwin = uint64_t(f * double(period));
                snprintf(name, sizeof name, "plain phased P=%.2fus f=%.2f", period / 100.0, f);
                time([&] { hipLaunchKernelGGL(plain, dim3(npieces), dim3(256), 0, 0, b); }, enc_bytes, name);
            }
        run_batched(batched<2, false>, 2, false, 0, 0);
        for (uint64_t period : {256u, 2048u})
            run_batched(batched<2, true>, 2, true, period, 0.7);
        run_batched(batched<4, true>, 4, true, 2048u, 0.7);
    }
    return 0;
}
