// membench9.hip -- movement-only twin of the RS(10,4) reconstruct.
//
// The headline reconstruct (rs_matmul_kernel K10_MG4, csrc/rs_kernels.hip)
// streams each stripe's 10 survivors and writes its e = 1..4 erased shards
// in place, stripes listed by a descriptor array grouped by pattern, one
// 4 KiB column chunk of one stripe per 256-thread block.  This twin keeps
// exactly that access pattern -- the same descriptors (random 1-4 erasures,
// Rebuild's survivors, pattern-sorted), the same block shape, nt 16-byte
// loads and stores -- and replaces the GF arithmetic by XORs, so its rate is
// the memory system's ceiling for the reconstruct's own shape.  Variants:
//   order:  natural (block b = stripe b / chunks) or a stripe per XCD
//           (xcd.hpp's map: XCD x runs stripes x, x+8, ...), as shipped;
//   sort:   descriptors grouped by pattern (shipped) or in stripe order;
//   fixed:  every stripe 4 erasures (10 reads + 4 writes) / none (10 reads).
// GB/s = algorithmic bytes (10 + e) * S per stripe / kernel time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "../noise-erasurecode-plugin_amd/csrc/xcd.hpp"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load((GlobalCU4*)p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, (GlobalU4*)p); }

constexpr int K = 10, M = 4, N = 14;

struct Pat {
    uint32_t src[K];  // survivor ids
    uint32_t dst[M];  // output ids (e used)
    uint32_t e;
};

// logical block of dispatch slot b: natural, or a stripe per XCD (the
// engine's own map, xcd.hpp)
__device__ __forceinline__ uint32_t logical(uint32_t b, uint32_t G, uint32_t chunks, bool xcd) {
    return xcd ? rsmi::xcd_block(b, chunks, G) : b;
}

__global__ __launch_bounds__(256) void rec(u32x4* __restrict__ data, u32x4* __restrict__ par, size_t pitch,
                                           const uint2* __restrict__ desc, const Pat* __restrict__ pats,
                                           uint32_t chunks, int xcd) {
    const uint32_t L = logical(blockIdx.x, gridDim.x, chunks, xcd != 0);
    const uint2 d = desc[L / chunks];
    const uint32_t chunk = L % chunks;
    const size_t s = __builtin_amdgcn_readfirstlane(d.x);
    const uint32_t pid = __builtin_amdgcn_readfirstlane(d.y);
    const Pat& p = pats[pid];
    const uint32_t e = p.e;
    auto shard = [&](uint32_t id) -> u32x4* {
        return id < K ? data + (s * K + id) * pitch : par + (s * M + (id - K)) * pitch;
    };
    const size_t col = size_t(chunk) * 256 + threadIdx.x;
    u32x4 acc[M];
#pragma unroll
    for (int t = 0; t < M; ++t) acc[t] = u32x4{0u, 0u, 0u, (unsigned)t};
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld(shard(p.src[j]) + col);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int t = 0; t < M; ++t) acc[t] ^= x[j] << ((t + j) & 7);
#pragma unroll
    for (int t = 0; t < M; ++t)
        if (t < (int)e) st(shard(p.dst[t]) + col, acc[t]);
}

// The same with the pattern inlined in a 32-byte descriptor (survivor and
// output ids as bytes): one scalar round trip before the survivor loads
// instead of descriptor -> pattern (the engine's chain).  Measures what
// shortening the prologue's dependent loads could buy.
struct DescX {
    uint32_t s, e;
    uint8_t src[16];
    uint8_t dst[8];
};

__global__ __launch_bounds__(256) void rec_inline(u32x4* __restrict__ data, u32x4* __restrict__ par, size_t pitch,
                                                  const DescX* __restrict__ desc, uint32_t chunks, int xcd) {
    const uint32_t L = logical(blockIdx.x, gridDim.x, chunks, xcd != 0);
    const DescX& d = desc[L / chunks];
    const uint32_t chunk = L % chunks;
    const size_t s = __builtin_amdgcn_readfirstlane(d.s);
    const uint32_t e = __builtin_amdgcn_readfirstlane(d.e);
    auto shard = [&](uint32_t id) -> u32x4* {
        return id < K ? data + (s * K + id) * pitch : par + (s * M + (id - K)) * pitch;
    };
    const size_t col = size_t(chunk) * 256 + threadIdx.x;
    u32x4 acc[M];
#pragma unroll
    for (int t = 0; t < M; ++t) acc[t] = u32x4{0u, 0u, 0u, (unsigned)t};
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld(shard(__builtin_amdgcn_readfirstlane(d.src[j])) + col);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int t = 0; t < M; ++t) acc[t] ^= x[j] << ((t + j) & 7);
#pragma unroll
    for (int t = 0; t < M; ++t)
        if (t < (int)e) st(shard(__builtin_amdgcn_readfirstlane(d.dst[t])) + col, acc[t]);
}

// Rebuild's survivors: slot i takes shard i if present, else the highest remaining.
static Pat make_pat(const std::vector<int>& erased) {
    Pat p{};
    bool present[N], used[N] = {};
    for (int i = 0; i < N; ++i) present[i] = true;
    for (int i : erased) present[i] = false;
    int hi = N - 1;
    for (int i = 0; i < K; ++i) {
        if (present[i] && !used[i]) {
            p.src[i] = i;
            used[i] = true;
            continue;
        }
        while (!present[hi] || used[hi]) --hi;
        p.src[i] = hi;
        used[hi] = true;
    }
    std::vector<int> er = erased;
    std::sort(er.begin(), er.end());
    p.e = er.size();
    for (size_t t = 0; t < er.size(); ++t) p.dst[t] = er[t];
    return p;
}

int main(int argc, char** argv) {
    const int stripes = argc > 1 ? atoi(argv[1]) : 6553;
    const size_t S = size_t(1) << 20;
    const size_t pitch = S / 16;
    const uint32_t chunks = S / 16 / 256;
    u32x4 *data, *par;
    CK(hipMalloc(&data, stripes * K * S));
    CK(hipMalloc(&par, stripes * M * S));
    CK(hipMemset(data, 1, stripes * K * S));
    CK(hipMemset(par, 2, stripes * M * S));
    // patterns: index of every erasure set of 1..4 shards
    std::map<std::vector<int>, uint32_t> idx;
    std::vector<Pat> pats;
    auto pid_of = [&](const std::vector<int>& er) {
        auto it = idx.find(er);
        if (it != idx.end()) return it->second;
        pats.push_back(make_pat(er));
        return idx[er] = uint32_t(pats.size() - 1);
    };
    std::mt19937_64 rng(0xE4A5);
    std::vector<uint32_t> mix(stripes), four(stripes), none(stripes);
    std::vector<int> ids(N);
    double mix_bytes = 0;
    for (int s = 0; s < stripes; ++s) {
        const int e = 1 + rng() % 4;
        for (int i = 0; i < N; ++i) ids[i] = i;
        std::shuffle(ids.begin(), ids.end(), rng);
        std::vector<int> er(ids.begin(), ids.begin() + e);
        std::sort(er.begin(), er.end());
        mix[s] = pid_of(er);
        mix_bytes += double(K + e) * S;
        std::vector<int> er4(ids.begin(), ids.begin() + 4);
        std::sort(er4.begin(), er4.end());
        four[s] = pid_of(er4);
    }
    const uint32_t zero_pat = [&] {
        Pat p = make_pat({});
        p.e = 0;
        pats.push_back(p);
        return uint32_t(pats.size() - 1);
    }();
    for (int s = 0; s < stripes; ++s) none[s] = zero_pat;
    Pat* d_pats;
    CK(hipMalloc(&d_pats, pats.size() * sizeof(Pat)));
    CK(hipMemcpy(d_pats, pats.data(), pats.size() * sizeof(Pat), hipMemcpyHostToDevice));
    uint2* d_desc;
    CK(hipMalloc(&d_desc, stripes * sizeof(uint2)));
    auto run = [&](const std::vector<uint32_t>& pid, bool sorted, int xcd, double bytes, const char* name) {
        std::vector<uint2> desc(stripes);
        for (int s = 0; s < stripes; ++s) desc[s] = make_uint2(s, pid[s]);
        if (sorted)
            std::stable_sort(desc.begin(), desc.end(), [](uint2 a, uint2 b) { return a.y < b.y; });
        CK(hipMemcpy(d_desc, desc.data(), stripes * sizeof(uint2), hipMemcpyHostToDevice));
        const dim3 g(stripes * chunks);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        hipLaunchKernelGGL(rec, g, dim3(256), 0, 0, data, par, pitch, d_desc, d_pats, chunks, xcd);
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(rec, g, dim3(256), 0, 0, data, par, pitch, d_desc, d_pats, chunks, xcd);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("%-34s %-8s %-10s %8.3f ms %8.1f GB/s\n", name, sorted ? "sorted" : "unsorted",
               xcd ? "xcd" : "natural", ms, bytes / ms / 1e6);
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
    };
    DescX* d_descx;
    CK(hipMalloc(&d_descx, stripes * sizeof(DescX)));
    auto run_inline = [&](const std::vector<uint32_t>& pid, int xcd, double bytes, const char* name) {
        std::vector<uint2> order(stripes);
        for (int s = 0; s < stripes; ++s) order[s] = make_uint2(s, pid[s]);
        std::stable_sort(order.begin(), order.end(), [](uint2 a, uint2 b) { return a.y < b.y; });
        std::vector<DescX> dx(stripes);
        for (int i = 0; i < stripes; ++i) {
            const Pat& p = pats[order[i].y];
            DescX& d = dx[i];
            d = DescX{};
            d.s = order[i].x;
            d.e = p.e;
            for (int j = 0; j < K; ++j) d.src[j] = static_cast<uint8_t>(p.src[j]);
            for (int t = 0; t < M; ++t) d.dst[t] = static_cast<uint8_t>(p.dst[t]);
        }
        CK(hipMemcpy(d_descx, dx.data(), stripes * sizeof(DescX), hipMemcpyHostToDevice));
        const dim3 g(stripes * chunks);
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        hipLaunchKernelGGL(rec_inline, g, dim3(256), 0, 0, data, par, pitch, d_descx, chunks, xcd);
        CK(hipDeviceSynchronize());
        const int reps = 5;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(rec_inline, g, dim3(256), 0, 0, data, par, pitch, d_descx, chunks, xcd);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("%-34s %-8s %-10s %8.3f ms %8.1f GB/s\n", name, "inline", xcd ? "xcd" : "natural", ms, bytes / ms / 1e6);
        CK(hipEventDestroy(a));
        CK(hipEventDestroy(b));
    };
    for (int rep = 0; rep < 2; ++rep) {
        run_inline(mix, 1, mix_bytes, "random 1-4 erasures (headline)");
        run(mix, true, 1, mix_bytes, "random 1-4 erasures (headline)");
        run(mix, true, 0, mix_bytes, "random 1-4 erasures (headline)");
        run(mix, false, 1, mix_bytes, "random 1-4 erasures (headline)");
        run(mix, false, 0, mix_bytes, "random 1-4 erasures (headline)");
        run(four, true, 1, double(stripes) * (K + 4) * S, "4 erasures (10 reads + 4 writes)");
        run(none, true, 0, double(stripes) * K * S, "no erasures (10 reads)");
    }
    return 0;
}
