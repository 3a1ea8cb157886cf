// solve_ubench.hip -- micro-benchmark of the syndrome solve's inner product
// (4 outputs x 16 syndromes per pass, 32 bytes per lane), VALU only:
//   split: byte domain, split-table v_perm MAC (the shipped kernel's method)
//   gpr:   bit-plane domain, four-Russians combos of each syndrome selected by
//          wave-uniform indices (s_set_gpr_idx), one v_bitop3 per output plane
// Same work per pass; time per pass per wave is what matters.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

typedef const __attribute__((address_space(4))) uint32_t CU32;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ void combos(const uint32_t* p, uint32_t* c) {
    c[0] = 0; c[1] = p[0]; c[2] = p[1]; c[3] = p[0] ^ p[1];
    c[4] = p[2]; c[5] = p[2] ^ p[0]; c[6] = p[2] ^ p[1]; c[7] = p[2] ^ c[3];
    c[8] = p[3];
#pragma unroll
    for (int i = 1; i < 8; ++i) c[8 + i] = p[3] ^ c[i];
}

constexpr int R = 4, T = 8;

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void split_kernel(uint32_t* out, const uint32_t* tabs, int iters) {
    __shared__ uint32_t mtab[R][T][5];
    for (int i = threadIdx.x; i < R * T * 5; i += 256) (&mtab[0][0][0])[i] = tabs[i];
    __syncthreads();
    const uint32_t tid = threadIdx.x + blockIdx.x * 256;
    uint32_t syn[T][8];
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int w = 0; w < 8; ++w) syn[s][w] = (tid * 0x9E3779B9u) ^ (s * 131u + w * 7919u);
    uint32_t acc[R][8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            asm volatile("" : "+v"(syn[s][0]), "+v"(syn[s][1]), "+v"(syn[s][2]), "+v"(syn[s][3]), "+v"(syn[s][4]),
                         "+v"(syn[s][5]), "+v"(syn[s][6]), "+v"(syn[s][7]));
            uint32_t Tb[R][5];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < 5; ++i) Tb[r][i] = mtab[r][s][i];
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const uint32_t x = syn[s][w];
                const uint32_t a = x & 0x07070707u, b = (x >> 3) & 0x07070707u, c = (x >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t la = __builtin_amdgcn_perm(Tb[r][1], Tb[r][0], a);
                    const uint32_t lb = __builtin_amdgcn_perm(Tb[r][3], Tb[r][2], b);
                    const uint32_t lc = __builtin_amdgcn_perm(Tb[r][4], Tb[r][4], c);
                    acc[r][w] = xor3(acc[r][w], la, lb) ^ lc;
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) out[(r * 8 + w) * (gridDim.x * 256) + tid] = acc[r][w];
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gpr_kernel(uint32_t* out, const uint32_t* idx, int iters) {
    const uint32_t tid = threadIdx.x + blockIdx.x * 256;
    uint32_t syn[T][8];
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int w = 0; w < 8; ++w) syn[s][w] = (tid * 0x9E3779B9u) ^ (s * 131u + w * 7919u);
    uint32_t acc[R][8] = {};
    CU32* ix = (CU32*)(idx);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            asm volatile("" : "+v"(syn[s][0]), "+v"(syn[s][1]), "+v"(syn[s][2]), "+v"(syn[s][3]), "+v"(syn[s][4]),
                         "+v"(syn[s][5]), "+v"(syn[s][6]), "+v"(syn[s][7]));
            uint32_t c[32];
            combos(&syn[s][0], c);
            combos(&syn[s][4], c + 16);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                CU32* q = ix + (r * T + s) * 16;
#pragma unroll
                for (int p = 0; p < 8; ++p) acc[r][p] = xor3(acc[r][p], c[q[2 * p]], c[q[2 * p + 1]]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) out[(r * 8 + w) * (gridDim.x * 256) + tid] = acc[r][w];
}

int main() {
    const int blocks = 2048, iters = 64;
    uint32_t *out, *tabs, *idx;
    hipMalloc(&out, size_t(blocks) * 256 * R * 8 * 4);
    hipMalloc(&tabs, R * T * 5 * 4);
    hipMalloc(&idx, R * T * 16 * 4);
    std::vector<uint32_t> ht(R * T * 5), hi(R * T * 16);
    for (size_t i = 0; i < ht.size(); ++i) ht[i] = 0x01234567u * (i + 3);
    for (size_t i = 0; i < hi.size(); ++i) hi[i] = (i % 2 ? 16 : 0) + (i * 7) % 16;
    hipMemcpy(tabs, ht.data(), ht.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        float ms_s = 0, ms_g = 0;
        hipEventRecord(a);
        hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, 0, out, tabs, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_s, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(gpr_kernel, dim3(blocks), dim3(256), 0, 0, out, idx, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_g, a, b);
        const double pairs = double(blocks) * 4 * iters * R * T;  // wave-pairs
        std::printf("split %.3f ms (%.1f ns/wave-pair)   gpr %.3f ms (%.1f ns/wave-pair)   gpr/split %.3f\n", ms_s,
                    ms_s * 1e6 / pairs * 1024, ms_g, ms_g * 1e6 / pairs * 1024, ms_g / ms_s);
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
