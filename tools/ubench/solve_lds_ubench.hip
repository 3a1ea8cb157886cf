// solve_lds_ubench.hip -- micro-benchmark of the syndrome solve's inner
// product, split-table MAC (the shipped kernel's method) against a bit-plane
// solve whose four-Russians combinations live in LDS:
//   split: byte domain, 3 v_perm + xor3 + xor per (output, syndrome, word);
//   lds:   per syndrome, its 2 x 16 plane combinations are written to the
//          wave's own 8 KiB of LDS (32 ds_write_b32), then every output plane
//          is acc ^= lds[lo] ^ lds[hi] with wave-uniform lo/hi (one v_add per
//          address, two ds_read_b32, one v_bitop3): 24 VALU + 16 LDS reads per
//          (output, syndrome) pair instead of 40 VALU (24 of them v_perm).
// R outputs x T syndromes per pass, 32 bytes per lane, 2 waves per SIMD
// (the shipped kernel's occupancy).  Prints ns per wave-pair of each and the
// ratio; the outputs of both are checked equal (same coefficients).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

typedef const __attribute__((address_space(4))) uint32_t CU32;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

constexpr int R = 8, T = 8;

// GF(2^8) 0x11D
__host__ __device__ inline uint32_t xt(uint32_t v) { return ((v << 1) ^ ((v & 0x80u) ? 0x1Du : 0u)) & 0xFFu; }
__host__ __device__ inline uint32_t gmul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if ((b >> i) & 1u) r ^= a;
        a = xt(a);
    }
    return r;
}

// 8 words of 4 bytes <-> 8 bit planes (plane p = bit p of each byte), the
// kernel's delta-swap transpose in its plain form.
__device__ __forceinline__ void swp(uint32_t& a, uint32_t& b, int s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}
__device__ __forceinline__ void to_planes(uint32_t* w) {
    for (int i = 0; i < 4; ++i) swp(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
    for (int i : {0, 1, 4, 5}) swp(w[i], w[i + 2], 2, 0x33333333u);
    for (int i : {0, 2, 4, 6}) swp(w[i], w[i + 1], 1, 0x55555555u);
}
__device__ __forceinline__ void from_planes(uint32_t* w) {
    for (int i : {0, 2, 4, 6}) swp(w[i], w[i + 1], 1, 0x55555555u);
    for (int i : {0, 1, 4, 5}) swp(w[i], w[i + 2], 2, 0x33333333u);
    for (int i = 0; i < 4; ++i) swp(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
}

__device__ __forceinline__ uint32_t seed_word(uint32_t tid, int s, int w) {
    uint32_t x = tid * 0x9E3779B9u ^ (s * 0x85EBCA6Bu + w * 0xC2B2AE35u);
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    return x ^ (x >> 12);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void split_kernel(uint32_t* out, const uint32_t* tabs, int iters) {
    __shared__ uint32_t mtab[R][T][5];
    for (int i = threadIdx.x; i < R * T * 5; i += 256) (&mtab[0][0][0])[i] = tabs[i];
    __syncthreads();
    const uint32_t tid = threadIdx.x + blockIdx.x * 256;
    uint32_t syn[T][8];
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int w = 0; w < 8; ++w) syn[s][w] = seed_word(tid, s, w);
    uint32_t acc[R][8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            asm volatile("" : "+v"(syn[s][0]), "+v"(syn[s][1]), "+v"(syn[s][2]), "+v"(syn[s][3]), "+v"(syn[s][4]),
                         "+v"(syn[s][5]), "+v"(syn[s][6]), "+v"(syn[s][7]));
#pragma unroll
            for (int r0 = 0; r0 < R; r0 += 4) {
                uint32_t Tb[4][5];
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int i = 0; i < 5; ++i) Tb[r][i] = mtab[r0 + r][s][i];
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    const uint32_t x = syn[s][w];
                    const uint32_t a = x & 0x07070707u, b = (x >> 3) & 0x07070707u, c = (x >> 6) & 0x03030303u;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t la = __builtin_amdgcn_perm(Tb[r][1], Tb[r][0], a);
                        const uint32_t lb = __builtin_amdgcn_perm(Tb[r][3], Tb[r][2], b);
                        const uint32_t lc = __builtin_amdgcn_perm(Tb[r][4], Tb[r][4], c);
                        acc[r0 + r][w] = xor3(acc[r0 + r][w], la, lb) ^ lc;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) out[(r * 8 + w) * (gridDim.x * 256) + tid] = acc[r][w];
}

// idx[(r * T + s) * 16 + 2p + h]: combination index (0..15) of output plane p
// for coefficient (r, s), half h (planes 0-3 / 4-7), in dwords (x 64 lanes)
// and offset by 16 combinations for h = 1.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void lds_kernel(uint32_t* out, const uint32_t* idx, int iters) {
    __shared__ uint32_t comb[4][32][64];  // per wave: 32 combinations x 64 lanes
    const uint32_t tid = threadIdx.x + blockIdx.x * 256;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t* my = &comb[wave][0][lane];
    typedef __attribute__((address_space(3))) const uint32_t LdsU32;
    LdsU32* lp = (LdsU32*)(&comb[wave][0][lane]);
    uint32_t syn[T][8];
#pragma unroll
    for (int s = 0; s < T; ++s) {
#pragma unroll
        for (int w = 0; w < 8; ++w) syn[s][w] = seed_word(tid, s, w);
        to_planes(syn[s]);
    }
    uint32_t acc[R][8] = {};
    CU32* ix = (CU32*)(idx);
    for (int it = 0; it < iters; ++it) {
#pragma unroll 1
        for (int s = 0; s < T; ++s) {
            uint32_t p[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) p[w] = syn[0][w];
            // (a runtime syndrome index keeps the loop rolled; select by s)
#pragma unroll
            for (int u = 1; u < T; ++u)
                if (s == u)
#pragma unroll
                    for (int w = 0; w < 8; ++w) p[w] = syn[u][w];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t* q = p + 4 * h;
                uint32_t c[16];
                c[0] = 0u; c[1] = q[0]; c[2] = q[1]; c[3] = q[0] ^ q[1];
                c[4] = q[2]; c[5] = q[2] ^ q[0]; c[6] = q[2] ^ q[1]; c[7] = q[2] ^ c[3];
                c[8] = q[3];
#pragma unroll
                for (int i = 1; i < 8; ++i) c[8 + i] = q[3] ^ c[i];
#pragma unroll
                for (int i = 0; i < 16; ++i) my[(16 * h + i) * 64] = c[i];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < R; ++r) {
                CU32* qi = ix + (r * T + s) * 16;
#pragma unroll
                for (int pl = 0; pl < 8; ++pl) {
                    const uint32_t vlo = lp[qi[2 * pl]];
                    const uint32_t vhi = lp[qi[2 * pl + 1]];
                    acc[r][pl] = xor3(acc[r][pl], vlo, vhi);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        from_planes(acc[r]);
#pragma unroll
        for (int w = 0; w < 8; ++w) out[(r * 8 + w) * (gridDim.x * 256) + tid] = acc[r][w];
    }
}

int main() {
    const int blocks = 2048, iters = 63;  // odd: the repeated XORs leave one pass's sum
    uint32_t *out_s, *out_l, *tabs, *idx;
    const size_t outw = size_t(blocks) * 256 * R * 8;
    hipMalloc(&out_s, outw * 4);
    hipMalloc(&out_l, outw * 4);
    hipMalloc(&tabs, R * T * 5 * 4);
    hipMalloc(&idx, R * T * 16 * 4);
    // coefficients, their split tables and their plane-combination indices
    std::vector<uint32_t> coef(R * T), ht(R * T * 5), hi(R * T * 16);
    for (int i = 0; i < R * T; ++i) coef[i] = 1 + (i * 37 + 11) % 255;
    for (int r = 0; r < R; ++r)
        for (int s = 0; s < T; ++s) {
            const uint32_t c = coef[r * T + s];
            auto tb = [&](uint32_t base, uint32_t step, int n) {
                uint32_t v = 0;
                for (int i = 0; i < n; ++i) v |= gmul(c, base + i * step) << (8 * i);
                return v;
            };
            uint32_t* t = &ht[(r * T + s) * 5];
            t[0] = tb(0, 1, 4); t[1] = tb(4, 1, 4);   // bits 0-2
            t[2] = tb(0, 8, 4); t[3] = tb(32, 8, 4);  // bits 3-5
            t[4] = tb(0, 64, 4);                      // bits 6-7
            for (int q = 0; q < 8; ++q) {
                int lo = 0, hi4 = 0;
                for (int p = 0; p < 4; ++p) lo |= ((gmul(c, 1u << p) >> q) & 1) << p;
                for (int p = 4; p < 8; ++p) hi4 |= ((gmul(c, 1u << p) >> q) & 1) << (p - 4);
                hi[(r * T + s) * 16 + 2 * q] = lo * 64;  // in dwords: combination x 64 lanes
                hi[(r * T + s) * 16 + 2 * q + 1] = (16 + hi4) * 64;
            }
        }
    hipMemcpy(tabs, ht.data(), ht.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        float ms_s = 0, ms_l = 0;
        hipEventRecord(a);
        hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, 0, out_s, tabs, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_s, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(lds_kernel, dim3(blocks), dim3(256), 0, 0, out_l, idx, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_l, a, b);
        const double pairs = double(blocks) * 4 * iters * R * T;  // wave-pairs
        std::printf("split %.3f ms (%.2f ns/wave-pair x 1024 SIMDs)   lds %.3f ms (%.2f)   lds/split %.3f\n", ms_s,
                    ms_s * 1e6 / pairs * 1024, ms_l, ms_l * 1e6 / pairs * 1024, ms_l / ms_s);
    }
    std::vector<uint32_t> hs(outw), hl(outw);
    hipMemcpy(hs.data(), out_s, outw * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hl.data(), out_l, outw * 4, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < outw; ++i) bad += hs[i] != hl[i];
    std::printf("outputs equal: %s (%zu of %zu words differ)\n", bad ? "NO" : "yes", bad, outw);
    return (hipGetLastError() == hipSuccess && !bad) ? 0 : 1;
}
