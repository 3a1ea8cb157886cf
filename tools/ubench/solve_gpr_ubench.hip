// solve_gpr_ubench.hip -- micro-benchmark of the config-5 syndrome solve:
//   split: byte domain, split-table v_perm MAC (the shipped kernel's method)
//   gpr:   bit planes; the 32 four-Russians combinations of a syndrome's planes
//          sit in v224..v255 and each output plane takes two GPR-indexed XORs
//          (s_set_gpr_idx_on + v_xor_b32 with an indexed SRC0), the indices
//          read by s_load_dwordx16 from a 16 KiB constant table indexed by the
//          coefficient (IDX[c][16]: lo/hi combination of output plane q).
// Same work per pass (R outputs x T syndromes x 32 bytes per lane); checks
// that both give the same bytes (planes transposed on the host side).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"

#ifndef R_OUT
#define R_OUT 4
#endif
#ifndef T_SYN
#define T_SYN 16
#endif
constexpr int R = R_OUT, T = T_SYN;

typedef const __attribute__((address_space(4))) uint32_t CU32;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
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

#define GI(k) "s_set_gpr_idx_on %[i" #k "], gpr_idx(SRC0)\n\t"
#define PLANE(q, k0, k1) GI(k0) "v_xor_b32 %[a" #q "], v224, %[a" #q "]\n\t" GI(k1) "v_xor_b32 %[a" #q "], v240, %[a" #q "]\n\t"

// acc (8 planes) ^= c * syndrome, the syndrome's combinations in v224..v255.
__device__ __forceinline__ void gpr_mac(uint32_t (&a)[8], const uint32_t (&c)[32], CU32* ix) {
    asm volatile(PLANE(0, 0, 1) PLANE(1, 2, 3) PLANE(2, 4, 5) PLANE(3, 6, 7) PLANE(4, 8, 9) PLANE(5, 10, 11)
                     PLANE(6, 12, 13) PLANE(7, 14, 15) "s_set_gpr_idx_off"
                 : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]),
                   [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7])
                 : [i0] "s"(ix[0]), [i1] "s"(ix[1]), [i2] "s"(ix[2]), [i3] "s"(ix[3]), [i4] "s"(ix[4]),
                   [i5] "s"(ix[5]), [i6] "s"(ix[6]), [i7] "s"(ix[7]), [i8] "s"(ix[8]), [i9] "s"(ix[9]),
                   [i10] "s"(ix[10]), [i11] "s"(ix[11]), [i12] "s"(ix[12]), [i13] "s"(ix[13]), [i14] "s"(ix[14]),
                   [i15] "s"(ix[15]),
                   "{v224}"(c[0]), "{v225}"(c[1]), "{v226}"(c[2]), "{v227}"(c[3]), "{v228}"(c[4]), "{v229}"(c[5]),
                   "{v230}"(c[6]), "{v231}"(c[7]), "{v232}"(c[8]), "{v233}"(c[9]), "{v234}"(c[10]), "{v235}"(c[11]),
                   "{v236}"(c[12]), "{v237}"(c[13]), "{v238}"(c[14]), "{v239}"(c[15]), "{v240}"(c[16]),
                   "{v241}"(c[17]), "{v242}"(c[18]), "{v243}"(c[19]), "{v244}"(c[20]), "{v245}"(c[21]),
                   "{v246}"(c[22]), "{v247}"(c[23]), "{v248}"(c[24]), "{v249}"(c[25]), "{v250}"(c[26]),
                   "{v251}"(c[27]), "{v252}"(c[28]), "{v253}"(c[29]), "{v254}"(c[30]), "{v255}"(c[31]));
}

__device__ __forceinline__ void combos16(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3, uint32_t* c) {
    c[0] = 0u; c[1] = p0; c[2] = p1; c[3] = p0 ^ p1;
    c[4] = p2; c[5] = p2 ^ p0; c[6] = p2 ^ p1; c[7] = p2 ^ c[3];
    c[8] = p3;
#pragma unroll
    for (int i = 1; i < 8; ++i) c[8 + i] = p3 ^ c[i];
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gpr_kernel(uint32_t* out, const uint8_t* coefs, const uint32_t* idxtab, int iters) {
    const uint32_t tid = threadIdx.x + blockIdx.x * 256;
    uint32_t syn[T][8];
#pragma unroll
    for (int s = 0; s < T; ++s)
#pragma unroll
        for (int w = 0; w < 8; ++w) syn[s][w] = (tid * 0x9E3779B9u) ^ (s * 131u + w * 7919u);
    uint32_t acc[R][8] = {};
    CU32* cf = (CU32*)coefs;  // coefficient bytes, 4 per dword (scalar loads)
    CU32* tab = (CU32*)idxtab;
    auto coef = [&](int i) { return (cf[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < T; ++s) {
            asm volatile("" : "+v"(syn[s][0]), "+v"(syn[s][1]), "+v"(syn[s][2]), "+v"(syn[s][3]), "+v"(syn[s][4]),
                         "+v"(syn[s][5]), "+v"(syn[s][6]), "+v"(syn[s][7]));
            uint32_t c[32];
            combos16(syn[s][0], syn[s][1], syn[s][2], syn[s][3], c);
            combos16(syn[s][4], syn[s][5], syn[s][6], syn[s][7], c + 16);
#pragma unroll
            for (int r = 0; r < R; ++r) gpr_mac(acc[r], c, tab + coef(r * T + s) * 16u);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) out[(r * 8 + w) * (gridDim.x * 256) + tid] = acc[r][w];
}

// ---- host reference ----
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (a & 0x80) ? (uint8_t)((a << 1) ^ 0x1D) : (uint8_t)(a << 1);
        b >>= 1;
    }
    return r;
}
static void split_tables(uint8_t c, uint32_t* w) {
    auto pack = [&](int base, int step) {
        uint32_t r = 0;
        for (int i = 0; i < 4; ++i) r |= (uint32_t)gmul(c, (uint8_t)(base + i * step)) << (8 * i);
        return r;
    };
    w[0] = pack(0, 1); w[1] = pack(4, 1); w[2] = pack(0, 8); w[3] = pack(32, 8); w[4] = pack(0, 64);
}

int main() {
    const int blocks = 4096, iters = 15;
    const size_t nout = size_t(blocks) * 256 * R * 8;
    uint32_t *out1, *out2, *tabs, *idx;
    uint8_t* cf;
    hipMalloc(&out1, nout * 4);
    hipMalloc(&out2, nout * 4);
    hipMalloc(&tabs, R * T * 5 * 4);
    hipMalloc(&idx, 256 * 16 * 4);
    hipMalloc(&cf, R * T);
    std::vector<uint8_t> hc(R * T);
    for (int i = 0; i < R * T; ++i) hc[i] = (uint8_t)(i * 37 + 11);
    std::vector<uint32_t> ht(R * T * 5), hi(256 * 16);
    for (int r = 0; r < R; ++r)
        for (int s = 0; s < T; ++s) split_tables(hc[r * T + s], &ht[(r * T + s) * 5]);
    for (int c = 0; c < 256; ++c) {
        uint8_t col[8];
        for (int p = 0; p < 8; ++p) col[p] = gmul((uint8_t)c, (uint8_t)(1u << p));
        for (int q = 0; q < 8; ++q) {
            uint32_t s1 = 0, s2 = 0;
            for (int p = 0; p < 4; ++p) s1 |= ((col[p] >> q) & 1u) << p;
            for (int p = 4; p < 8; ++p) s2 |= ((col[p] >> q) & 1u) << (p - 4);
            hi[c * 16 + 2 * q] = s1;
            hi[c * 16 + 2 * q + 1] = s2;
        }
    }
    hipMemcpy(tabs, ht.data(), ht.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(cf, hc.data(), hc.size(), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        float ms_s = 0, ms_g = 0;
        hipEventRecord(a);
        hipLaunchKernelGGL(split_kernel, dim3(blocks), dim3(256), 0, 0, out1, tabs, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_s, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(gpr_kernel, dim3(blocks), dim3(256), 0, 0, out2, cf, idx, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms_g, a, b);
        const double pairs = double(blocks) * 4 * iters * R * T;  // wave-pairs
        std::printf("R=%d T=%d  split %.3f ms (%.1f ns/wave-pair)   gpr %.3f ms (%.1f ns/wave-pair)   gpr/split %.3f\n", R, T, ms_s,
                    ms_s * 1e6 / pairs * 1024, ms_g, ms_g * 1e6 / pairs * 1024, ms_g / ms_s);
    }
    // check: split output (bytes) vs gpr output (planes) -> transpose planes to bytes on the host
    std::vector<uint32_t> o1(nout), o2(nout);
    hipMemcpy(o1.data(), out1, nout * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o2.data(), out2, nout * 4, hipMemcpyDeviceToHost);
    // planes: for a lane, plane p holds bit p of byte (w, b) at bit position 8b + w? Here the syndromes are
    // synthetic words treated as planes by the gpr kernel and as bytes by the split kernel, so compare
    // through a host model of each instead: recompute gpr on the host for a few lanes.
    const size_t L = size_t(blocks) * 256;
    long bad = 0;
    for (size_t tid = 0; tid < L; tid += 997) {
        uint32_t syn[T][8];
        for (int s = 0; s < T; ++s)
            for (int w = 0; w < 8; ++w) syn[s][w] = ((uint32_t)tid * 0x9E3779B9u) ^ (s * 131u + w * 7919u);
        for (int r = 0; r < R; ++r) {
            uint32_t accp[8] = {}, accb[8] = {};
            for (int s = 0; s < T; ++s) {
                const uint8_t c = hc[r * T + s];
                for (int q = 0; q < 8; ++q)
                    for (int p = 0; p < 8; ++p)
                        if ((gmul(c, (uint8_t)(1u << p)) >> q) & 1u) accp[q] ^= syn[s][p];
                for (int w = 0; w < 8; ++w)
                    for (int by = 0; by < 4; ++by)
                        accb[w] ^= (uint32_t)gmul(c, (uint8_t)(syn[s][w] >> (8 * by))) << (8 * by);
            }
            for (int w = 0; w < 8; ++w) {
                const uint32_t e1 = (iters % 2) ? accb[w] : 0u, e2 = (iters % 2) ? accp[w] : 0u;
                if (o1[(r * 8 + w) * L + tid] != e1) ++bad;
                if (o2[(r * 8 + w) * L + tid] != e2) ++bad;
            }
        }
    }
    std::printf("check: %ld mismatches\n", bad);
    return (hipGetLastError() == hipSuccess && bad == 0) ? 0 : 1;
}
