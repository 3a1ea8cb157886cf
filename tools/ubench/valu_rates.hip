// valu_rates.hip -- issue rate of the integer VALU instructions the bit-sliced
// kernels are made of, on gfx950: 8 independent self-dependent chains per
// lane, 8 waves per CU (2 per SIMD, like the kernels).  Reported as
// wave-instructions per SIMD per ns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

#define BODY(INS) asm volatile(INS : "+v"(a[i]) : "v"(m0), "v"(m1))
template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, uint32_t m0, uint32_t m1) {
    uint32_t a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * (i + 3) + blockIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) BODY("v_xor_b32 %0, %0, %1");
            if constexpr (KIND == 1) BODY("v_and_b32 %0, %0, %1");
            if constexpr (KIND == 2) BODY("v_lshlrev_b32 %0, 4, %0");
            if constexpr (KIND == 3) BODY("v_lshrrev_b32 %0, 4, %0");
            if constexpr (KIND == 4) BODY("v_bfi_b32 %0, %1, %0, %2");
            if constexpr (KIND == 5) BODY("v_bitop3_b32 %0, %1, %0, %2 bitop3:0xca");
            if constexpr (KIND == 6) BODY("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96");
            if constexpr (KIND == 7) BODY("v_perm_b32 %0, %1, %2, %0");
            if constexpr (KIND == 8) BODY("v_alignbit_b32 %0, %0, %1, 4");
            if constexpr (KIND == 9) BODY("v_lshl_or_b32 %0, %0, 4, %1");
            if constexpr (KIND == 10) BODY("v_and_or_b32 %0, %0, %1, %2");
            if constexpr (KIND == 11) BODY("v_xor_b32_e64 %0, %0, %1");
            if constexpr (KIND == 12) BODY("v_mov_b32 %0, %1");
            if constexpr (KIND == 13) BODY("v_lshlrev_b32 %0, %1, %0");
            if constexpr (KIND == 14) BODY("v_lshlrev_b32_e64 %0, 4, %0");
            if constexpr (KIND == 15) BODY("v_pk_lshlrev_b16 %0, 4, %0");
            if constexpr (KIND == 16) BODY("v_add_u32 %0, %0, %0");
            if constexpr (KIND == 17) BODY("v_lshl_add_u32 %0, %0, 4, %1");
            if constexpr (KIND == 18) BODY("v_lshrrev_b32 %0, %1, %0");
            if constexpr (KIND == 19) BODY("v_or_b32 %0, %0, %1");
            if constexpr (KIND == 20) BODY("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8");
            if constexpr (KIND == 21) BODY("v_pk_mul_lo_u16 %0, %0, 16");
            if constexpr (KIND == 22) BODY("v_mul_u32_u24 %0, %0, 16");
            if constexpr (KIND == 23) BODY("v_add3_u32 %0, %0, %0, %1");
            if constexpr (KIND == 24) BODY("v_pk_add_u16 %0, %0, %0");
        }
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int KIND> float run(uint32_t* out, int blocks, int iters) {
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x0F0F0F0Fu, 0x33333333u);
    hipEventRecord(s);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x0F0F0F0Fu, 0x33333333u);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    return ms;
}

int main() {
    uint32_t* out;
    const int blocks = 256 * 2, iters = 8192;  // 2 blocks of 4 waves per CU = 2 waves per SIMD
    CK(hipMalloc(&out, blocks * 256 * 4));
    const char* names[] = {"v_xor_b32", "v_and_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_bfi_b32", "v_bitop3 (bfi)",
                           "v_bitop3 (xor3)", "v_perm_b32", "v_alignbit_b32", "v_lshl_or_b32", "v_and_or_b32",
                           "v_xor_b32_e64", "v_mov_b32", "v_lshlrev (vgpr amt)", "v_lshlrev_e64", "v_pk_lshlrev_b16",
                           "v_add_u32 x+x", "v_lshl_add_u32", "v_lshrrev (vgpr)", "v_or_b32", "v_bitop3 (maj)",
                           "v_pk_mul_lo_u16", "v_mul_u32_u24", "v_add3_u32", "v_pk_add_u16"};
    float ms[25];
    ms[0] = run<0>(out, blocks, iters); ms[1] = run<1>(out, blocks, iters); ms[2] = run<2>(out, blocks, iters);
    ms[3] = run<3>(out, blocks, iters); ms[4] = run<4>(out, blocks, iters); ms[5] = run<5>(out, blocks, iters);
    ms[6] = run<6>(out, blocks, iters); ms[7] = run<7>(out, blocks, iters); ms[8] = run<8>(out, blocks, iters);
    ms[9] = run<9>(out, blocks, iters); ms[10] = run<10>(out, blocks, iters); ms[11] = run<11>(out, blocks, iters);
    ms[12] = run<12>(out, blocks, iters);
    ms[13] = run<13>(out, blocks, iters); ms[14] = run<14>(out, blocks, iters); ms[15] = run<15>(out, blocks, iters);
    ms[16] = run<16>(out, blocks, iters); ms[17] = run<17>(out, blocks, iters); ms[18] = run<18>(out, blocks, iters);
    ms[19] = run<19>(out, blocks, iters); ms[20] = run<20>(out, blocks, iters);
    ms[21] = run<21>(out, blocks, iters); ms[22] = run<22>(out, blocks, iters); ms[23] = run<23>(out, blocks, iters);
    ms[24] = run<24>(out, blocks, iters);
    const double winstr = double(blocks) * 4 * iters * 8;
    for (int i = 0; i < 25; ++i)
        printf("%-16s %.3f ms  %.3f wave-instr per SIMD per ns\n", names[i], ms[i], winstr / 1024 / (ms[i] * 1e6));
    return 0;
}
