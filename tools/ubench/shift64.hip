// shift64.hip -- issue rate of v_lshlrev_b64 against v_lshlrev_b32 and
// v_bfi_b32 on gfx950 (8 independent chains per lane, 2 waves per SIMD):
// could the bit-plane transpose shift two words per instruction?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters) {
    uint32_t a[8];
    uint64_t b[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3); b[i] = (uint64_t(a[i]) << 32) | (a[i] ^ 0x55u); }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(a[i]));
            if constexpr (KIND == 1) asm volatile("v_lshlrev_b64 %0, 4, %0" : "+v"(b[i]));
            if constexpr (KIND == 2) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            if constexpr (KIND == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
        }
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i] ^ uint32_t(b[i]) ^ uint32_t(b[i] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    uint32_t* out;
    const int blocks = 256 * 8, iters = 4096;  // 8 waves per CU = 2 per SIMD
    CK(hipMalloc(&out, blocks * 256 * 4));
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    const char* names[4] = {"v_lshlrev_b32", "v_lshlrev_b64", "v_bfi_b32", "v_bitop3_b32"};
    for (int rep = 0; rep < 2; ++rep)
        for (int kind = 0; kind < 4; ++kind) {
            CK(hipEventRecord(s));
            if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
            if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters);
            CK(hipEventRecord(e));
            CK(hipEventSynchronize(e));
            float ms;
            CK(hipEventElapsedTime(&ms, s, e));
            const double winstr = double(blocks) * 4 * iters * 8;  // wave-instructions
            printf("%-14s %.3f ms  %.2f wave-instr per SIMD per ns\n", names[kind], ms, winstr / 1024 / (ms * 1e6));
        }
    return 0;
}
