// valu_rates64.hip -- issue rates of the BLAKE2b kernel's building blocks on
// gfx950 (as valu_rates.hip): 64-bit add forms, DPP moves, alignbit.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, uint32_t m0) {
    uint64_t a[8];
    uint32_t b[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3) + blockIdx.x; b[i] = uint32_t(a[i]) ^ 0x1234u; }
    uint64_t c = m0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (KIND == 0) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(c));
            if constexpr (KIND == 1) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(b[i]) : "v"(m0) : "vcc");
            if constexpr (KIND == 2) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(b[i]));
            if constexpr (KIND == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(b[i]) : "v"(m0));
            if constexpr (KIND == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b[i]) : "v"(m0));
        }
    }
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r ^= uint32_t(a[i]) ^ b[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int KIND> float run(uint32_t* out, int blocks, int iters) {
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x0F0F0F0Fu);
    hipEventRecord(s);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x0F0F0F0Fu);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    return ms;
}

int main() {
    uint32_t* out;
    const int blocks = 256 * 2, iters = 8192;
    CK(hipMalloc(&out, blocks * 256 * 4));
    const char* names[] = {"v_lshl_add_u64", "v_add_co_u32", "v_mov_b32_dpp", "v_alignbit_b32", "v_xor_b32"};
    float ms[5] = {run<0>(out, blocks, iters), run<1>(out, blocks, iters), run<2>(out, blocks, iters),
                   run<3>(out, blocks, iters), run<4>(out, blocks, iters)};
    const double winstr = double(blocks) * 4 * iters * 8;
    for (int i = 0; i < 5; ++i)
        printf("%-16s %.3f ms  %.3f wave-instr per SIMD per ns\n", names[i], ms[i], winstr / 1024 / (ms[i] * 1e6));
    return 0;
}
