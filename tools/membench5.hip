// membench5.hip -- pure data movement on the RS(10,4) stripe shapes with
// non-temporal loads/stores: how the 10-read / e-write ceiling depends on
// occupancy (waves per SIMD, capped with dynamic LDS), on the bytes each lane
// keeps in flight (1 or 2 16-byte columns per shard) and on a dependent
// descriptor load before the data loads (the reconstruct kernel's prologue).
// Answers whether the reconstruct kernel (e = 1..4 outputs, 4 waves/SIMD) is
// below the movement ceiling of its shape and why.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;
// Compiler-managed nt loads/stores (global_load_dwordx4 ... nt): inline-asm
// loads would leave the waitcnt bookkeeping to hand-written s_waitcnt, and the
// compiler may reuse a register an in-flight load still writes.
__device__ __forceinline__ u32x4 ld(const u32x4* p) { return __builtin_nontemporal_load((GlobalCU4*)p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, (GlobalU4*)p); }

// C columns of 16 B per lane per shard (block covers 256*C columns).
template <int K, int M, int C, bool DEP>
__global__ __launch_bounds__(256) void stripe_k(const u32x4* __restrict__ data, u32x4* __restrict__ par,
                                                size_t pitch, int chunks, const uint2* desc) {
    extern __shared__ int lds_pad[];
    size_t s = blockIdx.x / chunks;
    const int chunk = blockIdx.x % chunks;
    if constexpr (DEP) {
        const uint2 d = desc[s];
        s = __builtin_amdgcn_readfirstlane(d.x);
        if (d.y == 0xFFFFFFFFu) lds_pad[threadIdx.x] = 1;  // never: keeps the LDS allocation
    }
    const u32x4* d = data + s * K * pitch;
    u32x4* p = par + s * (M ? M : 1) * pitch;
    u32x4 x[K][C];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) x[j][c] = ld(d + j * pitch + (size_t(chunk) * C + c) * 256 + threadIdx.x);
    if constexpr (M == 0) {
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int c = 0; c < C; ++c) acc ^= x[j][c];
        if (acc.x == 0x1234567u) par[0] = acc;
    }
#pragma unroll
    for (int t = 0; t < M; ++t)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
            for (int j = 0; j < K; ++j) acc ^= (x[j][c] << ((t + j) & 7));
            st(p + t * pitch + (size_t(chunk) * C + c) * 256 + threadIdx.x, acc);
        }
}

template <typename F> float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

const size_t S = 1 << 20;
int stripes = 4096;
u32x4 *data, *par;
uint2* desc;

template <int M, int C, bool DEP> void run(int lds_kb) {
    const int chunks = S / 16 / 256 / C;
    const size_t pitch = S / 16;
    auto fn = stripe_k<10, M, C, DEP>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    float ms = timeit([&] { hipLaunchKernelGGL(fn, dim3(stripes * chunks), dim3(256), lds_kb * 1024, 0, data, par, pitch, chunks, desc); }, 5);
    const char* occ = lds_kb == 0 ? "max" : (lds_kb >= 40 ? "4" : (lds_kb >= 32 ? "5" : "6"));
    printf("10r%dw cols/lane=%d dep=%d waves/SIMD<=%-3s %7.1f GB/s\n", M, C, DEP ? 1 : 0, occ,
           double(stripes) * (10 + M) * S / ms / 1e6);
}

template <int M> void shape() {
    run<M, 1, false>(0);
    run<M, 1, false>(40);
    run<M, 1, true>(40);
    run<M, 1, false>(32);
    run<M, 2, false>(40);
    run<M, 2, true>(40);
}

int main(int argc, char** argv) {
    if (argc > 1) stripes = atoi(argv[1]);
    CK(hipMalloc(&data, stripes * 10 * S));
    CK(hipMalloc(&par, stripes * 4 * S));
    CK(hipMalloc(&desc, stripes * sizeof(uint2)));
    CK(hipMemset(data, 1, stripes * 10 * S));
    CK(hipMemset(par, 0, stripes * 4 * S));
    uint2* h = static_cast<uint2*>(malloc(stripes * sizeof(uint2)));
    for (int i = 0; i < stripes; ++i) h[i] = make_uint2(static_cast<unsigned>(i), 0u);
    CK(hipMemcpy(desc, h, stripes * sizeof(uint2), hipMemcpyHostToDevice));
    shape<0>();
    shape<1>();
    shape<2>();
    shape<4>();
    return 0;
}
