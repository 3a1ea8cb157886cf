// membench4.hip -- cache-policy bits (sc0/sc1/nt) on the 10-read/4-write
// stripe shape of the RS(10,4) kernel, and on copy / read-only.  Pure data
// movement: answers whether non-temporal loads or stores raise the ceiling.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));


template <int P> __device__ __forceinline__ u32x4 ld(const u32x4* p) {
    u32x4 v;
    if constexpr (P == 0) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    if constexpr (P == 1) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    if constexpr (P == 2) asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    if constexpr (P == 3) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
    if constexpr (P == 4) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}
template <int P> __device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (P == 0) asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(p), "v"(v) : "memory");
    if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" :: "v"(p), "v"(v) : "memory");
    if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

static const char* pname[] = {"plain", "nt", "sc1", "sc0sc1", "sc0sc1nt"};

template <int K, int M, int LP, int SP>
__global__ __launch_bounds__(256) void stripe_k(const u32x4* __restrict__ data, u32x4* __restrict__ par,
                                                size_t pitch, int chunks) {
    const size_t s = blockIdx.x / chunks;
    const int chunk = blockIdx.x % chunks;
    const size_t c = size_t(chunk) * 256 + threadIdx.x;
    const u32x4* d = data + s * K * pitch;
    u32x4* p = par + s * (M ? M : 1) * pitch;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = ld<LP>(d + j * pitch + c);
    wait_vm();
    if constexpr (M == 0) {
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= x[j];
        if (acc.x == 0x1234567u) par[0] = acc;
    }
#pragma unroll
    for (int t = 0; t < M; ++t) {
        u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= (x[j] << ((t + j) & 7));
        st<SP>(p + t * pitch + c, acc);
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

template <int LP, int SP> void run_10r4w() {
    const int chunks = S / 16 / 256;
    const size_t pitch = S / 16;
    float ms = timeit([&] { stripe_k<10, 4, LP, SP><<<stripes * chunks, 256>>>(data, par, pitch, chunks); }, 5);
    printf("10r4w load=%-8s store=%-8s %7.1f GB/s\n", pname[LP], pname[SP], double(stripes) * 14 * S / ms / 1e6);
}
template <int LP, int SP> void run_copy() {
    const int chunks = S / 16 / 256;
    const size_t pitch = S / 16;
    float ms = timeit([&] { stripe_k<1, 1, LP, SP><<<stripes * 4 * chunks, 256>>>(data, par, pitch, chunks); }, 5);
    printf("copy  load=%-8s store=%-8s %7.1f GB/s\n", pname[LP], pname[SP], double(stripes) * 8 * S / ms / 1e6);
}
template <int LP> void run_read() {
    const int chunks = S / 16 / 256;
    const size_t pitch = S / 16;
    float ms = timeit([&] { stripe_k<10, 0, LP, 0><<<stripes * chunks, 256>>>(data, par, pitch, chunks); }, 5);
    printf("10r0w load=%-8s                %7.1f GB/s\n", pname[LP], double(stripes) * 10 * S / ms / 1e6);
}

int main(int argc, char** argv) {
    if (argc > 1) stripes = atoi(argv[1]);
    CK(hipMalloc(&data, stripes * 10 * S));
    CK(hipMalloc(&par, stripes * 4 * S));
    CK(hipMemset(data, 1, stripes * 10 * S));
    CK(hipMemset(par, 0, stripes * 4 * S));
    run_read<0>(); run_read<1>(); run_read<2>(); run_read<3>();
    run_copy<0, 0>(); run_copy<0, 1>(); run_copy<1, 1>(); run_copy<0, 2>(); run_copy<0, 3>(); run_copy<0, 4>();
    run_10r4w<0, 0>(); run_10r4w<0, 1>(); run_10r4w<0, 2>(); run_10r4w<0, 3>(); run_10r4w<0, 4>();
    run_10r4w<1, 0>(); run_10r4w<1, 1>(); run_10r4w<2, 1>(); run_10r4w<3, 1>(); run_10r4w<1, 4>();
    run_10r4w<0, 0>();
    return 0;
}
