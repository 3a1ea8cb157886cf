// membench6.hip -- does splitting the RS(10,4) stripe traffic into a read
// phase and a write phase beat the one-pass 10-read / 4-write mix?
//   one-pass : 10 nt loads + 4 nt stores per 16-B column (the encode's shape)
//   rd10     : 10 loads only;  wr4: 4 stores only
//   two-phase: per chunk of C stripes, kernel A reads the 10 data streams and
//              writes the 4 outputs to a temp buffer T (C x 4 MiB, reused for
//              every chunk, meant to stay in the 256 MiB Infinity Cache),
//              kernel B copies T to the parity region (pure HBM writes if T
//              hits on-die).
// All rates are (10 + 4) x S bytes per stripe over wall time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;

template <bool NT> __device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load((GlobalCU4*)p);
    return *(const GlobalCU4*)p;
}
template <bool NT> __device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (GlobalU4*)p);
    else *(GlobalU4*)p = v;
}

constexpr int K = 10, M = 4;
const size_t S = 1 << 20;
const size_t PITCH = S / 16;  // u32x4 per shard
const int CHUNKS = S / 16 / 256;

// out[s_out] <- f(data[s_in]); s_in = s0 + blockIdx / CHUNKS, s_out = s_in - obase
template <bool LD_NT, bool ST_NT, int KR, int MW>
__global__ __launch_bounds__(256) void pass(const u32x4* __restrict__ data, u32x4* __restrict__ out, size_t s0, size_t obase) {
    const size_t s = s0 + blockIdx.x / CHUNKS;
    const int chunk = blockIdx.x % CHUNKS;
    const size_t col = size_t(chunk) * 256 + threadIdx.x;
    const u32x4* d = data + s * KR * PITCH;
    u32x4 x[KR > 0 ? KR : 1];
#pragma unroll
    for (int j = 0; j < KR; ++j) x[j] = ld<LD_NT>(d + j * PITCH + col);
    if constexpr (MW == 0) {
        u32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < KR; ++j) acc ^= x[j];
        if (acc.x == 0x1234567u) out[0] = acc;
    }
    u32x4* p = out + (s - obase) * (MW ? MW : 1) * PITCH;
#pragma unroll
    for (int t = 0; t < MW; ++t) {
        u32x4 acc = {0u, 0u, 0u, (unsigned)t};
#pragma unroll
        for (int j = 0; j < KR; ++j) acc ^= (x[j] << ((t + j) & 7));
        if constexpr (KR == 0) acc.x ^= static_cast<unsigned>(col);
        st<ST_NT>(p + t * PITCH + col, acc);
    }
}

// T (chunk-local, M streams per stripe) -> P (global parity)
template <bool LD_NT, bool ST_NT>
__global__ __launch_bounds__(256) void copy_t(const u32x4* __restrict__ T, u32x4* __restrict__ P, size_t s0) {
    const size_t sl = blockIdx.x / CHUNKS;
    const int chunk = blockIdx.x % CHUNKS;
    const size_t col = size_t(chunk) * 256 + threadIdx.x;
    u32x4 v[M];
#pragma unroll
    for (int t = 0; t < M; ++t) v[t] = ld<LD_NT>(T + (sl * M + t) * PITCH + col);
#pragma unroll
    for (int t = 0; t < M; ++t) st<ST_NT>(P + ((s0 + sl) * M + t) * PITCH + col, v[t]);
}

template <typename F> float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a)); for (int r = 0; r < reps; ++r) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms / reps;
}

int stripes = 4096;
u32x4 *data, *par, *tmp;

void report(const char* name, float ms) {
    printf("%-44s %8.3f ms  %7.1f GB/s (k+m bytes)\n", name, ms, double(stripes) * (K + M) * S / ms / 1e6);
}

template <bool A_ST_NT, bool B_LD_NT> void two_phase(int C) {
    char name[96];
    float ms = timeit([&] {
        for (int s0 = 0; s0 < stripes; s0 += C) {
            const int nb = (s0 + C <= stripes) ? C : stripes - s0;
            hipLaunchKernelGGL((pass<true, A_ST_NT, K, M>), dim3(nb * CHUNKS), dim3(256), 0, 0, data, tmp, size_t(s0), size_t(s0));
            hipLaunchKernelGGL((copy_t<B_LD_NT, true>), dim3(nb * CHUNKS), dim3(256), 0, 0, tmp, par, size_t(s0));
        }
    }, 3);
    snprintf(name, sizeof name, "two-phase C=%d (T %d MiB) T-store %s T-load %s", C, C * 4, A_ST_NT ? "nt" : "plain", B_LD_NT ? "nt" : "plain");
    report(name, ms);
}

int main(int argc, char** argv) {
    if (argc > 1) stripes = atoi(argv[1]);
    CK(hipMalloc(&data, stripes * K * S));
    CK(hipMalloc(&par, stripes * M * S));
    CK(hipMalloc(&tmp, size_t(128) * M * S));
    CK(hipMemset(data, 1, stripes * K * S));
    CK(hipMemset(par, 0, stripes * M * S));
    const dim3 g(stripes * CHUNKS);
    for (int rep = 0; rep < 2; ++rep) {
        report("one-pass 10r4w (nt/nt)", timeit([&] { hipLaunchKernelGGL((pass<true, true, K, M>), g, dim3(256), 0, 0, data, par, size_t(0), size_t(0)); }, 3));
        float r = timeit([&] { hipLaunchKernelGGL((pass<true, true, K, 0>), g, dim3(256), 0, 0, data, par, size_t(0), size_t(0)); }, 3);
        float w = timeit([&] { hipLaunchKernelGGL((pass<true, true, 0, M>), g, dim3(256), 0, 0, data, par, size_t(0), size_t(0)); }, 3);
        printf("rd10 only %.3f ms (%.1f GB/s)  wr4 only %.3f ms (%.1f GB/s)  sum %.3f ms -> ", r, double(stripes) * K * S / r / 1e6, w, double(stripes) * M * S / w / 1e6, r + w);
        report("", r + w);
        for (int C : {4, 8, 16, 32, 64}) {
            two_phase<false, false>(C);
            two_phase<true, true>(C);
        }
        two_phase<false, true>(16);
        two_phase<true, false>(16);
    }
    return 0;
}
