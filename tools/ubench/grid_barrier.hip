// grid_barrier.hip -- cost of a grid-wide barrier between phases of a
// persistent kernel (agent-scope atomic add + acquire poll by one lane per
// workgroup, then a workgroup barrier).  Spin-limited: a grid that is not
// fully resident degrades instead of hanging.  Prints us per barrier.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__device__ __forceinline__ void grid_sync(unsigned* ctr, unsigned target, unsigned* timeouts) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins > (1u << 16)) { atomicAdd(timeouts, 1u); break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void barriers(unsigned* ctr, unsigned* timeouts, int n) {
    for (int i = 0; i < n; ++i) grid_sync(ctr, (i + 1u) * gridDim.x, timeouts);
}

int main() {
    unsigned *ctr, *to;
    CK(hipMalloc(&ctr, 4));
    CK(hipMalloc(&to, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int bpc : {1, 2, 4}) {
        const int grid = 256 * bpc, n = 1000;
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(ctr, 0, 4));
            CK(hipMemset(to, 0, 4));
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(barriers, dim3(grid), dim3(256), 0, 0, ctr, to, n);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            unsigned t;
            CK(hipMemcpy(&t, to, 4, hipMemcpyDeviceToHost));
            printf("blocks/CU %d grid %d: %.3f us per barrier (%d barriers, %u spin timeouts)\n", bpc, grid, ms * 1e3 / n, n, t);
        }
    }
    return 0;
}
