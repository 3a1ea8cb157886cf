// gf_invert.hip -- batched decode-matrix construction on the GPU: for every
// new erasure pattern, invert the k x k survivor submatrix of the systematic
// matrix over GF(2^8) and emit the decode rows of its erased shards.
//
// This is Rebuild's invertMatrix + row products (infectious, reference call
// site main.go:77) for many patterns at once -- one workgroup per pattern --
// so a batched reconstruct whose stripes carry thousands of distinct
// patterns (wide codes, BASELINE configs 3/5) does not wait for host
// inversions.  Results are bit-identical to the host path (gf256.cpp
// decode_rows): an inverse over a field is unique.
#include "gf_invert.hpp"

namespace rsmi {
namespace {

constexpr int kThreads = 256;

// In-place Gauss-Jordan with row pivoting on A (k x k, LDS), then the
// decode rows row_t = enc[target_t] . A^-1.
__global__ __launch_bounds__(kThreads) void invert_patterns_kernel(InvertArgs a) {
    extern __shared__ uint8_t sm[];
    const int k = static_cast<int>(a.k);
    const int m = static_cast<int>(a.m);
    uint8_t* A = sm;                // k * k
    uint8_t* ex = A + k * k;        // 512: 2^i, doubled so log sums need no mod
    uint8_t* lg = ex + 512;         // 256
    uint8_t* fac = lg + 256;        // k: column factors of the current step
    uint8_t* swp = fac + k;         // k: pivot row chosen at each column
    uint8_t* Et = swp + k;          // m * k: encode rows of the targets
    int* piv = reinterpret_cast<int*>(Et + ((m * k + 3) & ~3));

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, nwaves = kThreads / 64;
    const uint32_t p = a.first + blockIdx.x;
    const uint32_t* sv = a.src + static_cast<size_t>(p) * k;
    const uint32_t* tv = a.dst + static_cast<size_t>(p) * a.dst_stride;
    const int e = static_cast<int>(a.cnt[p]);

    for (int i = tid; i < 512; i += kThreads) ex[i] = a.gf_exp[i];
    for (int i = tid; i < 256; i += kThreads) lg[i] = a.gf_log[i];
    for (int r = wave; r < k; r += nwaves) {
        const uint8_t* row = a.enc + static_cast<size_t>(sv[r]) * k;
        for (int c = lane; c < k; c += 64) A[r * k + c] = row[c];
    }
    for (int t = wave; t < e; t += nwaves) {
        const uint8_t* row = a.enc + static_cast<size_t>(tv[t]) * k;
        for (int c = lane; c < k; c += 64) Et[t * k + c] = row[c];
    }
    __syncthreads();
    auto mul = [&](uint32_t x, uint32_t y) -> uint32_t {
        return (x && y) ? ex[lg[x] + lg[y]] : 0u;
    };

    for (int col = 0; col < k; ++col) {
        if (tid == 0) {
            int r = col;
            while (r < k && A[r * k + col] == 0) ++r;
            *piv = r < k ? r : -1;
            swp[col] = static_cast<uint8_t>(r < k ? r : col);
        }
        __syncthreads();
        const int pr = *piv;
        if (pr < 0) {  // singular: distinct survivors of an MDS code never are
            if (tid == 0) atomicOr(a.status, 1u);
            return;
        }
        if (pr != col)
            for (int c = tid; c < k; c += kThreads) {
                const uint8_t t = A[pr * k + c];
                A[pr * k + c] = A[col * k + c];
                A[col * k + c] = t;
            }
        __syncthreads();
        for (int r = tid; r < k; r += kThreads) fac[r] = r == col ? 0 : A[r * k + col];
        const uint32_t inv = ex[255 - lg[A[col * k + col]]];
        __syncthreads();
        // pivot row /= pivot, with the pivot entry standing in for the
        // identity column (in-place inversion)
        for (int c = tid; c < k; c += kThreads)
            A[col * k + c] = static_cast<uint8_t>(c == col ? inv : mul(inv, A[col * k + c]));
        __syncthreads();
        for (int r = wave; r < k; r += nwaves) {
            if (r == col) continue;
            const uint32_t f = fac[r];
            for (int c = lane; c < k; c += 64) {
                const uint32_t v = c == col ? 0u : A[r * k + c];
                A[r * k + c] = static_cast<uint8_t>(v ^ mul(f, A[col * k + c]));
            }
        }
        __syncthreads();
    }
    // (P.A)^-1 = A^-1 . P^-1: undo the row swaps as column swaps, last first.
    for (int col = k - 1; col >= 0; --col) {
        const int s = swp[col];
        if (s != col)
            for (int r = tid; r < k; r += kThreads) {
                const uint8_t t = A[r * k + s];
                A[r * k + s] = A[r * k + col];
                A[r * k + col] = t;
            }
        __syncthreads();
    }
    uint8_t* out = a.coef + static_cast<size_t>(p) * m * k;
    for (int t = wave; t < m; t += nwaves)
        for (int c = lane; c < k; c += 64) {
            uint32_t acc = 0;
            if (t < e)
                for (int i = 0; i < k; ++i) acc ^= mul(Et[t * k + i], A[i * k + c]);
            out[t * k + c] = static_cast<uint8_t>(acc);
        }
}

}  // namespace

size_t invert_lds_bytes(int k, int m) {
    return static_cast<size_t>(k) * k + 512 + 256 + 2 * k + ((m * k + 3) & ~3) + 16;
}

hipError_t launch_invert(const InvertArgs& a, uint32_t count, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    const size_t lds = invert_lds_bytes(static_cast<int>(a.k), static_cast<int>(a.m));
    static bool attr_set = false;
    if (!attr_set && lds > 65536) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(invert_patterns_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return hipErrorInvalidValue;
        attr_set = true;
    }
    hipLaunchKernelGGL(invert_patterns_kernel, dim3(count), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

}  // namespace rsmi
