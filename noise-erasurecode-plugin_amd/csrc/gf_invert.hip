// gf_invert.hip -- batched decode-matrix construction on the GPU: for every
// new erasure pattern, the decode rows E[target] . A^-1 of its erased shards,
// where A is the k x k survivor submatrix of the systematic matrix E.
//
// This is Rebuild's invertMatrix + row products (infectious, reference call
// site main.go:77) for many patterns at once -- one workgroup per pattern --
// so a batched reconstruct whose stripes carry thousands of distinct
// patterns (wide codes, BASELINE configs 3/5) does not wait for host
// inversions.  Results are bit-identical to the host path (gf256.cpp
// decode_rows): an inverse over a field is unique, so any exact method gives
// the same bytes.
//
// Two methods:
//  * structured (the normal case): Rebuild keeps every present data shard in
//    its own slot and fills the d erased data slots with parity survivors, so
//    A is the identity except for d rows.  With D the erased data indices and
//    B = E[parity survivors][D] (d x d), the data shares are
//        x_D = B^-1 (y_D + F y_present),  F = E[parity survivors][present],
//    which gives every decode row from one d x d inverse and O(e.d.k)
//    products instead of a k x k Gauss-Jordan (d <= m; RS(64,16): <= 16 vs 64
//    columns, each a few barriers).
//  * generic Gauss-Jordan on the whole k x k A, for survivor sets without
//    that shape (never produced by choose_survivors; kept so any survivor
//    list is handled) and for A/B runs (InvertArgs::generic).
#include "gf_invert.hpp"

#include <atomic>

namespace rsmi {
namespace {

// Threads per pattern.  One wave (barriers are cheap, more patterns
// resident): 16,384 fresh RS(64,16) patterns build in ~260 us vs ~370 us
// with 256 threads (profiles/r02z/) -- which matters since a build no
// longer overlaps the caller's queued kernels (rsmi.cpp flush_patterns_impl).
#ifndef RSMI_INVERT_THREADS
#define RSMI_INVERT_THREADS 64
#endif
constexpr int kThreads = RSMI_INVERT_THREADS;

// LDS bytes of the matrix work area: the generic k x k A, or the structured
// B (d x d), F and G (d x k each) for up to dm = min(k, m) erased data shards.
__host__ __device__ inline size_t invert_work_bytes(int k, int m) {
    const size_t dm = static_cast<size_t>(k < m ? k : m);
    const size_t generic = static_cast<size_t>(k) * k;
    const size_t structured = dm * dm + 2 * dm * static_cast<size_t>(k);
    return ((generic > structured ? generic : structured) + 15) & ~size_t(15);
}

constexpr uint8_t kNone = 0xFF;  // pos[j]: slot j holds its own data shard

struct GfTabs {
    const uint8_t* ex;  // 512: 2^i, doubled so log sums need no mod
    const uint8_t* lg;  // 256
    __device__ uint32_t mul(uint32_t x, uint32_t y) const { return (x && y) ? ex[lg[x] + lg[y]] : 0u; }
    __device__ uint32_t inv(uint32_t x) const { return ex[255 - lg[x]]; }
};

// In-place Gauss-Jordan with row pivoting on A (nn x nn, LDS, row-major),
// all threads of the block.  Returns false (uniformly) if A is singular.
__device__ bool gj_invert(uint8_t* A, int nn, uint8_t* fac, uint8_t* swp, int* piv, const GfTabs& gf) {
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, nwaves = kThreads / 64;
    for (int col = 0; col < nn; ++col) {
        if (tid == 0) {
            int r = col;
            while (r < nn && A[r * nn + col] == 0) ++r;
            *piv = r < nn ? r : -1;
            swp[col] = static_cast<uint8_t>(r < nn ? r : col);
        }
        __syncthreads();
        const int pr = *piv;
        if (pr < 0) return false;
        if (pr != col)
            for (int c = tid; c < nn; c += kThreads) {
                const uint8_t t = A[pr * nn + c];
                A[pr * nn + c] = A[col * nn + c];
                A[col * nn + c] = t;
            }
        __syncthreads();
        for (int r = tid; r < nn; r += kThreads) fac[r] = r == col ? 0 : A[r * nn + col];
        const uint32_t iv = gf.inv(A[col * nn + col]);
        __syncthreads();
        // pivot row /= pivot, with the pivot entry standing in for the
        // identity column (in-place inversion)
        for (int c = tid; c < nn; c += kThreads)
            A[col * nn + c] = static_cast<uint8_t>(c == col ? iv : gf.mul(iv, A[col * nn + c]));
        __syncthreads();
        for (int r = wave; r < nn; r += nwaves) {
            if (r == col) continue;
            const uint32_t f = fac[r];
            for (int c = lane; c < nn; c += 64) {
                const uint32_t v = c == col ? 0u : A[r * nn + c];
                A[r * nn + c] = static_cast<uint8_t>(v ^ gf.mul(f, A[col * nn + c]));
            }
        }
        __syncthreads();
    }
    // (P.A)^-1 = A^-1 . P^-1: undo the row swaps as column swaps, last first.
    for (int col = nn - 1; col >= 0; --col) {
        const int s = swp[col];
        if (s != col)
            for (int r = tid; r < nn; r += kThreads) {
                const uint8_t t = A[r * nn + s];
                A[r * nn + s] = A[r * nn + col];
                A[r * nn + col] = t;
            }
        __syncthreads();
    }
    return true;
}

__global__ __launch_bounds__(kThreads) void invert_patterns_kernel(InvertArgs a) {
    extern __shared__ uint8_t sm[];
    const int k = static_cast<int>(a.k);
    const int m = static_cast<int>(a.m);
    const int dm = k < m ? k : m;   // most erased data shards a pattern can have
    int* sh = reinterpret_cast<int*>(sm);  // [0] pivot row, [1] d, [2] structured
    uint8_t* A = sm + 16;           // k * k (generic) | B d*d, F d*k, G d*k (structured)
    uint8_t* ex = A + invert_work_bytes(k, m);
    uint8_t* lg = ex + 512;
    uint8_t* fac = lg + 256;        // k: column factors of the current step
    uint8_t* swp = fac + k;         // k: pivot row chosen at each column
    uint8_t* pos = swp + k;         // k: slot j's index in D, or kNone
    uint8_t* dl = pos + k;          // dm: erased data indices D (slot order)
    uint8_t* ds = dl + dm;          // dm: the parity survivor in each of those slots
    uint8_t* Et = ds + dm;          // m * k: encode rows of the targets
    uint32_t* svl = reinterpret_cast<uint32_t*>(sm + ((Et + m * k - sm + 3) & ~3));  // k: survivor ids
    uint32_t* tvl = svl + k;        // m: erased ids

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63, nwaves = kThreads / 64;
    const uint32_t p = a.first + blockIdx.x;
    const uint32_t* sv = a.src + static_cast<size_t>(p) * k;
    const uint32_t* tv = a.dst + static_cast<size_t>(p) * a.dst_stride;
    uint8_t* out = a.coef + static_cast<size_t>(p) * m * k;
    if (tid == 0) a.status[p] = 0u;  // set to 1 below if the survivor matrix is singular
    if (a.keys) {
        // The pattern's rows from its key.  Erased ids ascending (wave 0,
        // one ballot per 64 ids); survivors by Rebuild's rule (thread 0,
        // the loop of gf256.cpp choose_survivors_into): slot i keeps shard i
        // if present, else takes the highest present shard not yet used.
        const uint64_t* kw = a.keys + static_cast<size_t>(blockIdx.x) * 4;
        const int n = k + m;
        if (wave == 0) {
            int base = 0;
            for (int c0 = 0; c0 < n; c0 += 64) {
                const uint64_t valid = n - c0 >= 64 ? ~0ull : ((1ull << (n - c0)) - 1ull);
                const uint64_t er = kw[c0 >> 6] & valid;
                const int at = base + __builtin_popcountll(er & ((1ull << lane) - 1ull));
                if (((er >> lane) & 1ull) && at < m) tvl[at] = static_cast<uint32_t>(c0 + lane);
                base += __builtin_popcountll(er);
            }
            if (lane == 0) sh[3] = base;
        }
        if (tid == 0) {
            uint64_t used[4] = {0, 0, 0, 0};
            auto erased = [&](int j) { return (kw[j >> 6] >> (j & 63)) & 1ull; };
            auto taken = [&](int j) { return (used[j >> 6] >> (j & 63)) & 1ull; };
            int hi = n - 1;
            for (int i = 0; i < k; ++i) {
                int pick = i;
                if (erased(i) || taken(i)) {
                    while (hi >= 0 && (erased(hi) || taken(hi))) --hi;
                    pick = hi < 0 ? 0 : hi;  // hi < 0 needs > m erasures: the host rejects those
                }
                svl[i] = static_cast<uint32_t>(pick);
                used[pick >> 6] |= 1ull << (pick & 63);
            }
        }
        __syncthreads();
        const int e0 = sh[3];
        uint32_t* gsv = a.src + static_cast<size_t>(p) * k;
        uint32_t* gtv = a.dst + static_cast<size_t>(p) * a.dst_stride;
        for (int i = tid; i < k; i += kThreads) gsv[i] = svl[i];
        for (int t = tid; t < static_cast<int>(a.dst_stride); t += kThreads) gtv[t] = t < e0 && t < m ? tvl[t] : 0u;
        if (tid == 0) a.cnt[p] = static_cast<uint32_t>(e0);
        sv = svl;
        tv = tvl;
    }
    const int e = a.keys ? sh[3] : static_cast<int>(a.cnt[p]);

    for (int i = tid; i < 512; i += kThreads) ex[i] = a.gf_exp[i];
    for (int i = tid; i < 256; i += kThreads) lg[i] = a.gf_log[i];
    for (int t = wave; t < e; t += nwaves) {
        const uint8_t* row = a.enc + static_cast<size_t>(tv[t]) * k;
        for (int c = lane; c < k; c += 64) Et[t * k + c] = row[c];
    }
    // Slot classification by wave 0: present data (sv[i] == i), erased data
    // filled by a parity survivor (sv[i] >= k), anything else -> generic.
    if (wave == 0) {
        int d = 0;
        bool odd = a.generic != 0;
        for (int c0 = 0; c0 < k; c0 += 64) {
            const int i = c0 + lane;
            const uint32_t s = i < k ? sv[i] : static_cast<uint32_t>(i);
            const bool par = i < k && s >= static_cast<uint32_t>(k);
            const uint64_t pm = __builtin_amdgcn_ballot_w64(par);
            odd |= __builtin_amdgcn_ballot_w64(i < k && !par && s != static_cast<uint32_t>(i)) != 0;
            const int at = d + __builtin_popcountll(pm & ((1ull << lane) - 1ull));
            if (i < k) pos[i] = par ? static_cast<uint8_t>(at) : kNone;
            if (par && at < dm) {
                dl[at] = static_cast<uint8_t>(i);
                ds[at] = static_cast<uint8_t>(s);
            }
            d += __builtin_popcountll(pm);
        }
        odd |= d > dm;
        if (lane == 0) {
            sh[1] = d;
            sh[2] = odd ? 0 : 1;
        }
    }
    __syncthreads();
    const GfTabs gf{ex, lg};
    const int d = sh[1];

    if (sh[2]) {
        uint8_t* B = A;               // d x d, inverted in place
        uint8_t* F = B + dm * dm;     // d x k: E[ds[a]] (encode rows of the parity survivors)
        uint8_t* G = F + dm * k;      // d x k: decode rows of the erased data, in slot space
        for (int r = wave; r < d; r += nwaves) {
            const uint8_t* row = a.enc + static_cast<size_t>(ds[r]) * k;
            for (int c = lane; c < k; c += 64) F[r * k + c] = row[c];
        }
        __syncthreads();
        for (int i = tid; i < d * d; i += kThreads) {
            const int r = i / d, c = i - r * d;
            B[i] = F[r * k + dl[c]];
        }
        __syncthreads();
        if (!gj_invert(B, d, fac, swp, sh, gf)) {  // distinct survivors of an MDS code never are
            if (tid == 0) a.status[p] = 1u;
            return;
        }
        // G[b][j] = B^-1[b][pos j] for an erased slot j, else sum_a B^-1[b][a] F[a][j]
        for (int i = tid; i < d * k; i += kThreads) {
            const int b = i / k, j = i - b * k;
            uint32_t acc;
            if (pos[j] != kNone) {
                acc = B[b * d + pos[j]];
            } else {
                acc = 0;
                for (int q = 0; q < d; ++q) acc ^= gf.mul(B[b * d + q], F[q * k + j]);
            }
            G[i] = static_cast<uint8_t>(acc);
        }
        __syncthreads();
        // Erased data t: its G row.  Erased parity t: E[t] on the present
        // slots plus sum_b E[t][D_b] G[b].
        for (int i = tid; i < m * k; i += kThreads) {
            const int t = i / k, j = i - t * k;
            uint32_t acc = 0;
            if (t < e) {
                const uint32_t id = tv[t];
                if (id < static_cast<uint32_t>(k)) {
                    acc = G[pos[id] * k + j];
                } else {
                    acc = pos[j] == kNone ? Et[t * k + j] : 0u;
                    for (int b = 0; b < d; ++b) acc ^= gf.mul(Et[t * k + dl[b]], G[b * k + j]);
                }
            }
            out[i] = static_cast<uint8_t>(acc);
        }
        return;
    }

    // Generic: invert the whole survivor submatrix.
    for (int r = wave; r < k; r += nwaves) {
        const uint8_t* row = a.enc + static_cast<size_t>(sv[r]) * k;
        for (int c = lane; c < k; c += 64) A[r * k + c] = row[c];
    }
    __syncthreads();
    if (!gj_invert(A, k, fac, swp, sh, gf)) {  // distinct survivors of an MDS code never are
        if (tid == 0) a.status[p] = 1u;
        return;
    }
    for (int t = wave; t < m; t += nwaves)
        for (int c = lane; c < k; c += 64) {
            uint32_t acc = 0;
            if (t < e)
                for (int i = 0; i < k; ++i) acc ^= gf.mul(Et[t * k + i], A[i * k + c]);
            out[t * k + c] = static_cast<uint8_t>(acc);
        }
}

}  // namespace

size_t invert_lds_bytes(int k, int m) {
    const size_t dm = static_cast<size_t>(k < m ? k : m);
    const size_t bytes = 16 + invert_work_bytes(k, m) + 512 + 256 + 3 * static_cast<size_t>(k) + 2 * dm +
                         static_cast<size_t>(m) * k;
    return ((bytes + 3) & ~size_t(3)) + 4 * static_cast<size_t>(k + m);  // + survivor / erased ids
}

hipError_t launch_invert(const InvertArgs& a, uint32_t count, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    const size_t lds = invert_lds_bytes(static_cast<int>(a.k), static_cast<int>(a.m));
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static std::atomic<bool> attr_set{false};  // contexts on several threads may launch
    if (!attr_set.load() && lds > 65536) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(invert_patterns_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return hipErrorInvalidValue;
        attr_set.store(true);
    }
    hipLaunchKernelGGL(invert_patterns_kernel, dim3(count), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

}  // namespace rsmi
