// rs_kernels.hip -- CDNA4 (gfx950) kernels for GF(2^8) coding-matrix x
// shard-stripe products: the parity loop of infectious (*FEC).Encode
// (reference call site main.go:262) and the inverted-submatrix loop of
// (*FEC).Rebuild (reference call site main.go:77), batched over stripes.
//
// Arithmetic (no MFMA: GF(2^8) is not an FP contraction):
//   split-table GF(2^8) multiply (gf_device.hpp): three v_perm_b32 lookups
//   per coefficient on four packed bytes at once.
//   The five table dwords per coefficient are built per block from the raw
//   coefficient bytes and staged in LDS; a lane reads a coefficient's tables
//   with broadcast ds_read_b128 and XOR-accumulates in VGPRs (v_bitop3_b32).
// Memory: each lane owns one 16-byte column of every survivor shard
// (global_load_dwordx4, fully coalesced: 64 lanes = 1 KiB contiguous per
// shard); outputs are written once with global_store_dwordx4.
#include "rs_kernels.hpp"

#include "gf_device.hpp"
#include "xcd.hpp"

#include <algorithm>
#include <cstdlib>

namespace rsmi {
namespace {

constexpr int kBlock = 256;

using gfd::build_tables;
using gfd::gf_mac;
using gfd::xor3;

// Compiler fence for memory operations: keeps LDS table reads where they are
// written (LICM would otherwise hoist all k*MG*5 table dwords into VGPRs).
#define RS_MEM_FENCE() asm volatile("" ::: "memory")

constexpr int kRowsPerStep = 4;               // output rows per table sub-step
constexpr int kStepWords = kRowsPerStep * 5;  // table dwords per sub-step (5 x b128)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 GlobalCU4;
typedef __attribute__((address_space(1))) u32x4 GlobalU4;

// Global (not flat) 16-byte load/store: flat ops would count on lgkmcnt too
// and serialise against the LDS table reads.  NT sets the non-temporal cache
// policy bit: every shard byte is touched exactly once per launch, and on
// MI355X nt loads + nt stores raise the 10-read/4-write movement ceiling from
// 5.84 to 6.26 TB/s (profiles/r01_membench_cachepolicy.log).
template <bool NT>
__device__ __forceinline__ uint4 gload16(const uint8_t* p) {
    u32x4 v;
    if constexpr (NT) v = __builtin_nontemporal_load((GlobalCU4*)(p));
    else v = *(GlobalCU4*)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ void gstore16(uint8_t* p, uint4 v) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    if constexpr (NT) __builtin_nontemporal_store(w, (GlobalU4*)(p));
    else *(GlobalU4*)(p) = w;
}

// Wave-uniform 64-bit value into SGPRs.
__device__ __forceinline__ uint8_t* uniform_ptr(uint8_t* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
    return reinterpret_cast<uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}

__device__ __forceinline__ void load_step(const uint4* src, uint32_t (&T)[kStepWords]) {
#pragma unroll
    for (int w = 0; w < kStepWords / 4; ++w) {
        const uint4 v = src[w];
        T[4 * w + 0] = v.x;
        T[4 * w + 1] = v.y;
        T[4 * w + 2] = v.z;
        T[4 * w + 3] = v.w;
    }
}

// acc[r][w] ^= coef(row r) * x.w for the first R rows of one sub-step (R < 4
// only in the last sub-step of a row group that is not a multiple of 4).
template <int R = kRowsPerStep>
__device__ __forceinline__ void mac_step(uint32_t (&acc)[kRowsPerStep][4], const uint4& x,
                                         const uint32_t (&T)[kStepWords]) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t ia = xw[w] & 0x07070707u;
        const uint32_t ib = (xw[w] >> 3) & 0x07070707u;
        const uint32_t ic = (xw[w] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][w] = gf_mac(acc[r][w], &T[r * 5], ia, ib, ic);
    }
}

// mac_step for the first `rows` (1..4, wave-uniform) rows: one branch per
// row past the first, around all four words.
__device__ __forceinline__ void mac_step_rows(uint32_t (&acc)[kRowsPerStep][4], const uint4& x,
                                              const uint32_t (&T)[kStepWords], int rows) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    uint32_t ia[4], ib[4], ic[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        ia[w] = xw[w] & 0x07070707u;
        ib[w] = (xw[w] >> 3) & 0x07070707u;
        ic[w] = (xw[w] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int r = 0; r < kRowsPerStep; ++r) {
        if (r > 0 && r >= rows) break;
#pragma unroll
        for (int w = 0; w < 4; ++w) acc[r][w] = gf_mac(acc[r][w], &T[r * 5], ia[w], ib[w], ic[w]);
    }
}

// Step boundary: the accumulators of the finished sub-step are inputs of the
// asm, so its arithmetic completes before the boundary, and the memory
// clobber keeps the next sub-step's LDS reads after it.  At most two
// sub-steps of tables (2 x 20 dwords) are live at any time.
__device__ __forceinline__ void step_fence(uint32_t (&acc)[kRowsPerStep][4]) {
#pragma unroll
    for (int r = 0; r < kRowsPerStep; ++r)
        asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3])::"memory");
}

// One block codes a chunk of 16-byte columns of one stripe for one group of
// MG output rows: logical block `blk` of `nblk` (rs_matmul_kernel: blockIdx.x
// of the grid; rs_resident_kernel: each job's blocks in turn).  LDS: [k][MG/4][20]
// table dwords | k survivor pointers.
template <int K, int MG, int BT, bool NT>
__device__ __forceinline__ void matmul_block(const MatArgs& a, uint32_t blk, uint32_t nblk, uint4* lds4) {
    static_assert(MG % 2 == 0, "MG must be even");
    constexpr int TG = (MG + kRowsPerStep - 1) / kRowsPerStep;  // sub-steps per survivor
    constexpr int RL = MG - (TG - 1) * kRowsPerStep;            // rows in the last sub-step
    constexpr bool kRegPtrs = K > 0 && K <= 16;           // survivor bases kept in SGPRs
    // A single 4-row group (the RS(10,4), RS(4,2), RS(8,14) reconstructs)
    // codes only the stripe's e rows: one MG = 4 launch serves stripes of
    // 1..4 erasures, and coding all 4 rows for each cost 1.6x the VALU of the
    // 1..4 mix (e = 2.5 on average).
#ifdef RSMI_NO_DYNROWS  // A/B builds only
    constexpr bool kDynRows = false;
#else
    constexpr bool kDynRows = TG == 1 && RL == kRowsPerStep && kRegPtrs;
#endif
    constexpr int JB = (K == 0) ? 8 : (K <= 16 ? K : 8);  // survivor loads in flight
    const int k = K ? K : static_cast<int>(a.k);
    uint32_t* tw = reinterpret_cast<uint32_t*>(lds4);
    uint8_t** sptr = reinterpret_cast<uint8_t**>(tw + k * MG * 5);

    // XCD-aware order (xcd.hpp): regions of a.xcd blocks per XCD in turn.
    uint64_t b = a.xcd ? xcd_block(blk, a.xcd, nblk) : blk;
    const uint32_t grp = static_cast<uint32_t>(b % a.groups);
    b /= a.groups;
    const uint32_t chunk = static_cast<uint32_t>(b % a.chunks);
    const uint64_t sv = b / a.chunks;
    // Stripe descriptor = {stripe, pattern id << 8 | outputs} (one dependent
    // load); without a table it is stripe sv with a.desc0 (encode: pattern 0,
    // all m parity rows) -- a single-message decode then starts its pattern
    // and survivor reads without a dependent read of host memory first.
    uint2 desc = make_uint2(static_cast<uint32_t>(sv), a.desc0 ? a.desc0 : a.m);
    if (a.stripe_desc) desc = a.stripe_desc[sv];
    else if (a.n_inline) desc = a.inl_desc[sv];
    const uint64_t s = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(desc.x));
    const uint32_t sw = __builtin_amdgcn_readfirstlane(desc.y);
    const uint32_t pat = sw >> 8;
    const int e = static_cast<int>(sw & 0xFFu);
    const int row0 = static_cast<int>(grp) * MG;
    if (row0 >= e) return;  // whole block: uniform
    const int eg = min(MG, e - row0);

    // This lane's coefficient byte for the table build is requested first, so
    // waiting for it later does not wait for the survivor loads behind it.
    const uint8_t* coef = a.coef + (static_cast<size_t>(pat) * a.m + row0) * k;
    uint32_t cbyte[(K > 0 && K * MG <= BT) ? 1 : 1];
    const bool one_coef = (K > 0 && K * MG <= BT);
    if (one_coef) {
        const int j = threadIdx.x / MG, t = threadIdx.x - j * MG;
        cbyte[0] = (static_cast<int>(threadIdx.x) < k * MG && t < eg) ? coef[t * k + j] : 0u;
    }

    auto shard = [&](uint32_t id) -> uint8_t* {
        if (a.shard_ptrs) return reinterpret_cast<uint8_t*>(a.shard_ptrs[s * (a.k + a.m) + id]);
        return id < a.k ? a.data + s * a.data_ss + static_cast<uint64_t>(id) * a.pitch
                        : a.parity + s * a.parity_ss + static_cast<uint64_t>(id - a.k) * a.pitch;
    };
    // a.src == nullptr: survivor j is shard id j (no id read before the
    // survivor loads).
    const uint32_t* srcid = a.src ? a.src + static_cast<size_t>(pat) * k : nullptr;
    const uint32_t* dstid = a.dst + static_cast<size_t>(pat) * a.dst_stride + row0;
    uint8_t* sp[kRegPtrs ? K : 1];
    if constexpr (kRegPtrs) {
        // All K survivor ids in one batch of scalar loads, then all K
        // addresses (pointer mode: one more batch): the mode branches sit
        // outside the loops.  Round 4 resolved the survivors one at a time
        // (id load, wait, mode branch, address load, wait): K dependent
        // scalar round trips before the first survivor load.
        uint32_t ids[K];
#pragma unroll
        for (int j = 0; j < K; ++j) ids[j] = static_cast<uint32_t>(j);
        if (srcid) {
#pragma unroll
            for (int j = 0; j < K; ++j) ids[j] = __builtin_amdgcn_readfirstlane(srcid[j]);
        }
        if (a.shard_ptrs) {
            const uint64_t* tp = a.shard_ptrs + s * (a.k + a.m);
#pragma unroll
            for (int j = 0; j < K; ++j) sp[j] = uniform_ptr(reinterpret_cast<uint8_t*>(tp[ids[j]]));
        } else {
            uint8_t* dbase = a.data + s * a.data_ss;
            uint8_t* pbase = a.parity + s * a.parity_ss;
#pragma unroll
            for (int j = 0; j < K; ++j)
                sp[j] = ids[j] < static_cast<uint32_t>(K) ? dbase + static_cast<uint64_t>(ids[j]) * a.pitch
                                                         : pbase + static_cast<uint64_t>(ids[j] - K) * a.pitch;
        }
    } else {
        for (int i = threadIdx.x; i < k; i += BT) sptr[i] = shard(srcid ? srcid[i] : static_cast<uint32_t>(i));
    }
    const uint32_t last = a.ncols16 - 1;
    // Survivor loads of the block's first iteration are issued before the
    // table build, so the prologue (pattern lookup, tables, barrier) overlaps
    // their HBM latency; with one iteration per block (the default) this is
    // the whole data path.
    uint4 xpre[kRegPtrs ? K : 1];
    // Iteration it of block `chunk` codes column chunk (it * chunks + chunk):
    // blocks running together stay on adjacent 4 KiB pieces of the same
    // shards (DRAM row locality) whatever the iteration count.
    const uint32_t cstride = a.chunks * BT;
    const uint32_t col0 = chunk * BT + threadIdx.x;
    const uint32_t off0 = (col0 <= last ? col0 : last) * 16u;
    if constexpr (kRegPtrs) {
#pragma unroll
        for (int j = 0; j < K; ++j) xpre[j] = gload16<NT>(sp[j] + off0);
    }
    // Output pointers are only needed at store time.  Rows are padded to 16
    // ids, so whole 4-id groups load unconditionally (s_load_dwordx4); rows
    // past eg point at a valid shard and are never stored.
    uint8_t* dp[TG * 4];
    {
        uint32_t oid[TG * 4];
#pragma unroll
        for (int g = 0; g < TG; ++g) {
            const uint4 ids = *reinterpret_cast<const uint4*>(dstid + 4 * g);
            oid[4 * g + 0] = __builtin_amdgcn_readfirstlane(ids.x);
            oid[4 * g + 1] = __builtin_amdgcn_readfirstlane(ids.y);
            oid[4 * g + 2] = __builtin_amdgcn_readfirstlane(ids.z);
            oid[4 * g + 3] = __builtin_amdgcn_readfirstlane(ids.w);
        }
        if (a.shard_ptrs) {
            const uint64_t* tp = a.shard_ptrs + s * (a.k + a.m);
#pragma unroll
            for (int r = 0; r < TG * 4; ++r) dp[r] = uniform_ptr(reinterpret_cast<uint8_t*>(tp[oid[r]]));
        } else {
            uint8_t* dbase = a.data + s * a.data_ss;
            uint8_t* pbase = a.parity + s * a.parity_ss;
#pragma unroll
            for (int r = 0; r < TG * 4; ++r)
                dp[r] = oid[r] < a.k ? dbase + static_cast<uint64_t>(oid[r]) * a.pitch
                                     : pbase + static_cast<uint64_t>(oid[r] - a.k) * a.pitch;
        }
    }
    // Split tables of rows [row0, row0 + MG): sub-step (j, g) holds rows
    // 4g..4g+3 as 4 x 5 dwords.
    if (one_coef) {
        if (static_cast<int>(threadIdx.x) < k * MG) {
            const int j = threadIdx.x / MG, t = threadIdx.x - j * MG;
            build_tables(cbyte[0], &tw[(j * TG + t / kRowsPerStep) * kStepWords + (t % kRowsPerStep) * 5]);
        }
    } else {
        for (int idx = threadIdx.x; idx < k * MG; idx += BT) {
            const int j = idx / MG, t = idx - j * MG;
            const uint32_t c = (t < eg) ? coef[t * k + j] : 0u;
            build_tables(c, &tw[(j * TG + t / kRowsPerStep) * kStepWords + (t % kRowsPerStep) * 5]);
        }
    }
    __syncthreads();

    for (uint32_t it = 0; it < a.iters; ++it) {
        const uint32_t colbase = chunk * BT + it * cstride;
        if (colbase >= a.ncols16) break;
        RS_MEM_FENCE();
        const uint32_t col = colbase + threadIdx.x;
        const bool ok = col <= last;
        // Tail lanes re-read the last column (always in bounds) and skip the store.
        const uint32_t off = (ok ? col : last) * 16u;
        uint32_t acc[TG][kRowsPerStep][4];
#pragma unroll
        for (int g = 0; g < TG; ++g)
#pragma unroll
            for (int r = 0; r < kRowsPerStep; ++r)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[g][r][w] = 0u;
        // Row groups of 4 beyond the pattern's outputs are skipped (uniform).
        const int tg_used = (eg + kRowsPerStep - 1) / kRowsPerStep;

        for (int jb = 0; jb < k; jb += JB) {
            uint4 xb[kRegPtrs ? 1 : JB];
            uint4* x = kRegPtrs ? xpre : xb;
            if constexpr (!kRegPtrs) {
#pragma unroll
                for (int q = 0; q < JB; ++q) {
                    if (K == 0 && jb + q >= k) break;
                    x[q] = gload16<NT>(uniform_ptr(sptr[jb + q]) + off);
                }
            }
            uint32_t TA[kStepWords], TB[kStepWords];
            load_step(lds4 + static_cast<size_t>(jb * TG) * (kStepWords / 4), TA);
#pragma unroll
            for (int q = 0; q < JB; ++q) {
                if (K == 0 && jb + q >= k) break;
#pragma unroll
                for (int g = 0; g < TG; ++g) {
                    // Sub-step (jb+q, g): prefetch the next one's tables, then
                    // multiply with the current ones (TA/TB alternate; the
                    // unrolled loop turns the copy into register renaming).
                    const int step = (jb + q) * TG + g;
                    const bool more = (g + 1 < TG) || (q + 1 < JB && (K != 0 || jb + q + 1 < k));
                    if (more) load_step(lds4 + static_cast<size_t>(step + 1) * (kStepWords / 4), TB);
                    if constexpr (kDynRows) {
                        mac_step_rows(acc[g], x[q], TA, eg);
                    } else if (TG == 1 || g < tg_used) {
                        if (g == TG - 1) mac_step<RL>(acc[g], x[q], TA);
                        else mac_step(acc[g], x[q], TA);
                    }
                    step_fence(acc[g]);
#pragma unroll
                    for (int w = 0; w < kStepWords; ++w) TA[w] = TB[w];
                }
            }
        }
        if constexpr (kRegPtrs) {
            // Software pipelining: the next iteration's survivor loads go out
            // before this iteration's stores.
            const uint32_t ncol = colbase + cstride + threadIdx.x;
            if (it + 1 < a.iters && colbase + cstride < a.ncols16) {
                const uint32_t noff = (ncol <= last ? ncol : last) * 16u;
#pragma unroll
                for (int j = 0; j < K; ++j) xpre[j] = gload16<NT>(sp[j] + noff);
            }
        }
#pragma unroll
        for (int g = 0; g < TG; ++g)
#pragma unroll
            for (int r = 0; r < kRowsPerStep; ++r) {
                const int t = g * kRowsPerStep + r;
                if (t >= eg) break;
                if (ok) gstore16<NT>(dp[t] + off, make_uint4(acc[g][r][0], acc[g][r][1], acc[g][r][2], acc[g][r][3]));
            }
    }
}

template <int K, int MG, int BT, bool NT>
__global__ __launch_bounds__(BT) void rs_matmul_kernel(MatArgs a) {
    extern __shared__ uint4 lds4[];
    matmul_block<K, MG, BT, NT>(a, blockIdx.x, gridDim.x, lds4);
}

// ------------------------------------------------------------- mailbox --
// One grid per single-message call (rs_kernels.hpp MailboxHost), a group of
// `per_job` blocks per job: the group's blocks poll `posted` over PCIe and
// code their job as soon as it is posted -- while the groups of earlier jobs
// are still reading theirs, so the PCIe reads of consecutive chunks overlap
// instead of each chunk paying the read latency ramp again (a kernel reading
// 256 KiB / 512 KiB / 1 MiB of pinned host memory takes 11 / 17 / 30 us,
// profiles/r06n/pcie_rates.txt).  The last block of a group to finish
// writes done[j - 1].  The call's chunks then cost the host one word each
// instead of a launch and an event, and the grid's dispatch overlaps the
// staging of the first chunk (profiles/r06h/: 4.3 us to launch a chunk,
// 5 us to dispatch it, 5.4 us between two chunks' kernels).  The jobs'
// arguments ride in the kernel arguments: read from the job board in pinned
// memory they cost each group 1.6-3.5 us of PCIe round trips before its
// first survivor load (profiles/r06u/).  Every wave leaves: after its job,
// on quit, or when its job is not posted in time.
__device__ __forceinline__ uint64_t mb_clock() { return __builtin_amdgcn_s_memrealtime(); }

template <int K, int MG, int BT>
__global__ __launch_bounds__(BT) void rs_mailbox_kernel(MailboxHost* h, MailboxDev* d, uint32_t per_job,
                                                        uint64_t timeout, uint32_t stamps, MailboxJobs jobs) {
    extern __shared__ uint4 lds4[];
    __shared__ uint32_t go_s;
    const uint32_t j = blockIdx.x / per_job;  // this block's job, 0-based
    const bool stamper = stamps && threadIdx.x == 0 && blockIdx.x == j * per_job;
    if (stamps && threadIdx.x == 0 && blockIdx.x == 0) d->stamp[0] = mb_clock();
    if (threadIdx.x == 0) {
        uint32_t go = 0;
        const uint64_t since = mb_clock();
        for (;;) {
            if (__hip_atomic_load(&h->posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) > j) {
                go = 1;
                break;
            }
            if (__hip_atomic_load(&h->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || mb_clock() - since > timeout)
                break;
            __builtin_amdgcn_s_sleep(4);
        }
        go_s = go;
        if (!go)  // the waiting caller launches the job itself at once, not after its own deadline
            __hip_atomic_store(&h->gave_up, uint64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (stamper) d->stamp[1 + 3 * j] = mb_clock();
    }
    __syncthreads();
    if (go_s) {
        // Job j's inputs (and a decode's pattern table) are in host memory
        // the host wrote before posting it: nothing cached from earlier may
        // be used.
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (stamper) d->stamp[2 + 3 * j] = mb_clock();
        const MailboxJob& job = jobs.job[j];
        const uint32_t nblk = job.blocks;
        for (uint32_t lb = blockIdx.x - j * per_job; lb < nblk; lb += per_job) {
            matmul_block<K, MG, BT, true>(job.a, lb, nblk, lds4);
            __syncthreads();  // the next logical block rebuilds the LDS tables
        }
        // This wave's outputs reach host memory before the block reports.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add(&d->arrive[j], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 == per_job) {
            if (stamps) d->stamp[3 + 3 * j] = mb_clock();
            __hip_atomic_store(&h->done[j], static_cast<uint64_t>(j + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // The last block out zeroes the device counters for the next launch on
    // this stream (kernel boundaries order the two).
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&d->left, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 == gridDim.x) {
        for (int i = 0; i < kMailboxJobs; ++i)
            __hip_atomic_store(&d->arrive[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&d->left, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

struct MailboxVariant {
    int K, MG;
    void (*fn)(MailboxHost*, MailboxDev*, uint32_t, uint64_t, uint32_t, MailboxJobs);  // (h, d, per_job, timeout, stamps, jobs)
};
const MailboxVariant kMailbox[] = {
    {10, 4, rs_mailbox_kernel<10, 4, 256>},  // RS(10,4): BASELINE config 1
    {4, 4, rs_mailbox_kernel<4, 4, 256>},    // RS(4,2): the plugin default (main.go:34-35)
};
const MailboxVariant* mailbox_variant(int k, int rows) {
    for (const MailboxVariant& v : kMailbox)
        if (v.K == k && rows >= 1 && rows <= v.MG) return &v;
    return nullptr;
}

__global__ __launch_bounds__(kBlock) void fill_splitmix_kernel(uint8_t* p, size_t len,
                                                               uint64_t seed) {
    const size_t nq = len / 8;
    const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t q = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; q <= nq; q += stride) {
        uint64_t z = seed + (q + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (q < nq) {
            reinterpret_cast<uint64_t*>(p)[q] = z;
        } else {
            for (size_t i = nq * 8; i < len; ++i) p[i] = static_cast<uint8_t>(z >> (8 * (i - nq * 8)));
        }
    }
}

struct Variant {
    int K, MG, BT;
    bool nt;
    const char* name;
    void (*fn)(MatArgs);
};

#define RS_VARIANT(K, MG, BT) {K, MG, BT, true, "K" #K "_MG" #MG "_B" #BT, rs_matmul_kernel<K, MG, BT, true>}
#define RS_VARIANT_T(K, MG, BT) {K, MG, BT, false, "K" #K "_MG" #MG "_B" #BT "_T", rs_matmul_kernel<K, MG, BT, false>}
// Specialised variants for the configurations the plugin and BASELINE use,
// then runtime-k fall-backs (k up to 256).
const Variant kVariants[] = {
    RS_VARIANT(10, 4, 256),   // RS(10,4): BASELINE configs 1-4
    RS_VARIANT(4, 4, 256),    // RS(4,2): plugin default (main.go:34-35)
    RS_VARIANT(8, 4, 256),    // infectious example RS(8,14): reconstructs of <= 4 erasures
    RS_VARIANT(8, 6, 256),    // ... its encode (6 rows: no padded rows' products)
    RS_VARIANT(8, 8, 256),
    RS_VARIANT(64, 4, 256),   // RS(64,16) reconstructs of <= 4 erasures (fewer VGPRs, smaller tables)
    RS_VARIANT(64, 8, 256),   // ... and <= 8
    RS_VARIANT(64, 16, 256),  // RS(64,16): BASELINE config 5
    RS_VARIANT(0, 4, 256),
    RS_VARIANT(0, 8, 256),
    // Temporal-policy twin of the headline variant, for A/B (RSMI_NT=0).
    RS_VARIANT_T(10, 4, 256),
    // 512/1024-thread blocks measured 3-13% slower for RS(10,4) on one box
    // (profiles/r01_ab_block.log); RSMI_BLOCK selects among compiled sizes.
};
#undef RS_VARIANT
#undef RS_VARIANT_T

// The variant for a launch coding up to `rows` output rows per stripe: the
// first specialised one for k whose row group holds them all (smaller row
// groups are listed first), else row groups of the runtime-k kernels.
const Variant& pick(int k, int rows) {
    static const int want_bt = [] {
        const char* e = std::getenv("RSMI_BLOCK");  // tuning knob
        return e ? std::atoi(e) : 256;
    }();
    static const bool want_nt = [] {
        const char* e = std::getenv("RSMI_NT");  // tuning knob (default 1: non-temporal)
        return e ? std::atoi(e) != 0 : true;
    }();
    for (const Variant& v : kVariants)
        if (v.K != 0 && v.K == k && rows <= v.MG && v.BT == want_bt && v.nt == want_nt) return v;
    for (const Variant& v : kVariants)
        if (v.K != 0 && v.K == k && rows <= v.MG && v.BT == want_bt) return v;
    for (const Variant& v : kVariants)
        if (v.K != 0 && v.K == k && rows <= v.MG) return v;
    for (const Variant& v : kVariants)
        if (v.K == 64 && k == 64 && v.MG == 16) return v;  // RS(64, m > 16): row groups of 16
    const int want_mg = rows <= 4 ? 4 : 8;  // runtime-k fall-backs
    for (const Variant& v : kVariants)
        if (v.K == 0 && v.MG == want_mg) return v;
    return kVariants[0];  // unreachable: both runtime-k variants are listed
}

}  // namespace

const char* variant_name(int k, int rows) { return pick(k, rows).name; }

bool mailbox_supported(int k, int rows) { return mailbox_variant(k, rows) != nullptr; }

void plan_mailbox_job(const MatArgs& a, int max_e, MailboxJob* job) {
    const MailboxVariant* v = mailbox_variant(static_cast<int>(a.k), max_e);
    const int mg = v ? v->MG : 4;
    job->a = a;
    job->a.iters = 1;
    job->a.chunks = (a.ncols16 + kBlock - 1) / kBlock;
    job->a.groups = static_cast<uint32_t>((max_e + mg - 1) / mg);
    job->a.xcd = 0;  // the logical blocks are dealt over the grid's blocks anyway
    job->blocks = static_cast<uint32_t>(a.stripes * job->a.chunks * job->a.groups);
}

hipError_t launch_mailbox(MailboxHost* h, MailboxDev* d, const MailboxJobs& jobs, int njobs, int k, int rows,
                          uint32_t per_job, uint64_t timeout, hipStream_t stream, bool stamps) {
    const MailboxVariant* v = mailbox_variant(k, rows);
    if (!v || per_job == 0 || njobs < 1 || njobs > kMailboxJobs) return hipErrorInvalidValue;
    const size_t lds = static_cast<size_t>(k) * ((v->MG + 3) / 4) * kStepWords * 4 + k * sizeof(void*);
    hipLaunchKernelGGL(v->fn, dim3(per_job * static_cast<uint32_t>(njobs)), dim3(kBlock), lds, stream, h, d, per_job,
                       timeout, static_cast<uint32_t>(stamps), jobs);
    return hipGetLastError();
}

hipError_t launch_matmul(MatArgs a, int max_e, hipStream_t stream) {
    if (a.stripes == 0 || a.ncols16 == 0 || max_e <= 0) return hipSuccess;
    const Variant& v = pick(static_cast<int>(a.k), max_e);
    const uint32_t total_it = (a.ncols16 + v.BT - 1) / v.BT;
    static const uint32_t iters_cap = [] {
        const char* e = std::getenv("RSMI_ITERS");  // tuning knob (default 1: one 4 KiB column chunk per block)
        const int v = e ? std::atoi(e) : 1;
        return static_cast<uint32_t>(v > 0 ? v : 1);
    }();
    a.iters = std::min<uint32_t>(iters_cap, total_it);
    a.chunks = (total_it + a.iters - 1) / a.iters;
    a.groups = static_cast<uint32_t>((max_e + v.MG - 1) / v.MG);
    size_t lds = static_cast<size_t>(a.k) * ((v.MG + 3) / 4) * kStepWords * 4 + a.k * sizeof(void*);
    static const size_t lds_floor = [] {
        const char* e = std::getenv("RSMI_LDS_PAD_KB");  // A/B knob: LDS per block >= this (caps occupancy)
        const int kb = e ? std::atoi(e) : 0;
        return static_cast<size_t>(kb > 0 && kb <= 64 ? kb : 0) * 1024;
    }();
    lds = std::max(lds, lds_floor);
    const uint64_t blocks = a.stripes * a.chunks * a.groups;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidConfiguration;
    if (a.xcd == ~0u) a.xcd = a.chunks * a.groups;  // a stripe per XCD region
    hipLaunchKernelGGL(v.fn, dim3(static_cast<uint32_t>(blocks)), dim3(v.BT), lds, stream, a);
    return hipGetLastError();
}

namespace {
// One block per (piece, 4 KiB chunk): 256 lanes x 16 bytes.
__global__ __launch_bounds__(256) void copy_pieces_kernel(const uint8_t* src, uint8_t* dst, const uint64_t* pieces,
                                                          uint32_t chunks, uint32_t cols16) {
    const uint32_t piece = blockIdx.x / chunks;
    const uint32_t col = (blockIdx.x - piece * chunks) * 256u + threadIdx.x;
    if (col >= cols16) return;
    // readfirstlane returns int: the low words go through uint32_t, or an
    // offset with bit 31 set would sign-extend over the high word.
    const uint64_t s0 = pieces[2 * piece];
    const uint64_t so = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(s0))) |
                        (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(s0 >> 32)))) << 32);
    const uint64_t d0 = pieces[2 * piece + 1];
    const uint64_t dof = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(d0))) |
                         (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(d0 >> 32)))) << 32);
    const uint4 v = gload16<true>(src + so + static_cast<uint64_t>(col) * 16u);
    gstore16<true>(dst + dof + static_cast<uint64_t>(col) * 16u, v);
}
}  // namespace

hipError_t launch_copy_pieces(const uint8_t* src, uint8_t* dst, const uint64_t* pieces, uint32_t count,
                              size_t bytes, hipStream_t stream) {
    if (count == 0 || bytes == 0) return hipSuccess;
    if (bytes % 16 != 0) return hipErrorInvalidValue;
    const uint64_t cols16 = bytes / 16, chunks = (cols16 + 255) / 256;
    if (cols16 > 0xFFFFFFFFull || static_cast<uint64_t>(count) * chunks > 0x7FFFFFFFull)
        return hipErrorInvalidConfiguration;
    hipLaunchKernelGGL(copy_pieces_kernel, dim3(static_cast<uint32_t>(count * chunks)), dim3(256), 0, stream, src, dst,
                       pieces, static_cast<uint32_t>(chunks), static_cast<uint32_t>(cols16));
    return hipGetLastError();
}

hipError_t launch_fill_splitmix(void* dev, size_t len, uint64_t seed, hipStream_t stream) {
    if (len == 0) return hipSuccess;
    const size_t nq = len / 8 + 1;
    const size_t blocks = std::min<size_t>((nq + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                       stream, static_cast<uint8_t*>(dev), len, seed);
    return hipGetLastError();
}

}  // namespace rsmi
