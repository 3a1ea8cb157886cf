// bitslice.hpp -- launch interface of the generated bit-sliced encode kernels
// (source written at build time by gen_bitslice.cpp from the systematic
// encode matrix of each listed (k, n)).
//
// Why: for wide codes such as RS(64,16) the split-table kernel
// (rs_kernels.hip) is VALU-bound (about 17 VALU ops per byte of traffic).
// Multiplication by a fixed coefficient is a GF(2)-linear map of a byte's
// 8 bits, so with every lane's 32 bytes of a shard transposed into 8 bit
// planes, the whole encode is an XOR network over planes whose wiring is
// known at compile time.  Per data shard and lane: a 48-op transpose, 22
// XORs building the 4-plane combinations (method of four Russians), then one
// v_bitop3 (3-way XOR) per output plane -- about 5 VALU ops per byte of
// traffic instead of 17.
//
// Reconstruct (k <= 64) reuses the fixed network through syndromes: with the
// erased data shards read as zero, the network yields q_t = sum over present
// data of E[t][j] * d_j for every parity row t.  For each parity survivor t,
// s_t = p_t ^ q_t depends on the erased data alone, and every output is
//     out_o = sum_t row_o[slot(t)] * s_t  (^ q_o if output o is parity o),
// where row_o is the pattern's decode row (gf_invert.hip) and slot(t) the
// survivor slot Rebuild gave parity t.  The per-pattern part is an e x d
// split-table product on d <= m syndromes instead of e x k on the survivors.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rsmi {

struct BitsliceArgs {
    const uint8_t* data;   // shard j of stripe s at data + s*data_ss + j*pitch
    uint8_t* parity;       // parity row t at parity + s*parity_ss + t*pitch
    uint64_t data_ss, parity_ss, pitch;
    uint64_t stripes;
    uint32_t ncols16;      // 16-byte columns per shard (ceil(S / 16))
    uint32_t blocks_per_stripe;
    uint32_t xcd;          // XCD-aware block order (xcd.hpp): stripes per region, 0 = natural
};

using BitsliceLaunch = hipError_t (*)(const BitsliceArgs&, hipStream_t);

// Per-descriptor record of what Rebuild does with the stripe's pattern
// (k <= 64, m <= 32), written by the host next to the stripe descriptor so a
// block knows which inputs to load from the same scalar load round trip as
// its descriptor, with no dependent load of the pattern's id rows and no
// ballots before its first data loads.
struct alignas(16) BsStripeMask {
    uint32_t dlo, dhi;  // bit j: data shard j present (it keeps its own slot)
    uint32_t pmask;     // bit t: parity t is one of Rebuild's survivors (fills an erased data slot)
    uint32_t qmask;     // bit t: parity t is erased (an output)
};

// Reconstruct launch: same stripe descriptors and pattern cache as the
// split-table kernel (rs_kernels.hpp MatArgs).
struct BitsliceRecArgs {
    uint8_t* data;               // shard id i < k at data + s*data_ss + i*pitch
    uint8_t* parity;             // shard id k + t at parity + s*parity_ss + t*pitch
    uint64_t data_ss, parity_ss, pitch;
    uint64_t count;              // descriptors
    const uint2* stripe_desc;    // [count] {stripe, pattern id << 8 | outputs}
    const BsStripeMask* stripe_mask;  // [count] the descriptors' mask records
    const uint8_t* coef;         // [npat][m][k] decode rows
    const uint32_t* src;         // [npat][k] survivor ids (Rebuild's slots)
    const uint32_t* dst;         // [npat][dst_stride] output ids
    uint32_t dst_stride;
    uint32_t ncols16;
    uint32_t blocks_per_stripe;
    const uint8_t* zpage;        // 2 KiB (one wave window) loaded for absent inputs
    const uint64_t* shard_ptrs;  // [stripe][k + m] shard addresses (pointer mode), or nullptr
    uint32_t xcd;                // XCD-aware block order (xcd.hpp): stripes per region, 0 = natural
    // Small reconstructs: stripe_desc == nullptr, the count <= kInlineDesc
    // descriptors and their mask records in the kernel arguments (no upload).
    static constexpr int kInlineDesc = 16;
    uint2 inl_desc[kInlineDesc];
    BsStripeMask inl_mask[kInlineDesc];
};

using BitsliceRecLaunch = hipError_t (*)(const BitsliceRecArgs&, hipStream_t);

struct BitsliceKernel {
    int k, m;
    const char* name;       // "bitslice_k<k>_m<m>"
    const uint8_t* matrix;  // [m][k] parity rows the kernel was generated from
    BitsliceLaunch launch;
    const char* rec_name;         // "bitslice_rec_k<k>_m<m>", or nullptr
    BitsliceRecLaunch reconstruct;  // nullptr when k > 64
    int rec_iters;                  // 8 KiB column windows per reconstruct block (gen_bitslice -I)
    // Row-subset reconstruct variants, ascending: rec_tops[i] top parity rows
    // (m - top .. m - 1) covered by rec_top_launch[i] (gen_bitslice -T).  A
    // stripe may use one when every parity row its pattern uses -- Rebuild's
    // parity survivors and the erased parity rows -- is among them.
    int n_rec_tops;
    int rec_tops[4];
    BitsliceRecLaunch rec_top_launch[4];
    const char* rec_top_names[4];
};

// Generated kernel for encode of (k, k+m), or nullptr.
const BitsliceKernel* bitslice_kernel(int k, int m);

}  // namespace rsmi
