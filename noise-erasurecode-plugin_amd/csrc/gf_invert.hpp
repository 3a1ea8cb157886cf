// gf_invert.hpp -- batched GPU construction of decode rows (gf_invert.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rsmi {

struct InvertArgs {
    const uint8_t* enc;      // [n][k] systematic matrix
    const uint8_t* gf_exp;   // [512] 2^i (i < 510)
    const uint8_t* gf_log;   // [256]
    // With keys: pattern first + i is the erasure bitmask keys[i][0..3] (bit
    // j set <=> shard j erased); the kernel derives its survivor ids
    // (Rebuild's choice), erased ids and count and writes them to src, dst
    // and cnt.  Without keys the three are inputs.
    const uint64_t* keys;    // [count][4] or nullptr
    uint32_t* src;           // [npat][k] survivor ids
    uint32_t* dst;           // [npat][dst_stride] erased ids (zero past the count)
    uint32_t* cnt;           // [npat] erased count
    uint32_t dst_stride;
    uint8_t* coef;           // [npat][m][k] decode rows (output)
    uint32_t first;          // first pattern id to build
    uint32_t k, m;
    uint32_t* status;        // [npat]: 1 if the pattern's survivor matrix is singular, else 0
    uint32_t generic;        // 1: whole k x k Gauss-Jordan even for Rebuild-shaped survivor sets (A/B)
};

// Builds patterns [first, first + count): one workgroup each.
hipError_t launch_invert(const InvertArgs& a, uint32_t count, hipStream_t stream);
size_t invert_lds_bytes(int k, int m);

}  // namespace rsmi
