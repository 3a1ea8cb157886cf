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
};

using BitsliceLaunch = hipError_t (*)(const BitsliceArgs&, hipStream_t);

struct BitsliceKernel {
    int k, m;
    const char* name;       // "bitslice_k<k>_m<m>"
    const uint8_t* matrix;  // [m][k] parity rows the kernel was generated from
    BitsliceLaunch launch;
};

// Generated kernel for encode of (k, k+m), or nullptr.
const BitsliceKernel* bitslice_kernel(int k, int m);

}  // namespace rsmi
