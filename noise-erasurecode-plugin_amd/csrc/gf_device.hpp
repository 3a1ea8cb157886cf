// gf_device.hpp -- GF(2^8) (poly 0x11D) device primitives shared by the
// split-table kernels (rs_kernels.hip) and the generated bit-sliced kernels
// (gen_bitslice.cpp output).
//
//   c * x for a byte x is split over the bit fields x[2:0], x[5:3], x[7:6]:
//       c*x = Ta[x & 7] ^ Tb[(x >> 3) & 7] ^ Tc[x >> 6]
//   Ta/Tb are 8-entry byte tables (two dwords each), Tc a 4-entry table (one
//   dword); each lookup is one v_perm_b32 on four packed bytes at once.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rsmi {
namespace gfd {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t xtime(uint32_t a) {
    a <<= 1;
    return a ^ ((a & 0x100u) ? 0x11Du : 0u);
}

// Split-table words of coefficient c (host twin: gf256.cpp coef_tables).
__device__ inline void build_tables(uint32_t c, uint32_t* w) {
    uint32_t p[8];
    p[0] = c;
#pragma unroll
    for (int b = 1; b < 8; ++b) p[b] = xtime(p[b - 1]);
    auto val = [&](uint32_t v) {
        uint32_t r = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) r ^= ((v >> b) & 1u) ? p[b] : 0u;
        return r;
    };
    auto pack = [&](uint32_t base, uint32_t step) {
        return val(base) | (val(base + step) << 8) | (val(base + 2 * step) << 16) |
               (val(base + 3 * step) << 24);
    };
    w[0] = pack(0, 1);
    w[1] = pack(4, 1);
    w[2] = pack(0, 8);
    w[3] = pack(32, 8);
    w[4] = pack(0, 64) & 0xFFFFFFFFu;
}

// Per-byte bit-field selectors of four packed bytes x.
struct Fields {
    uint32_t a, b, c;
};
__device__ __forceinline__ Fields fields(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// acc ^= c * x on four packed bytes, c given by its table words T[0..4].
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, const uint32_t* T, uint32_t ia,
                                           uint32_t ib, uint32_t ic) {
    const uint32_t la = __builtin_amdgcn_perm(T[1], T[0], ia);
    const uint32_t lb = __builtin_amdgcn_perm(T[3], T[2], ib);
    const uint32_t lc = __builtin_amdgcn_perm(T[4], T[4], ic);
    return xor3(acc, la, lb) ^ lc;
}

}  // namespace gfd
}  // namespace rsmi
