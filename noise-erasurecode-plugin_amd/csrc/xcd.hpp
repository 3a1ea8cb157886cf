// xcd.hpp -- XCD-aware block order for the streaming kernels.
//
// The MI355X dispatcher hands workgroups to its 8 XCDs round-robin (block b
// runs on XCD b % 8).  With the natural order (block = stripe * per + piece)
// the `per` blocks of one stripe land on 8 different XCDs at once, and every
// XCD reads a scattered 1/8 of every shard.  xcd_block() renumbers the grid
// so that XCD x runs stripes x, x + 8, x + 16, ... and walks all `per` pieces
// of each in order: a stripe's shards are streamed by one XCD, contiguously.
// Movement-only twins of the encode shapes (tools/membench8.hip,
// profiles/r02aj/): RS(64,16) with 64 KiB shards 5.48 -> 6.58 TB/s,
// RS(10,4) with 1 MiB shards 6.18 -> 6.29 TB/s.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rsmi {

// Logical block of hardware block b in a grid of `total` blocks, with the
// grid cut into regions of `region` consecutive logical blocks dealt to the
// XCDs in turn: XCD x runs regions x, x + 8, x + 16, ... and each region's
// blocks in order.  region = blocks per stripe gives every stripe to one XCD;
// region = 1 is the natural order.  A bijection on [0, total): the tail that
// does not fill 8 regions keeps the natural order (it is dispatched last
// either way).  Grids are < 2^31 blocks.
__host__ __device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t region, uint32_t total) {
    const uint32_t full = total - total % (8u * region);
    if (b >= full) return b;
    const uint32_t x = b & 7u, i = b >> 3;
    const uint32_t q = i / region;
    return (q * 8u + x) * region + (i - q * region);
}

}  // namespace rsmi
