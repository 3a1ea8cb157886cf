// xcd_check.cpp -- host check of csrc/xcd.hpp: xcd_block() is a bijection on
// [0, total) for every region size and grid size tried, every full group of
// 8 regions gives each region to one XCD (hardware block b runs on XCD
// b % 8), and an XCD walks each of its regions in order.
#include <cstdio>
#include <vector>

#include "xcd.hpp"

int main() {
    long checked = 0;
    for (uint32_t region : {1u, 2u, 3u, 4u, 7u, 8u, 9u, 16u, 100u, 256u, 1000u}) {
        for (uint32_t total : {1u, 7u, 8u, 9u, 63u, 64u, 65u, 255u, 256u, 257u, 1000u, 2048u, 4096u + 5u,
                               8u * 256u * 3u + 17u, 131072u}) {
            std::vector<int> seen(total, 0);
            std::vector<long> last(8 * 0 + total + 1, -1);
            const uint32_t full = total - total % (8u * region);
            for (uint32_t b = 0; b < total; ++b) {
                const uint32_t L = rsmi::xcd_block(b, region, total);
                if (L >= total || seen[L]++) {
                    std::printf("not a bijection: region %u total %u b %u -> %u\n", region, total, b, L);
                    return 1;
                }
                if (b < full) {
                    const uint32_t g = L / region;  // logical region
                    if (g % 8u != b % 8u) {
                        std::printf("region %u of block %u not on XCD %u\n", g, b, b % 8u);
                        return 1;
                    }
                    // within an XCD, blocks of one region come in logical order
                    if (last[g] >= 0 && static_cast<long>(L) != last[g] + 1) {
                        std::printf("region %u out of order at block %u\n", g, b);
                        return 1;
                    }
                    last[g] = L;
                } else if (L != b) {
                    std::printf("tail block %u moved to %u\n", b, L);
                    return 1;
                }
            }
            ++checked;
        }
    }
    std::printf("xcd_block: %ld (region, total) cases ok\n", checked);
    return 0;
}
