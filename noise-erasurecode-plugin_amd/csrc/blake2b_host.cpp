// blake2b_host.cpp -- BLAKE2b (RFC 7693) on the host CPU, the short-batch
// side of the engine's hash policy (rs_blake2b, rsmi.h).
//
// BLAKE2b chains a message's 128-byte blocks, so the GPU kernel
// (blake2b.hip) wins only with many messages in flight: one long message
// runs a single chain on 4 lanes at ~70 MB/s there, against ~1 GB/s on one
// host core.  The plugin's single-message paths (prepareShards, Receive:
// main.go:219-223, :82-89) and small batches whose longest chain dominates
// hash here instead; the digests are identical (both follow RFC 7693 and are
// checked against hashlib in tests/).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "blake2b.hpp"

namespace rsmi {
namespace {

constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                             0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                             0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

constexpr uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline uint64_t load64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);  // x86-64 is little-endian, as BLAKE2b's words are
    return v;
}

#define B2_G(a, b, c, d, x, y)      \
    do {                            \
        a = a + b + (x);            \
        d = rotr(d ^ a, 32);        \
        c = c + d;                  \
        b = rotr(b ^ c, 24);        \
        a = a + b + (y);            \
        d = rotr(d ^ a, 16);        \
        c = c + d;                  \
        b = rotr(b ^ c, 63);        \
    } while (0)

// One 128-byte block into h; t = bytes hashed so far including this block.
inline void compress(uint64_t h[8], const uint8_t* block, uint64_t t, bool last) {
    uint64_t m[16];
    for (int i = 0; i < 16; ++i) m[i] = load64(block + 8 * i);
    uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
    uint64_t v8 = kIV[0], v9 = kIV[1], v10 = kIV[2], v11 = kIV[3];
    uint64_t v12 = kIV[4] ^ t, v13 = kIV[5];  // t < 2^64: the counter's high word stays 0
    uint64_t v14 = last ? ~kIV[6] : kIV[6], v15 = kIV[7];
#pragma GCC unroll 12
    for (int r = 0; r < 12; ++r) {
        const uint8_t* s = kSigma[r];
        B2_G(v0, v4, v8, v12, m[s[0]], m[s[1]]);
        B2_G(v1, v5, v9, v13, m[s[2]], m[s[3]]);
        B2_G(v2, v6, v10, v14, m[s[4]], m[s[5]]);
        B2_G(v3, v7, v11, v15, m[s[6]], m[s[7]]);
        B2_G(v0, v5, v10, v15, m[s[8]], m[s[9]]);
        B2_G(v1, v6, v11, v12, m[s[10]], m[s[11]]);
        B2_G(v2, v7, v8, v13, m[s[12]], m[s[13]]);
        B2_G(v3, v4, v9, v14, m[s[14]], m[s[15]]);
    }
    h[0] ^= v0 ^ v8;
    h[1] ^= v1 ^ v9;
    h[2] ^= v2 ^ v10;
    h[3] ^= v3 ^ v11;
    h[4] ^= v4 ^ v12;
    h[5] ^= v5 ^ v13;
    h[6] ^= v6 ^ v14;
    h[7] ^= v7 ^ v15;
}

#undef B2_G

}  // namespace

void blake2b_host(const uint8_t* msg, size_t len, int digest_len, uint8_t* out) {
    uint64_t h[8];
    std::memcpy(h, kIV, sizeof(h));
    h[0] ^= 0x01010000ull ^ static_cast<uint64_t>(digest_len);  // unkeyed, fanout 1, depth 1
    size_t off = 0;
    // Every block but the last goes straight from the message; the last
    // (1..128 bytes, or the single all-zero block of an empty message) is
    // zero-padded in a local buffer.
    while (len - off > 128) {
        compress(h, msg + off, off + 128, false);
        off += 128;
    }
    uint8_t last[128] = {};
    if (len > off) std::memcpy(last, msg + off, len - off);
    compress(h, last, len, true);
    uint8_t full[64];
    std::memcpy(full, h, 64);
    std::memcpy(out, full, static_cast<size_t>(digest_len));
}

void blake2b_host_batch(int count, const uint8_t* const* msgs, const size_t* lens, int digest_len, uint8_t* out,
                        int threads) {
    if (count <= 0) return;
    threads = std::max(1, std::min(threads, count));
    if (threads == 1) {
        for (int i = 0; i < count; ++i) blake2b_host(msgs[i], lens[i], digest_len, out + static_cast<size_t>(i) * digest_len);
        return;
    }
    // Longest first, handed out one at a time: the threads finish together.
    std::vector<int> order(count);
    for (int i = 0; i < count; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return lens[a] > lens[b]; });
    std::atomic<int> next{0};
    auto work = [&] {
        for (int q; (q = next.fetch_add(1)) < count;) {
            const int i = order[q];
            blake2b_host(msgs[i], lens[i], digest_len, out + static_cast<size_t>(i) * digest_len);
        }
    };
    std::vector<std::thread> pool;
    pool.reserve(threads - 1);
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (std::thread& t : pool) t.join();
}

}  // namespace rsmi
