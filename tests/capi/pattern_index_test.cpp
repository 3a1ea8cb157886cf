// pattern_index_test.cpp -- the pattern cache's host index
// (csrc/pattern_index.cpp) against plain reference implementations, built
// with AddressSanitizer/UBSan on the CPU (run by tests/test_capi_c.py):
//   * pattern_key: every n in 1..256, flags 0/1 and arbitrary non-zero
//     bytes, at unaligned addresses -- same bits and count as a byte loop;
//   * PatIndex: 300k random keys inserted, found, missed and cleared against
//     std::unordered_map, across rehashes.
#include <cstdio>
#include <cstring>
#include <random>
#include <unordered_map>
#include <vector>

#include "pattern_index.hpp"

using rsmi::PatIndex;
using rsmi::PatKey;

namespace {

struct Hash {
    size_t operator()(const PatKey& k) const { return static_cast<size_t>(rsmi::pattern_hash(k)); }
};

int failures = 0;
#define CHECK(c, ...)                                                  \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                         \
            std::fprintf(stderr, "\n");                                \
            ++failures;                                                \
        }                                                              \
    } while (0)

PatKey slow_key(const uint8_t* e, int n, int* count) {
    PatKey k{{0, 0, 0, 0}};
    *count = 0;
    for (int i = 0; i < n; ++i)
        if (e[i]) {
            k.w[i >> 6] |= uint64_t(1) << (i & 63);
            ++*count;
        }
    return k;
}

}  // namespace

int main() {
    std::mt19937_64 rng(7);
    std::vector<uint8_t> buf(300);
    for (int n = 1; n <= 256; ++n)
        for (int rep = 0; rep < 40; ++rep) {
            const int off = static_cast<int>(rng() % 8);
            const int mode = rep % 4;
            for (int i = 0; i < n; ++i) {
                const uint64_t r = rng();
                uint8_t v = 0;
                if (mode == 0) v = r % 5 == 0;                      // sparse 0/1
                else if (mode == 1) v = r & 1;                      // dense 0/1
                else if (mode == 2) v = (r % 3 == 0) ? static_cast<uint8_t>(r >> 8) : 0;  // any byte
                else v = (r % 2) ? static_cast<uint8_t>(0x80 >> (r % 8)) : 0;              // single high bits
                buf[off + i] = v;
            }
            int c1 = -1, c2 = -2;
            const PatKey a = rsmi::pattern_key(buf.data() + off, n, &c1);
            const PatKey b = slow_key(buf.data() + off, n, &c2);
            CHECK(a == b && c1 == c2, "pattern_key n=%d mode=%d", n, mode);
        }

    PatIndex idx;
    std::unordered_map<PatKey, int, Hash> ref;
    std::vector<PatKey> keys;
    for (int round = 0; round < 2; ++round) {
        for (int i = 0; i < 150000; ++i) {
            PatKey k{{rng() & rng(), (i % 3) ? 0 : rng(), 0, (i % 7) ? 0 : rng()}};
            if (ref.count(k)) continue;
            const int id = static_cast<int>(ref.size());
            CHECK(idx.find(k) == -1, "fresh key found");
            idx.insert(k, id);
            ref.emplace(k, id);
            keys.push_back(k);
        }
        CHECK(idx.size() == ref.size(), "size %zu vs %zu", idx.size(), ref.size());
        for (const PatKey& k : keys) CHECK(idx.find(k) == ref.at(k), "lookup");
        for (int i = 0; i < 100000; ++i) {
            const PatKey k{{rng(), rng(), rng(), rng()}};
            CHECK(idx.find(k) == (ref.count(k) ? ref.at(k) : -1), "miss");
        }
        // drop_from (a failed build's rollback): ids >= cut vanish, the rest
        // stay findable, and dropped keys can be inserted again.
        const int cut = static_cast<int>(ref.size()) * 2 / 3;
        idx.drop_from(cut);
        CHECK(idx.size() == static_cast<size_t>(cut), "drop_from size %zu vs %d", idx.size(), cut);
        for (const PatKey& k : keys) CHECK(idx.find(k) == (ref.at(k) < cut ? ref.at(k) : -1), "after drop_from");
        for (const PatKey& k : keys)
            if (ref.at(k) >= cut) idx.insert(k, ref.at(k));
        CHECK(idx.size() == ref.size(), "reinsert size");
        for (const PatKey& k : keys) CHECK(idx.find(k) == ref.at(k), "lookup after reinsert");
        idx.clear();
        CHECK(idx.size() == 0, "clear");
        for (const PatKey& k : keys) CHECK(idx.find(k) == -1, "found after clear");
        ref.clear();
        keys.clear();
    }
    std::printf("pattern_index_test: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
