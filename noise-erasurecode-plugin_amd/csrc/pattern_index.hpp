// pattern_index.hpp -- host side of the decode-pattern cache: erasure
// patterns as 256-bit keys and an open-addressing index from key to pattern
// id.  Pure host code (no HIP), unit-tested on the CPU
// (tests/capi/pattern_index_test.cpp).
//
// A batched reconstruct looks up one pattern per stripe (BASELINE configs
// 3/5: thousands of stripes per call, up to one fresh pattern each), so the
// lookup is on every call's critical path: the key is built 8 flags at a
// time and the index is a flat table probed linearly (one or two cache lines
// per lookup, no allocation per pattern).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace rsmi {

// Bit i set <=> shard i erased (n <= 256).
struct PatKey {
    uint64_t w[4];
    bool operator==(const PatKey& o) const {
        return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3];
    }
    bool has(int i) const { return (w[i >> 6] >> (i & 63)) & 1u; }
};

// Key of n erasure flags (any non-zero byte = erased); *count = erased shards.
PatKey pattern_key(const uint8_t* erased, int n, int* count);

uint64_t pattern_hash(const PatKey& k);

class PatIndex {
public:
    PatIndex() { rehash(1024); }
    // Pattern id of `key`, or -1.
    int find(const PatKey& key) const;
    // Adds key -> id; the key must be absent.
    void insert(const PatKey& key, int id);
    void clear();
    // Removes every entry whose id is >= first_id (a failed build's patterns).
    void drop_from(int first_id);
    size_t size() const { return size_; }

private:
    void rehash(size_t cap);
    std::vector<PatKey> keys_;
    std::vector<int32_t> ids_;  // -1: empty slot
    size_t mask_ = 0, size_ = 0;
};

}  // namespace rsmi
