// pattern_index.cpp -- see pattern_index.hpp.
#include "pattern_index.hpp"

#include <algorithm>
#include <cstring>

namespace rsmi {

PatKey pattern_key(const uint8_t* erased, int n, int* count) {
    PatKey key{{0, 0, 0, 0}};
    int i = 0;
    // 8 flags at a time: fold each byte onto its low bit, then gather the 8
    // low bits into one byte (bit 8j of t lands on bit 56 + j of the
    // product; no two partial products share a bit, so nothing carries).
    for (; i + 8 <= n; i += 8) {
        uint64_t t;
        std::memcpy(&t, erased + i, 8);
        t |= t >> 4;
        t |= t >> 2;
        t |= t >> 1;
        t &= 0x0101010101010101ull;
        const uint64_t bits = (t * 0x0102040810204080ull) >> 56;
        key.w[i >> 6] |= bits << (i & 63);
    }
    for (; i < n; ++i)
        if (erased[i]) key.w[i >> 6] |= uint64_t(1) << (i & 63);
    *count = __builtin_popcountll(key.w[0]) + __builtin_popcountll(key.w[1]) + __builtin_popcountll(key.w[2]) +
             __builtin_popcountll(key.w[3]);
    return key;
}

uint64_t pattern_hash(const PatKey& k) {
    uint64_t h = k.w[0] * 0x9E3779B97F4A7C15ull;
    h ^= (k.w[1] + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull;
    h ^= (k.w[2] + 0x8CB92BA72F3D8DD7ull) * 0x94D049BB133111EBull;
    h ^= (k.w[3] + 0xD6E8FEB86659FD93ull) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 31;
    h *= 0xC4CEB9FE1A85EC53ull;
    return h ^ (h >> 29);
}

int PatIndex::find(const PatKey& key) const {
    for (size_t s = pattern_hash(key) & mask_;; s = (s + 1) & mask_) {
        const int32_t id = ids_[s];
        if (id < 0) return -1;
        if (keys_[s] == key) return id;
    }
}

void PatIndex::insert(const PatKey& key, int id) {
    if (2 * (size_ + 1) > ids_.size()) rehash(2 * ids_.size());
    size_t s = pattern_hash(key) & mask_;
    while (ids_[s] >= 0) s = (s + 1) & mask_;
    keys_[s] = key;
    ids_[s] = id;
    ++size_;
}

void PatIndex::clear() {
    std::fill(ids_.begin(), ids_.end(), -1);
    size_ = 0;
}

void PatIndex::drop_from(int first_id) {
    // Linear probing cannot leave holes inside a probe run, so the kept
    // entries are reinserted into a cleared table of the same size.
    std::vector<PatKey> keys;
    std::vector<int32_t> ids;
    for (size_t s = 0; s < ids_.size(); ++s)
        if (ids_[s] >= 0 && ids_[s] < first_id) {
            keys.push_back(keys_[s]);
            ids.push_back(ids_[s]);
        }
    clear();
    for (size_t i = 0; i < ids.size(); ++i) insert(keys[i], ids[i]);
}

void PatIndex::rehash(size_t cap) {
    std::vector<PatKey> keys(cap);
    std::vector<int32_t> ids(cap, -1);
    const size_t mask = cap - 1;
    for (size_t s = 0; s < ids_.size(); ++s) {
        if (ids_[s] < 0) continue;
        size_t t = pattern_hash(keys_[s]) & mask;
        while (ids[t] >= 0) t = (t + 1) & mask;
        keys[t] = keys_[s];
        ids[t] = ids_[s];
    }
    keys_.swap(keys);
    ids_.swap(ids);
    mask_ = mask;
}

}  // namespace rsmi
