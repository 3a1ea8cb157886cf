// wire_fuzz.cpp -- the erasurecode.Shard codec (csrc/shard_wire.cpp) under
// AddressSanitizer/UBSan on the CPU (run by tests/test_capi_c.py).  The
// parser reads bytes that arrive from peers (noise Receive, main.go:52), so
// every input is fed from an exactly-sized heap buffer: any read past the
// end is an ASan report.
//   * random Shards: marshal -> unmarshal round trip, views inside the input;
//   * mutations of valid encodings (byte flips, truncation, appended bytes,
//     spliced fields) and random bytes: unmarshal returns 0 or a negative
//     code, and on success every view lies inside the input;
//   * marshal into buffers of every size below rs_shard_size: RS_EWIRE_SHORT.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/rsmi.h"
#include "../../include/rsmi_wire.h"

namespace {

int failures = 0;
#define CHECK(c, ...)                                                  \
    do {                                                               \
        if (!(c)) {                                                    \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                         \
            std::fprintf(stderr, "\n");                                \
            if (++failures > 20) std::exit(1);                         \
        }                                                              \
    } while (0)

bool inside(const void* p, size_t n, const uint8_t* buf, size_t len) {
    if (n == 0) return true;
    const uint8_t* q = static_cast<const uint8_t*>(p);
    return q >= buf && q + n <= buf + len;
}

// Unmarshal from an exact-size heap copy; checks the result's invariants.
// The copy stays alive in *keep (views point into it) until the caller
// frees it.
int parse(const std::vector<uint8_t>& bytes, rs_shard_view* v, uint8_t** keep = nullptr) {
    uint8_t* buf = static_cast<uint8_t*>(std::malloc(bytes.size() ? bytes.size() : 1));
    if (!bytes.empty()) std::memcpy(buf, bytes.data(), bytes.size());
    const int rc = rs_shard_unmarshal(buf, bytes.size(), v);
    if (rc == 0) {
        CHECK(inside(v->file_signature, v->file_signature_len, buf, bytes.size()), "signature view outside input");
        CHECK(inside(v->shard_data, v->shard_data_len, buf, bytes.size()), "data view outside input");
        if (v->shard_data_len) {
            volatile uint8_t x = v->shard_data[v->shard_data_len - 1];  // touch the last byte
            (void)x;
        }
    } else {
        CHECK(rc < 0, "unmarshal returned %d", rc);
    }
    if (keep) *keep = buf;
    else std::free(buf);
    return rc;
}

std::vector<uint8_t> marshal(const rs_shard_view& v) {
    const size_t n = rs_shard_size(&v);
    std::vector<uint8_t> out(n);
    size_t w = 0;
    CHECK(rs_shard_marshal(&v, out.data(), n, &w) == 0 && w == n, "marshal");
    return out;
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    std::mt19937_64 rng(99);
    auto rnd = [&](uint64_t n) { return n ? rng() % n : 0; };
    int ok_parses = 0, err_parses = 0;
    for (int it = 0; it < iters; ++it) {
        std::vector<uint8_t> sig(rnd(3) == 0 ? 0 : rnd(130)), data(rnd(4) == 0 ? rnd(20) : rnd(3000));
        for (auto& b : sig) b = static_cast<uint8_t>(rng());
        for (auto& b : data) b = static_cast<uint8_t>(rng());
        const uint64_t big[] = {0, 1, 127, 128, 16383, 16384, (1ull << 32) - 1, 1ull << 32, ~0ull};
        rs_shard_view v{sig.data(), sig.size(), data.data(), data.size(),
                        rnd(2) ? rng() : big[rnd(9)], rnd(2) ? rnd(257) : big[rnd(9)], rnd(2) ? rnd(257) : big[rnd(9)]};
        const std::vector<uint8_t> enc = marshal(v);
        // every short output buffer is refused
        for (size_t cap = 0; cap < enc.size() && it % 50 == 0; ++cap) {
            std::vector<uint8_t> small(cap ? cap : 1);
            size_t w = 0;
            CHECK(rs_shard_marshal(&v, small.data(), cap, &w) == RS_EWIRE_SHORT, "short buffer accepted (cap %zu)", cap);
        }
        rs_shard_view u{};
        uint8_t* held = nullptr;
        CHECK(parse(enc, &u, &held) == 0, "round trip failed");
        CHECK(u.file_signature_len == sig.size() && u.shard_data_len == data.size() && u.shard_number == v.shard_number &&
                  u.total_shards == v.total_shards && u.minimum_needed_shards == v.minimum_needed_shards,
              "round trip fields");
        CHECK((sig.empty() || std::memcmp(u.file_signature, sig.data(), sig.size()) == 0) &&
                  (data.empty() || std::memcmp(u.shard_data, data.data(), data.size()) == 0),
              "round trip bytes");
        std::free(held);
        // mutations
        for (int mu = 0; mu < 8; ++mu) {
            std::vector<uint8_t> d = enc;
            switch (rnd(6)) {
                case 0:  // flip bytes
                    for (uint64_t f = 0, nf = 1 + rnd(4); f < nf && !d.empty(); ++f) d[rnd(d.size())] = static_cast<uint8_t>(rng());
                    break;
                case 1:  // truncate
                    d.resize(rnd(d.size() + 1));
                    break;
                case 2:  // append junk
                    for (uint64_t a = 0, na = 1 + rnd(12); a < na; ++a) d.push_back(static_cast<uint8_t>(rng()));
                    break;
                case 3: {  // splice a prefix of another encoding
                    const size_t cut = rnd(d.size() + 1);
                    d.resize(cut);
                    d.insert(d.end(), enc.begin(), enc.begin() + static_cast<long>(rnd(enc.size() + 1)));
                    break;
                }
                case 4:  // huge length prefix on field 1 or 2
                    d = {static_cast<uint8_t>(rnd(2) ? 0x0a : 0x12), 0xff, 0xff, 0xff, 0xff, 0x0f, 1, 2, 3};
                    break;
                default:  // random bytes
                    d.resize(rnd(64));
                    for (auto& b : d) b = static_cast<uint8_t>(rng());
            }
            rs_shard_view w{};
            (parse(d, &w) == 0 ? ok_parses : err_parses)++;
        }
    }
    // 11-byte varints and overflowing lengths
    const std::vector<std::vector<uint8_t>> edge = {
        {0x18, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x01},
        {0x18, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x01},
        {0x0a, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x01},
        {0x12, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x7f},
        {0x0a}, {0x12, 0x05, 1, 2}, {0x28}, {0x00}, {0x07}, {0x0b, 0x0c}};
    for (const auto& e : edge) {
        rs_shard_view w{};
        (parse(e, &w) == 0 ? ok_parses : err_parses)++;
    }
    std::printf("wire_fuzz: %s (%d failures; %d mutated inputs parsed, %d refused)\n", failures ? "FAILED" : "ok",
                failures, ok_parses, err_parses);
    return failures ? 1 : 0;
}
