// blake2b.hpp -- batched BLAKE2b (RFC 7693, unkeyed) on the GPU: the hash
// the plugin's sign/verify policy applies to serializeMessage(id, message)
// (main.go:38-41 defaultHashPolicy = blake2b.New(); Sign main.go:219-223,
// Verify main.go:82-89; framing main.go:276-302), for many messages per
// launch.
//
// One message per quad of lanes: lane j holds column j of the 4x4 state
// (v[j], v[4+j], v[8+j], v[12+j]), so the four column G functions run in
// parallel and the diagonal step is a DPP quad rotation of rows b, c, d.
// The 128-byte block sits in LDS, where each lane reads the message words
// its G needs in each round.  BLAKE2b chains blocks sequentially, so a
// single message uses 4 lanes; the GPU pays off for batches (hundreds to
// thousands of messages), which the host API sorts longest first so the
// quads of a wave finish together.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rsmi {

struct Blake2bArgs {
    const uint64_t* ptrs;   // [count] device addresses of the messages (any alignment)
    const uint64_t* lens;   // [count] message bytes
    const uint32_t* order;  // [count] message handled by quad q, or nullptr (identity)
    uint8_t* out;           // [count][digest_len]
    uint32_t count;
    uint32_t digest_len;    // 1..64
};

hipError_t launch_blake2b(const Blake2bArgs& a, hipStream_t stream);

// Host BLAKE2b (blake2b_host.cpp): one message, and a batch spread over
// `threads` threads (longest messages first).
void blake2b_host(const uint8_t* msg, size_t len, int digest_len, uint8_t* out);
void blake2b_host_batch(int count, const uint8_t* const* msgs, const size_t* lens, int digest_len, uint8_t* out,
                        int threads);

}  // namespace rsmi
