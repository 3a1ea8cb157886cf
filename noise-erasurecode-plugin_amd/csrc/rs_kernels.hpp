// rs_kernels.hpp -- launch interface of the GF(2^8) matrix x stripe kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rsmi {

// One launch codes many stripes.  For stripe s the kernel reads the k
// survivor shards src[pat][0..k-1] and writes the e = cnt[pat] output shards
// dst[pat][0..e-1]:  out_t = sum_c coef[pat][t][c] * shard[src[pat][c]].
// Encode is the single pattern {src = 0..k-1, dst = k..n-1, coef = E_bottom}.
// Pattern p's outputs count lives in the stripe word (stripe_desc[b].y & 0xFF).
// Reconstruct lists stripes grouped by pattern: concurrently running blocks
// then read and write the same shard positions (measured ~6% faster than
// address order with mixed patterns).
// Shard id i < k lives in the data region, i >= k in the parity region
// (see rsmi.h, rs_encode_stripes).
struct MatArgs {
    uint8_t* data;
    uint8_t* parity;
    uint64_t data_ss;    // data stripe stride (bytes)
    uint64_t parity_ss;  // parity stripe stride (bytes)
    uint64_t pitch;      // shard pitch (bytes)
    uint64_t stripes;
    uint32_t ncols16;    // 16-byte columns per shard = ceil(shard_len / 16)
    uint32_t chunks;     // column chunks per stripe
    uint32_t groups;     // output-row groups per stripe
    uint32_t iters;      // block iterations per chunk
    uint32_t k, m;
    const uint8_t* coef;         // [npat][m][k]
    const uint32_t* src;         // [npat][k]   survivor shard ids, or nullptr: survivor j is
                                 // shard id j (single-pattern launches whose shard table or
                                 // strided layout is already in survivor order)
    const uint32_t* dst;         // [npat][dst_stride] output shard ids (padded, >= 16)
    uint32_t dst_stride;
    const uint2* stripe_desc;    // [stripes] {stripe index, pattern id << 8 | outputs}
                                 // in processing order, or nullptr: stripe b, pattern 0
                                 // with all m rows (encode)
    const uint64_t* shard_ptrs;  // [stripe][k + m] device address of every shard (pointer
                                 // mode: data/parity/strides/pitch unused), or nullptr
    uint32_t xcd;                // XCD-aware block order (xcd.hpp): blocks per region, or 0
                                 // (natural); ~0u = all of a stripe's blocks (set at launch)
    uint32_t desc0;              // stripe_desc == nullptr: every stripe's {pattern << 8 |
                                 // outputs} word (0: pattern 0 with all m rows, the encode)
    // Small reconstructs (at most kInlineDesc descriptors): the descriptors
    // ride in the kernel arguments (stripe_desc == nullptr, n_inline > 0) --
    // no upload of a descriptor array ahead of the kernel.
    static constexpr int kInlineDesc = 16;
    uint32_t n_inline;
    uint2 inl_desc[kInlineDesc];
};

// Fills in chunks/groups/iters from k, m, ncols16 and launches the kernel
// variant for (k, m).  max_e bounds cnt[] over all patterns.
hipError_t launch_matmul(MatArgs a, int max_e, hipStream_t stream);

// Mailbox grid (rs_encode / rs_decode of one small message): one launch per
// call of the split-table kernel, a group of blocks per column-chunk job,
// each group coding its job as soon as the host has staged it and bumped
// `posted` -- instead of a launch, a dispatch and a completion event per
// chunk.  Every job's arguments are known before the staging starts and go
// in the launch's kernel arguments; the host's post is one word, and job j's
// group writes done[j - 1] = j.  quit (host) makes the groups still waiting
// for their job leave.
constexpr int kMailboxJobs = 4;
struct MailboxJob {
    MatArgs a;        // chunks / groups / iters planned (plan_mailbox_job), xcd 0
    uint32_t blocks;  // logical blocks of the job
    uint32_t pad[3];
};
struct MailboxJobs {  // by value in the kernel arguments
    MailboxJob job[kMailboxJobs];
};
struct MailboxHost {  // pinned (coherent), device-mapped; read by the grid with system-scope loads
    uint64_t posted;  // host: jobs posted (staged) so far
    uint64_t quit;    // host: nonzero = groups still waiting leave
    uint64_t pad0[14];
    uint64_t done[kMailboxJobs];  // grid: done[j - 1] = j once job j is coded
    uint64_t gave_up;             // grid: nonzero once a group left without its job (timeout or quit)
    uint64_t pad1[11];
};
struct MailboxDev {  // device memory: zero between launches (the grid's last block out zeroes it)
    uint32_t left;    // blocks that have left
    uint32_t arrive[kMailboxJobs];  // blocks of job j's group finished with it
    uint32_t pad[11];
    // Diagnostics (launch_mailbox's stamps flag, RSMI_MAILBOX_STAMPS):
    // device wall clock at block 0's entry, then per job when its group's
    // first block saw it posted, had its arguments, and when the group's
    // last block stored done.
    uint64_t stamp[1 + 3 * kMailboxJobs];
};

// Whether a mailbox grid serves jobs of k survivors and up to `rows`
// outputs per stripe (the split-table variants for RS(10,4) and RS(4,2)).
bool mailbox_supported(int k, int rows);
// Fills job->a's launch plan (as launch_matmul would) and job->blocks.
void plan_mailbox_job(const MatArgs& a, int max_e, MailboxJob* job);
// Launches njobs (1..kMailboxJobs) groups of per_job blocks for jobs[0 ..
// njobs) (a group codes its job's logical blocks in turn).  A block waits at most `timeout` device
// wall-clock ticks (hipDeviceAttributeWallClockRate) for its job to be
// posted; a job whose group gave up stays undone (the caller codes it with
// an ordinary launch after the stream drained).  h is the device alias of
// the MailboxHost.
hipError_t launch_mailbox(MailboxHost* h, MailboxDev* d, const MailboxJobs& jobs, int njobs, int k, int rows,
                          uint32_t per_job, uint64_t timeout, hipStream_t stream, bool stamps = false);

// Which compiled variant serves (k, m): "K10_MG4" etc. (diagnostics).
const char* variant_name(int k, int rows);  // kernel coding up to `rows` outputs per stripe

// Device-side copy of `count` pieces of `bytes` bytes (a multiple of 16):
// piece i copies src + pieces[2i] to dst + pieces[2i+1] (16-byte aligned
// offsets).  rs_decode_batch packs survivors / unpacks regenerated shards
// with it so PCIe carries only those.
hipError_t launch_copy_pieces(const uint8_t* src, uint8_t* dst, const uint64_t* pieces, uint32_t count,
                              size_t bytes, hipStream_t stream);

// splitmix64 byte stream fill (bench/test utility).
hipError_t launch_fill_splitmix(void* dev, size_t len, uint64_t seed, hipStream_t stream);

}  // namespace rsmi
