// rsmi.cpp -- C ABI of the engine (include/rsmi.h).  Host-side bookkeeping
// around the HIP kernels: encode/decode matrices, the per-ctx decode-pattern
// cache, and the per-call leases of streams, device workspaces and pinned
// staging.  The GF products themselves always run on the GPU; there is no CPU
// compute fallback.
#include "../../include/rsmi.h"

#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <functional>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <thread>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <vector>

#include "bitslice.hpp"
#include "blake2b.hpp"
#include "device_set.hpp"
#include "gf256.hpp"
#include "gf_invert.hpp"
#include "host_pipeline.hpp"
#include "pattern_index.hpp"
#include "pinned.hpp"
#include "rs_kernels.hpp"

namespace {

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Restores the caller's current HIP device on scope exit.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// A growable device buffer.  reserve() is for buffers sized once (the
// context's immutable tables, at rs_new).  reserve_on() is stream-ordered
// (hipMallocAsync / hipFreeAsync on s): the caller has ordered s after every
// earlier user of the buffer (a lease's begin()), so the outgrown allocation
// is freed on the device timeline with no host or device-wide sync -- a
// caller whose request outgrows the buffer never stalls the others (hipFree
// would: it implies a hipDeviceSynchronize).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool stream_ordered = false;  // allocated by reserve_on
    bool reserve(size_t bytes) {
        if (bytes <= cap) return true;
        release();
        size_t want = std::max(bytes, size_t(4096));
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = want;
        return true;
    }
    bool reserve_on(size_t bytes, hipStream_t s) {
        if (bytes <= cap) return true;
        const size_t want = std::max({bytes, size_t(4096), 2 * cap});
        if (p) {
            if ((stream_ordered ? hipFreeAsync(p, s) : hipFree(p)) != hipSuccess) return false;
            p = nullptr;
            cap = 0;
        }
        if (hipMallocAsync(&p, want, s) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = want;
        stream_ordered = true;
        return true;
    }
    // Callers have drained every user of the buffer (rs_free / lease
    // teardown); the stream of the allocation may be gone (a caller's), so a
    // stream-ordered buffer is freed on the null stream.
    void release() {
        if (p) {
            if (stream_ordered) {
                (void)hipFreeAsync(p, nullptr);
                (void)hipStreamSynchronize(nullptr);
            } else {
                (void)hipFree(p);
            }
        }
        p = nullptr;
        cap = 0;
        stream_ordered = false;
    }
};

// A growable device buffer whose first `used` bytes survive growth, read by
// launches on many streams (the pattern tables).  Growth is stream-ordered on
// the build stream s, which the caller has first ordered after the last
// launch of every lease (order_after_readers): the old allocation is copied
// and then freed on s, never by a host-side sync.
struct GrowBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool reserve_keep(size_t bytes, size_t used, hipStream_t s) {
        if (bytes <= cap) return true;
        const size_t want = std::max({bytes, size_t(4096), 4 * cap});
        void* np = nullptr;
        if (hipMallocAsync(&np, want, s) != hipSuccess) return false;
        if (p && used &&
            hipMemcpyAsync(np, p, std::min(used, cap), hipMemcpyDeviceToDevice, s) != hipSuccess) {
            (void)hipFreeAsync(np, s);
            return false;
        }
        if (p) (void)hipFreeAsync(p, s);
        p = np;
        cap = want;
        return true;
    }
    bool needs(size_t bytes) const { return bytes > cap; }
    void release() {  // every reader drained (rs_free)
        if (p) {
            (void)hipFreeAsync(p, nullptr);
            (void)hipStreamSynchronize(nullptr);
        }
        p = nullptr;
        cap = 0;
    }
};

// Pinned host staging whose reuse waits for the copies that read it.
// Growth never frees on the hot path (hipHostFree implies a device-wide
// sync): the outgrown buffer is retired and freed at destroy(); growth is
// x2, so the retired buffers never exceed the live one.
struct Staging {
    void* p = nullptr;
    void* dev = nullptr;  // p's device alias (queried once per allocation, not per call)
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;  // hipHostMallocWriteCombined: the host only ever writes it
    hipEvent_t done = nullptr;
    bool pending = false;
    std::vector<void*> retired;
    bool acquire(size_t bytes) {
        if (pending) {
            (void)hipEventSynchronize(done);
            pending = false;
        }
        if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) return false;
        if (bytes <= cap) return true;
        const size_t want = std::max({bytes, size_t(1) << 16, 2 * cap});
        void* np = nullptr;
        if (hipHostMalloc(&np, want, flags) != hipSuccess) return false;
        if (p) retired.push_back(p);
        p = np;
        if (hipHostGetDevicePointer(&dev, np, 0) != hipSuccess) dev = np;
        cap = want;
        return true;
    }
    void release_after(hipStream_t s) {
        if (hipEventRecord(done, s) == hipSuccess) pending = true;
    }
    void destroy() {
        if (pending) (void)hipEventSynchronize(done);
        for (void* r : retired) (void)hipHostFree(r);
        retired.clear();
        if (p) (void)hipHostFree(p);
        if (done) (void)hipEventDestroy(done);
        p = nullptr;
        dev = nullptr;
        done = nullptr;
    }
};

}  // namespace

// rs_decode_batch moves survivors in / regenerated shards out in up to
// kBatchChunks pieces once a direction carries kBatchChunkMin bytes.
constexpr size_t kBatchChunks = 4;
constexpr size_t kBatchChunksMax = 8;  // the direct batch forms' cap (RSMI_BATCH_CHUNKS); events per lease
constexpr size_t kBatchChunkMin = size_t(16) << 20;

// An erasure pattern as a 256-bit set of shard ids (n <= 256).
using rsmi::PatKey;

namespace {

// Per-call resources: every C-ABI call that needs a stream, staging or a
// device workspace leases one of these from its ctx, so concurrent callers
// (noise runs Receive once per peer connection, main.go:49-52) never share
// them.  dev_done is recorded after the last GPU operation that reads the
// lease's device buffers; the next user of the lease -- possibly on another
// stream -- waits for it on the device (begin()), never on the host.
struct Lease {
    hipStream_t stream = nullptr;  // host API / decode_batch / pattern rows
    // A single message's odd column chunks (decode_launch, encode_staged) with
    // RSMI_CHUNK_STREAMS=2: on one stream a chunk's kernel starts 5.4 us after
    // the previous one ends (profiles/r06h/); on a stream of its own it
    // overlaps it, but the host copies that run meanwhile slowed 2.5x and the
    // config-1 decode went 58.0 -> 67.2 us (profiles/r06i/), so one stream is
    // the default.  Created on first use; joined back into `stream` before the
    // lease's end().
    hipStream_t stream2 = nullptr;
    hipEvent_t dev_done = nullptr;
    std::atomic<bool> dev_pending{false};
    hipEvent_t ev[kBatchChunksMax] = {};  // per-chunk events (single messages, batches)
    Staging st_stripe;                 // stripe descriptors
    Staging st_batch, st_pieces;       // rs_decode_batch
    Staging st_onepat;                 // host-API decode: the one-pattern table, read in place by the kernel
    Staging st_out;                    // decode_in_place: regenerated shares when dst is not engine-pinned
    Staging st_in;                     // decode_staged / encode_staged: a small message's survivors
    // Mailbox grid of a staged single message (MailboxCall): the job board
    // in pinned coherent memory, its device alias and the grid's device
    // words; allocated on first use.
    rsmi::MailboxHost* mb = nullptr;
    rsmi::MailboxHost* mb_dev = nullptr;
    rsmi::MailboxDev* mbd = nullptr;
    uint64_t mb_timeout = 0;  // the grid's wait for a post in device wall-clock ticks (mailbox_timeout_us)
    DevBuf d_stripe_pat, d_batch, d_pack, d_pieces, d_onepat;
    std::unique_ptr<rsmi::HostPipeline> pipe;  // host-buffer API, created on first use
    std::vector<uint32_t> pid, start;          // reconstruct scratch
    std::vector<uint64_t> sort_a, sort_b;      // (bucket, stripe) radix-sort scratch
    std::vector<PatKey> miss_keys;             // distinct new patterns of a call
    // The pattern rows this lease's launches are known to be ordered after:
    // ids below seen_uploaded of table generation seen_tables (launch_reconstruct
    // waits for pat_ev only for a pattern built since, or after the tables
    // moved -- growth or eviction -- so a caller whose patterns are all old
    // never queues behind another caller's build).
    size_t seen_uploaded = 0;
    uint64_t seen_tables = ~uint64_t(0);

    bool init() {
        // RSMI_STAGE_WC=1: a single message's input staging in write-combined
        // memory -- the host writes it with streaming stores only, and the
        // kernel's PCIe reads of it need not snoop the CPU's caches.
        static const bool wc = [] {
            const char* e = std::getenv("RSMI_STAGE_WC");
            return e && std::atoi(e) != 0;
        }();
        if (wc) st_in.flags = hipHostMallocWriteCombined;
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&dev_done, hipEventDisableTiming) != hipSuccess) return false;
        for (hipEvent_t& e : ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
        return true;
    }
    // The next GPU use of the lease's device buffers, on stream s, follows
    // the previous one (which may have been on another stream).
    void begin(hipStream_t s) {
        if (dev_pending.load()) (void)hipStreamWaitEvent(s, dev_done, 0);
    }
    void end(hipStream_t s) {
        if (hipEventRecord(dev_done, s) == hipSuccess) dev_pending.store(true);
    }
    rsmi::HostPipeline* pipeline() {
        if (!pipe) pipe.reset(new (std::nothrow) rsmi::HostPipeline());
        return pipe.get();
    }
    // The stream of a single message's chunk ch: chunk 0 (and, without a
    // second stream, every chunk) on `stream`, odd chunks on stream2 when
    // two streams are in use (RSMI_CHUNK_STREAMS=2).
    hipStream_t chunk_stream(int ch) {
        static const bool two = [] {
            const char* e = std::getenv("RSMI_CHUNK_STREAMS");
            return e && std::atoi(e) == 2;
        }();
        if (!two || ch % 2 == 0) return stream;
        if (!stream2 && hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking) != hipSuccess) stream2 = nullptr;
        return stream2 ? stream2 : stream;
    }
    ~Lease() {
        if (stream2) (void)hipStreamSynchronize(stream2);
        if (stream) (void)hipStreamSynchronize(stream);
        if (dev_pending.load()) (void)hipEventSynchronize(dev_done);
        pipe.reset();
        st_stripe.destroy();
        st_batch.destroy();
        st_pieces.destroy();
        st_onepat.destroy();
        st_out.destroy();
        st_in.destroy();
        for (DevBuf* b : {&d_stripe_pat, &d_batch, &d_pack, &d_pieces, &d_onepat}) b->release();
        if (mb) (void)hipHostFree(mb);
        if (mbd) (void)hipFree(mbd);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (dev_done) (void)hipEventDestroy(dev_done);
        if (stream2) (void)hipStreamDestroy(stream2);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

}  // namespace

struct rs_ctx {
    int k = 0, n = 0, m = 0, device = 0;
    std::vector<uint8_t> enc;  // n x k systematic matrix
    // Device-set context (rs_new_devices): the members do all the work and
    // every entry point forwards to them (device_set.hpp); nullptr for a
    // single-device context, whose state is everything below.
    rsmi::DeviceSet* set = nullptr;
    bool set_member = false;  // owned by a device set: rs_free on it is a no-op (the set frees it)
    // Generated bit-sliced encode kernel for this (k, n), if one was built
    // and its embedded matrix equals enc (bitslice.hpp); nullptr otherwise.
    const rsmi::BitsliceKernel* bitslice = nullptr;
    bool bitslice_rec = false;  // batched reconstruct uses bitslice->reconstruct ...
    int bitslice_rec_min_e = 1;  // ... for stripes with at least this many erasures
    uint32_t xcd = 1;            // XCD-aware block order in the streaming kernels (RSMI_XCD) ...
    uint32_t xcd_split_enc = 0;  // ... split-table encode: blocks per region (0: natural order; RSMI_XCD_ENC_REGION)
    uint32_t xcd_split_rec = ~0u;  // ... split-table reconstruct: blocks per region (~0u: a stripe; RSMI_XCD_REC_REGION)
    std::string rec_name;        // rs_kernel_name(ctx, 1) when bitslice_rec
    bool inline_desc = true;     // small reconstructs: descriptors in the kernel arguments
    size_t small_split = 16;     // bit-sliced codes: calls of at most this many erased stripes use the split table

    // Immutable after rs_new: encode pattern (PatBlob layout, one pattern)
    // and enc [n][k] | gf exp [512] | gf log [256] | 2 KiB zero page.
    DevBuf d_encpat;
    DevBuf d_gf;

    // Decode-pattern cache, the only state calls share.  The host keeps each
    // pattern's survivor / erased ids; the device holds the same plus its
    // decode rows and status, which the GPU builds (gf_invert.hip) when a
    // pattern is first seen.  Lookups and the launches that read the device
    // tables hold pat_mu shared; creating patterns, growing the tables and
    // eviction hold it exclusively.  pat_ev is recorded after every build
    // (each build first waits for the previous one), so a launch on any
    // stream that waits for it sees every row built so far.
    mutable std::shared_mutex pat_mu;
    rsmi::PatIndex pat_index;
    std::vector<uint32_t> h_cnt;  // [npat] erased count of each pattern
    std::vector<uint8_t> h_lo;    // [npat] lowest parity row the pattern uses (m: none)
    std::vector<rsmi::BsStripeMask> h_mask;  // [npat] Rebuild's slots and rows (bit-sliced reconstruct)
    int n_tops = 0;               // row-subset syndrome kernels in use (RSMI_BITSLICE_TOPS=0: none)
    std::vector<PatKey> h_key;    // keys of the patterns created since the last flush
    GrowBuf d_pcoef, d_psrc, d_pdst, d_pcnt, d_pstat, d_pkey;
    size_t uploaded = 0;    // patterns built on the device
    size_t pat_cap = 0;     // soft bound; reaching it evicts the whole cache
    int test_fail_flush = 0, flush_attempts = 0;  // RSMI_TEST_FAIL_FLUSH (tests)
    uint64_t evictions = 0;
    uint64_t tables_gen = 0;  // bumped when the device tables move (growth) or are rebuilt (eviction)
    std::atomic<int64_t> batches_in_place{0}, batches_staged{0};  // rs_decode_batch paths (rs_stat)
    std::atomic<int64_t> encodes_in_place{0};                     // rs_encode from engine-pinned memory
    std::atomic<int64_t> decodes_in_place{0};                     // rs_decode from engine-pinned memory
    std::atomic<int64_t> rec_stripes_table{0}, rec_stripes_syndrome{0};  // launch_reconstruct's kernels (rs_stat)
    std::atomic<int64_t> encode_batches{0};                              // rs_encode_batch calls through the GPU
    std::atomic<int64_t> mailbox_calls{0}, mailbox_recovered{0};         // MailboxCall (rs_stat)
    hipEvent_t pat_ev = nullptr;
    hipStream_t build_stream = nullptr;  // pattern builds (flush_patterns), off every caller's stream
    hipEvent_t caller_ev = nullptr;      // the building caller's stream tail (build_after_caller)
    bool build_after_caller = true;      // RSMI_BUILD_OVERLAP=1: builds overlap the caller's queued kernels
    bool pat_ev_valid = false;
    Staging st_pat;  // pattern-table uploads

    // Lease pool (FIFO: the least recently released lease is handed out).
    std::mutex lease_mu;
    std::condition_variable lease_cv;
    std::vector<std::unique_ptr<Lease>> leases;
    std::deque<Lease*> free_leases;
    size_t max_leases = 16;
};


namespace {

int hip_status(hipError_t e) { return e == hipSuccess ? RS_OK : RS_EDEVICE; }

// ------------------------------------------------------------- leases ----
Lease* acquire_lease(rs_ctx* c) {
    std::unique_lock<std::mutex> lk(c->lease_mu);
    c->lease_cv.wait(lk, [&] { return !c->free_leases.empty() || c->leases.size() < c->max_leases; });
    if (!c->free_leases.empty()) {
        Lease* L = c->free_leases.front();
        c->free_leases.pop_front();
        return L;
    }
    std::unique_ptr<Lease> L(new (std::nothrow) Lease());
    if (!L || !L->init()) return nullptr;
    c->leases.push_back(std::move(L));
    return c->leases.back().get();
}

void release_lease(rs_ctx* c, Lease* L) {
    {
        std::lock_guard<std::mutex> lk(c->lease_mu);
        c->free_leases.push_back(L);
    }
    c->lease_cv.notify_one();
}

struct LeaseGuard {
    rs_ctx* c;
    Lease* L;
    explicit LeaseGuard(rs_ctx* ctx) : c(ctx), L(acquire_lease(ctx)) {}
    ~LeaseGuard() {
        if (L) release_lease(c, L);
    }
};

// Output ids per pattern are padded to a multiple of 16 so the kernel can
// load a whole row group's ids unconditionally.
size_t dst_stride(const rs_ctx* c) { return std::max<size_t>(16, round_up(c->m, 16)); }

// Device blob of npat patterns: coef bytes [npat][m][k] (padded to 16) |
// src u32 [npat][k] | dst u32 [npat][dst_stride] | sw u32x2 [npat], where
// sw[p] = {0, p << 8 | outputs} is the descriptor of stripe 0 using pattern p.
struct PatLayout {
    size_t coef, src, dst, sw, total;
    PatLayout(const rs_ctx* c, size_t npat) {
        coef = 0;
        src = round_up(npat * c->m * c->k, 16);
        dst = src + npat * c->k * 4;
        sw = round_up(dst + npat * dst_stride(c) * 4, 8);
        total = sw + npat * 8;
    }
};

void pack_patterns(const rs_ctx* c, size_t npat, const uint8_t* coef, const uint32_t* src,
                   const uint32_t* dst, const uint32_t* cnt, uint8_t* out) {
    PatLayout L(c, npat);
    const size_t ds = dst_stride(c);
    std::memset(out, 0, L.total);
    std::memcpy(out + L.coef, coef, npat * c->m * c->k);
    std::memcpy(out + L.src, src, npat * c->k * 4);
    for (size_t p = 0; p < npat; ++p) {
        std::memcpy(out + L.dst + p * ds * 4, dst + p * c->m, c->m * 4);
        const uint32_t desc[2] = {0u, static_cast<uint32_t>(p << 8) | cnt[p]};
        std::memcpy(out + L.sw + p * 8, desc, 8);
    }
}

void set_patterns(const rs_ctx* c, size_t npat, const void* dev, rsmi::MatArgs& a) {
    PatLayout L(c, npat);
    const uint8_t* b = static_cast<const uint8_t*>(dev);
    a.coef = b + L.coef;
    a.src = reinterpret_cast<const uint32_t*>(b + L.src);
    a.dst = reinterpret_cast<const uint32_t*>(b + L.dst);
    a.dst_stride = static_cast<uint32_t>(dst_stride(c));
    a.stripe_desc = nullptr;
}

// Descriptor {stripe 0, sw[0]} of a one-pattern blob (single-stripe launches
// with e < m outputs): the blob's sw section holds {0, p << 8 | cnt} pairs.
const uint2* first_stripe_desc(const rs_ctx* c, const void* dev) {
    return reinterpret_cast<const uint2*>(static_cast<const uint8_t*>(dev) + PatLayout(c, 1).sw);
}

bool check_stripes_args(const rs_ctx* c, const void* data, size_t dss, const void* parity,
                        size_t pss, size_t pitch, size_t len) {
    auto al = [](uintptr_t v) { return (v & 15u) == 0; };
    if (!data || (!parity && c->m > 0)) return false;
    if (!al(reinterpret_cast<uintptr_t>(data)) || !al(reinterpret_cast<uintptr_t>(parity)))
        return false;
    if (!al(dss) || !al(pss) || !al(pitch)) return false;
    if (pitch < round_up(len, 16)) return false;
    if (round_up(len, 16) / 16 >= (size_t(1) << 28)) return false;  // 32-bit column offsets
    return true;
}

rsmi::MatArgs base_args(const rs_ctx* c, void* data, size_t dss, void* parity, size_t pss,
                        size_t pitch, size_t len, size_t stripes) {
    rsmi::MatArgs a{};
    a.data = static_cast<uint8_t*>(data);
    a.parity = static_cast<uint8_t*>(parity);
    a.data_ss = dss;
    a.parity_ss = pss;
    a.pitch = pitch;
    a.stripes = stripes;
    a.ncols16 = static_cast<uint32_t>(round_up(len, 16) / 16);
    a.k = static_cast<uint32_t>(c->k);
    a.m = static_cast<uint32_t>(c->m);
    a.xcd = c->xcd_split_rec;  // split-table reconstruct: a stripe per XCD region by default
    return a;
}

// Generated bit-sliced encode kernel for (k, m) if the build has one whose
// embedded matrix is this context's.  By default it serves the codes whose
// split-table encode does at least 3 MACs per byte moved, k*m >= 3(k+m):
// RS(64,16) (12.8) and RS(8,14) (3.4, profiles/r02bq), not RS(10,4) (2.9,
// at its movement ceiling either way).  The RSMI_BITSLICE knob forces it on
// (1) or off (0) for A/B runs.
const rsmi::BitsliceKernel* pick_bitslice(const std::vector<uint8_t>& enc, int k, int m) {
    const char* e = std::getenv("RSMI_BITSLICE");
    if (e && std::atoi(e) == 0) return nullptr;
    if (!e && k * m < 3 * (k + m)) return nullptr;
    const rsmi::BitsliceKernel* b = rsmi::bitslice_kernel(k, m);
    if (!b) return nullptr;
    const uint8_t* bottom = enc.data() + static_cast<size_t>(k) * k;
    return std::memcmp(b->matrix, bottom, static_cast<size_t>(m) * k) == 0 ? b : nullptr;
}

// Encode launch (all parity rows of every stripe): the generated bit-sliced
// kernel when there is one for this code, else the split-table kernel.
hipError_t launch_encode(const rs_ctx* c, const rsmi::MatArgs& a, hipStream_t s) {
    if (!c->bitslice) {
        rsmi::MatArgs e = a;
        e.xcd = c->xcd_split_enc;
        return rsmi::launch_matmul(e, c->m, s);
    }
    rsmi::BitsliceArgs b{};
    b.data = a.data;
    b.parity = a.parity;
    b.data_ss = a.data_ss;
    b.parity_ss = a.parity_ss;
    b.pitch = a.pitch;
    b.stripes = a.stripes;
    b.ncols16 = a.ncols16;
    b.blocks_per_stripe = (a.ncols16 + 511u) / 512u;  // 256 lanes x 2 columns per block
    b.xcd = c->xcd;
    return c->bitslice->launch(b, s);
}

// Batched reconstruct through the generated bit-sliced kernel: whenever the
// code's encode is bit-sliced and a reconstruct twin was generated (k <= 64).
// RSMI_BITSLICE_REC=0 keeps the split-table kernel (A/B runs).
// Read at rs_new, like RSMI_BITSLICE.
bool use_bitslice_rec(const rs_ctx* c) { return c->bitslice_rec; }

bool pick_bitslice_rec(const rsmi::BitsliceKernel* b) {
    const char* e = std::getenv("RSMI_BITSLICE_REC");
    if (e && std::atoi(e) == 0) return false;
    return b && b->reconstruct;
}

// ----------------------------------------------------- pattern cache ----
// Creates the decode pattern for `key` (pat_mu held exclusively): an id, its
// erased count and a pending key.  The survivor and erased-id rows are
// derived from the key on the GPU when the pattern is built
// (invert_patterns_kernel), so a fresh pattern costs the host one index
// insert and 32 bytes of upload.
// Lowest parity row a pattern uses (m if none): its erased parity rows
// (outputs) and Rebuild's parity survivors, which fill the d erased data
// slots from the top: the d highest-numbered present parity rows.  Decides
// which row-subset syndrome kernel covers the pattern.
int lowest_parity_row(const PatKey& key, int k, int n) {
    const int m = n - k;
    int d = 0;
    for (int i = 0; i < k; ++i) d += key.has(i);
    int lo = m;
    for (int t = m - 1; t >= 0; --t) {
        if (key.has(k + t)) {
            lo = t;  // erased parity row: an output
        } else if (d > 0) {
            lo = t;  // parity survivor filling an erased data slot
            --d;
        }
    }
    return lo;
}

// The syndrome kernel's mask record of a pattern (bitslice.hpp
// BsStripeMask; k <= 64, m <= 32, zeros otherwise): present data shards,
// Rebuild's parity survivors -- the d highest-numbered present parity rows,
// d = erased data shards -- and the erased parity rows.
rsmi::BsStripeMask stripe_mask(const PatKey& key, int k, int n) {
    const int m = n - k;
    rsmi::BsStripeMask r{0u, 0u, 0u, 0u};
    if (k > 64 || m > 32) return r;
    uint64_t present = 0;
    int d = 0;
    for (int i = 0; i < k; ++i) {
        if (key.has(i)) ++d;
        else present |= 1ull << i;
    }
    for (int t = m - 1; t >= 0; --t) {
        if (key.has(k + t)) {
            r.qmask |= 1u << t;
        } else if (d > 0) {
            r.pmask |= 1u << t;
            --d;
        }
    }
    r.dlo = static_cast<uint32_t>(present);
    r.dhi = static_cast<uint32_t>(present >> 32);
    return r;
}

int create_pattern(rs_ctx* c, const PatKey& key, int e) {
    const int id = static_cast<int>(c->h_cnt.size());
    c->h_cnt.push_back(static_cast<uint32_t>(e));
    c->h_lo.push_back(static_cast<uint8_t>(lowest_parity_row(key, c->k, c->n)));
    c->h_mask.push_back(stripe_mask(key, c->k, c->n));
    c->h_key.push_back(key);
    c->pat_index.insert(key, id);
    return id;
}

constexpr uint32_t kMissing = 0xFFFFFFFFu;

void rollback_patterns(rs_ctx* c);

// Pattern id of every stripe into pid.  With `create` (pat_mu exclusive)
// missing patterns are added (and rolled back if the call fails); without
// (pat_mu shared) they are counted in *missing -- distinct patterns, so the
// eviction check is not inflated by stripes sharing one new pattern -- and
// their pid is kMissing.  A pattern not yet built (id >= uploaded) counts as
// missing too.  With `only_missing`, stripes whose pid is already set are
// skipped (the exclusive pass after a shared one).  More than m erasures in a
// stripe -> RS_ENOT_ENOUGH.
int lookup_patterns(rs_ctx* c, const uint8_t* erased, size_t stripes, std::vector<uint32_t>& pid,
                    bool create, size_t* missing, bool only_missing = false,
                    std::vector<PatKey>* miss_keys = nullptr) {
    if (!only_missing) pid.assign(stripes, kMissing);
    if (miss_keys) miss_keys->clear();
    size_t miss = 0;
    for (size_t i = 0; i < stripes; ++i) {
        if (only_missing && pid[i] != kMissing) continue;
        int e = 0;
        const PatKey key = rsmi::pattern_key(erased + i * c->n, c->n, &e);
        if (e > c->m) {
            if (create) rollback_patterns(c);
            return RS_ENOT_ENOUGH;
        }
        const int id = c->pat_index.find(key);
        if (id >= 0 && (create || static_cast<size_t>(id) < c->uploaded)) {
            pid[i] = static_cast<uint32_t>(id);
        } else if (create) {
            pid[i] = static_cast<uint32_t>(create_pattern(c, key, e));
        } else {
            pid[i] = kMissing;
            ++miss;
            if (miss_keys) miss_keys->push_back(key);
        }
    }
    if (missing) {
        if (miss_keys && !miss_keys->empty()) {
            std::vector<PatKey>& mk = *miss_keys;
            auto lt = [](const PatKey& a, const PatKey& b) {
                return std::lexicographical_compare(a.w, a.w + 4, b.w, b.w + 4);
            };
            std::sort(mk.begin(), mk.end(), lt);
            miss = static_cast<size_t>(std::unique(mk.begin(), mk.end()) - mk.begin());
        }
        *missing = miss;
    }
    return RS_OK;
}

// Orders the build stream after the last launch of every lease (pat_mu
// exclusive): every launch that reads the pattern tables recorded its lease's
// event while holding pat_mu, so this covers all of them -- on the device,
// without a host sync.
void order_after_readers(rs_ctx* c) {
    std::lock_guard<std::mutex> lk(c->lease_mu);
    for (const std::unique_ptr<Lease>& L : c->leases) L->begin(c->build_stream);
}

// Drops every cached pattern (pat_mu exclusive) without a host sync: the
// build stream waits for every reader before it overwrites rows.
void evict_patterns(rs_ctx* c) {
    order_after_readers(c);
    c->pat_index.clear();
    c->h_key.clear();
    c->h_cnt.clear();
    c->h_lo.clear();
    c->h_mask.clear();
    c->uploaded = 0;
    ++c->evictions;
    ++c->tables_gen;
}

// Undoes the patterns created since the last successful build (pat_mu
// exclusive): after a failed lookup or build they must not stay in the index,
// or a later call would find them and launch on rows never written.
void rollback_patterns(rs_ctx* c) {
    if (c->h_cnt.size() == c->uploaded) return;
    c->pat_index.drop_from(static_cast<int>(c->uploaded));
    c->h_cnt.resize(c->uploaded);
    c->h_lo.resize(c->uploaded);
    c->h_mask.resize(c->uploaded);
    c->h_key.clear();
}

const uint8_t* dev_enc(const rs_ctx* c) { return static_cast<const uint8_t*>(c->d_gf.p); }
// 2 KiB of zeros: the address the bit-sliced reconstruct loads for absent
// inputs (one wave's window, so those loads hit in L2 instead of HBM).
const uint8_t* dev_zpage(const rs_ctx* c) {
    return static_cast<const uint8_t*>(c->d_gf.p) + round_up(static_cast<size_t>(c->n) * c->k + 768, 16);
}

// The stream s will read pattern rows: order it after every build so far.
void wait_patterns(rs_ctx* c, hipStream_t s) {
    if (c->pat_ev_valid) (void)hipStreamWaitEvent(s, c->pat_ev, 0);
}

// launch_reconstruct's wait (pat_mu held; L.begin(s) already queued): only
// when a pattern the launch reads -- ids up to max_pid -- was built after
// the lease's last wait, or the tables moved since.  Otherwise the rows are
// complete before the lease's previous launch, which s follows through
// L.begin.  With build_after_caller, pat_ev also covers the building
// caller's queued work; an unconditional wait would put every concurrent
// caller behind that backlog.
// Returns whether it waited; the caller commits the lease's watermark
// (seen_patterns) only after L.end(s), so a failed launch leaves no claim.
// Skipping the wait is sound only while three invariants hold (ADVICE r04;
// tests/test_gpu_concurrency.py test_watermark_reuse_while_tables_move):
//   1. launch_reconstruct holds pat_mu from this wait until L.end(s), so no
//      build, growth or eviction can slip between the check and the launch;
//   2. a lease's dev_pending is never cleared, so L.begin(s) always orders s
//      after the lease's previous launch (which followed the rows it read);
//   3. every move of the device tables (growth copy, eviction rebuild) bumps
//      tables_gen, so a moved table never passes the first test below.
bool wait_patterns_for(rs_ctx* c, Lease& L, size_t max_pid, hipStream_t s) {
    if (L.seen_tables == c->tables_gen && max_pid < L.seen_uploaded) return false;
    wait_patterns(c, s);
    return true;
}

void seen_patterns(const rs_ctx* c, Lease& L) {
    L.seen_tables = c->tables_gen;
    L.seen_uploaded = c->uploaded;
}

// Uploads the keys of the patterns created since the last flush and builds
// them on the GPU (one workgroup per pattern: survivor and erased-id rows
// from the key, then the decode rows), pat_mu exclusive.  Builds run on the
// context's build stream, in order (growth copies included), so a build can
// overlap the kernels already queued on the callers' streams; readers wait
// for pat_ev (wait_patterns).
int flush_patterns_impl(rs_ctx* c, hipStream_t caller, bool has_caller) {
    const size_t npat = c->h_cnt.size(), first = c->uploaded;
    if (npat == first) return RS_OK;
    if (npat > (size_t(1) << 24)) return RS_EINVAL;  // 24-bit ids in the stripe descriptors
    const hipStream_t s = c->build_stream;
    const size_t k = c->k, m = c->m, ds = dst_stride(c);
    const size_t cnt = npat - first, b_key = cnt * sizeof(PatKey);
    if (c->h_key.size() != cnt) return RS_EINVAL;  // internal invariant
    // Growth frees the outgrown tables on the build stream: order it after
    // every launch that may still read them first.
    if (c->d_pcoef.needs(npat * m * k) || c->d_psrc.needs(npat * k * 4) || c->d_pdst.needs(npat * ds * 4) ||
        c->d_pcnt.needs(npat * 4) || c->d_pstat.needs(npat * 4)) {
        order_after_readers(c);
        ++c->tables_gen;  // old rows are copied into the new tables on the build stream
    }
    if (!c->d_pcoef.reserve_keep(npat * m * k, first * m * k, s) ||
        !c->d_psrc.reserve_keep(npat * k * 4, first * k * 4, s) ||
        !c->d_pdst.reserve_keep(npat * ds * 4, first * ds * 4, s) ||
        !c->d_pcnt.reserve_keep(npat * 4, first * 4, s) ||
        !c->d_pstat.reserve_keep(npat * 4, first * 4, s) || !c->d_pkey.reserve_keep(b_key, 0, s))
        return RS_ENOMEM;
    if (!c->st_pat.acquire(b_key)) return RS_ENOMEM;
    std::memcpy(c->st_pat.p, c->h_key.data(), b_key);
    hipError_t e = hipMemcpyAsync(c->d_pkey.p, c->st_pat.p, b_key, hipMemcpyHostToDevice, s);
    c->st_pat.release_after(s);
    if (e != hipSuccess) return RS_EDEVICE;
    // The build runs after the work the calling stream already queued (its
    // previous reconstruct, an encode): the inversion's small, barrier-bound
    // workgroups then get the chip to themselves for ~0.3 ms instead of
    // taking wave slots from a bandwidth-bound kernel for its whole length
    // (config-5 fresh patterns: the overlapped kernel ran 0.9 ms longer).
    if (has_caller && c->build_after_caller &&
        (hipEventRecord(c->caller_ev, caller) != hipSuccess ||
         hipStreamWaitEvent(s, c->caller_ev, 0) != hipSuccess))
        return RS_EDEVICE;
    rsmi::InvertArgs ia{};
    ia.enc = dev_enc(c);
    ia.gf_exp = dev_enc(c) + static_cast<size_t>(c->n) * c->k;
    ia.gf_log = ia.gf_exp + 512;
    ia.keys = static_cast<const uint64_t*>(c->d_pkey.p);
    ia.src = static_cast<uint32_t*>(c->d_psrc.p);
    ia.dst = static_cast<uint32_t*>(c->d_pdst.p);
    ia.cnt = static_cast<uint32_t*>(c->d_pcnt.p);
    ia.dst_stride = static_cast<uint32_t>(ds);
    ia.coef = static_cast<uint8_t*>(c->d_pcoef.p);
    ia.first = static_cast<uint32_t>(first);
    ia.k = static_cast<uint32_t>(c->k);
    ia.m = static_cast<uint32_t>(c->m);
    ia.status = static_cast<uint32_t*>(c->d_pstat.p);
    {
        const char* g = std::getenv("RSMI_INVERT_GENERIC");
        ia.generic = g && std::atoi(g) != 0 ? 1u : 0u;
    }
    e = rsmi::launch_invert(ia, static_cast<uint32_t>(cnt), s);
    if (e != hipSuccess) return RS_EDEVICE;
    if (hipEventRecord(c->pat_ev, s) != hipSuccess) return RS_EDEVICE;
    c->pat_ev_valid = true;
    c->uploaded = npat;
    c->h_key.clear();
    return RS_OK;
}

// Test hook (RSMI_TEST_FAIL_FLUSH=N at rs_new): the context's N-th build
// attempt fails with RS_ENOMEM before touching the device, as an allocation
// would.
bool injected_flush_failure(rs_ctx* c) {
    return c->test_fail_flush > 0 && ++c->flush_attempts == c->test_fail_flush;
}

// Builds the pending patterns; on any failure they are rolled back, so the
// cache only ever holds patterns whose rows were built (a retry recreates
// them).
int flush_patterns(rs_ctx* c, hipStream_t caller = nullptr, bool has_caller = false) {
    const int st = c->h_cnt.size() != c->uploaded && injected_flush_failure(c) ? RS_ENOMEM
                                                                             : flush_patterns_impl(c, caller, has_caller);
    if (st != RS_OK) rollback_patterns(c);
    return st;
}

void set_cache_patterns(const rs_ctx* c, rsmi::MatArgs& a) {
    a.coef = static_cast<const uint8_t*>(c->d_pcoef.p);
    a.src = static_cast<const uint32_t*>(c->d_psrc.p);
    a.dst = static_cast<const uint32_t*>(c->d_pdst.p);
    a.dst_stride = static_cast<uint32_t>(dst_stride(c));
}

// Launches the reconstruct of `stripes` whose patterns are in L.pid (pat_mu
// held, shared or exclusive, and every pattern built): stripe descriptors
// through L's staging and device buffer, then one launch per kernel.
int launch_reconstruct(rs_ctx* c, Lease& L, void* data, size_t dss, void* parity, size_t pss, size_t pitch,
                       size_t len, size_t stripes, const uint64_t* shard_ptrs, hipStream_t s) {
    const std::vector<uint32_t>& pid = L.pid;
    int max_e = 0;
    for (size_t i = 0; i < stripes; ++i) max_e = std::max<int>(max_e, static_cast<int>(c->h_cnt[pid[i]]));
    if (max_e == 0) return RS_OK;  // nothing erased anywhere
    // Kernel of each stripe.  0: the split-table kernel.  With a bit-sliced
    // reconstruct: stripes with at least split_e erasures go to the syndrome
    // kernel (the split table's cost grows with e while the syndrome network
    // costs a whole encode; profiles/r01e_ab_minrec.log: it wins from e = 1),
    // 1..T to the smallest row-subset variant covering every parity row the
    // pattern uses (bitslice.hpp rec_tops: fewer accumulators, more waves per
    // SIMD), T + 1 to the full kernel.
    // A small call (at most c->small_split erased stripes; 0: never) goes to
    // the split-table kernel whole: its blocks load 8 survivors at a time
    // where the syndrome kernel walks 4 ahead through k + m input slots, so
    // one RS(64,16) 64 KiB stripe reconstructs in 0.0375 ms instead of 0.048
    // (profiles/r05c/, r05d/lat_*.json); past ~16 stripes its VALU cost loses.
    size_t erased_stripes = 0;
    if (use_bitslice_rec(c) && c->small_split > 0)
        for (size_t i = 0; i < stripes && erased_stripes <= c->small_split; ++i) erased_stripes += c->h_cnt[pid[i]] != 0;
    const bool small_split = use_bitslice_rec(c) && c->small_split > 0 && erased_stripes <= c->small_split;
    const int split_e = use_bitslice_rec(c) && !small_split ? c->bitslice_rec_min_e : (c->m + 1);
    const int T = use_bitslice_rec(c) && !small_split ? c->n_tops : 0;
    const size_t nk = static_cast<size_t>(T) + 2;
    auto kernel_of = [&](uint32_t p) -> size_t {
        if (static_cast<int>(c->h_cnt[p]) < split_e) return 0;
        const int lo = c->h_lo[p];
        for (int v = 0; v < T; ++v)
            if (c->m - c->bitslice->rec_tops[v] <= lo) return static_cast<size_t>(v) + 1;
        return static_cast<size_t>(T) + 1;
    };
    // Sort of the stripes by (kernel, pattern): each launch lists its
    // stripes grouped by pattern (see rs_kernels.hpp stripe_desc).  The
    // RSMI_NO_SORT knob keeps address order within a kernel (A/B runs).
    static const bool no_sort = std::getenv("RSMI_NO_SORT") != nullptr;
    const size_t npat = no_sort ? 1 : c->h_cnt.size();
    const size_t nb = nk * npat;
    auto bucket = [&](size_t i) -> size_t { return kernel_of(pid[i]) * npat + (no_sort ? 0 : pid[i]); };
    size_t count[8] = {};  // stripes per kernel (nk <= 6)
    int max_lo = 0;
    size_t used = 0, max_pid = 0;
    for (size_t i = 0; i < stripes; ++i) {
        const uint32_t p = pid[i];
        if (!c->h_cnt[p]) continue;  // stripes with nothing erased are skipped
        ++used;
        max_pid = std::max<size_t>(max_pid, p);
        const size_t kk = kernel_of(p);
        ++count[kk];
        if (kk == 0) max_lo = std::max<int>(max_lo, static_cast<int>(c->h_cnt[p]));
    }
    // Descriptors, then (for the syndrome kernels) each descriptor's mask
    // record, in one upload -- or, for a small call, in the kernel arguments
    // (no descriptor copy queued ahead of the kernel).
    constexpr size_t kInline = rsmi::MatArgs::kInlineDesc;
    static_assert(kInline == rsmi::BitsliceRecArgs::kInlineDesc, "inline descriptor counts differ");
    const bool inl = used <= kInline && c->inline_desc;
    const bool masks = used > count[0];
    const size_t mask_off = round_up(used * sizeof(uint2), 16);
    const size_t desc_bytes = masks ? mask_off + used * sizeof(rsmi::BsStripeMask) : used * sizeof(uint2);
    uint2 ldesc[kInline];
    rsmi::BsStripeMask lmask[kInline];
    if (!inl && !L.st_stripe.acquire(desc_bytes)) return RS_ENOMEM;
    uint2* desc = inl ? ldesc : static_cast<uint2*>(L.st_stripe.p);
    rsmi::BsStripeMask* mrec =
        inl ? lmask : reinterpret_cast<rsmi::BsStripeMask*>(static_cast<uint8_t*>(L.st_stripe.p) + mask_off);
    auto put = [&](size_t slot, size_t i) {
        const uint32_t p = pid[i];
        desc[slot] = make_uint2(static_cast<uint32_t>(i), (p << 8) | c->h_cnt[p]);
        if (masks) mrec[slot] = c->h_mask[p];
    };
    if (nb <= 4 * stripes + 4096) {
        std::vector<uint32_t>& start = L.start;
        start.assign(nb + 1, 0);
        for (size_t i = 0; i < stripes; ++i)
            if (c->h_cnt[pid[i]]) ++start[bucket(i) + 1];
        for (size_t b = 0; b < nb; ++b) start[b + 1] += start[b];
        for (size_t i = 0; i < stripes; ++i)
            if (c->h_cnt[pid[i]]) put(start[bucket(i)]++, i);
    } else {
        // Many more patterns than stripes (fresh-pattern workloads): an LSD
        // radix sort of (bucket, stripe) pairs, 8 bucket bits per pass, instead
        // of a histogram over every cached pattern.  Stable, like the
        // counting sort: stripes of one bucket stay in address order.
        std::vector<uint64_t>& keys = L.sort_a;
        std::vector<uint64_t>& tmp = L.sort_b;
        keys.clear();
        for (size_t i = 0; i < stripes; ++i)
            if (c->h_cnt[pid[i]]) keys.push_back(static_cast<uint64_t>(bucket(i)) << 32 | i);
        tmp.resize(keys.size());
        const int bits = 64 - __builtin_clzll(static_cast<unsigned long long>(nb));
        for (int shift = 32; shift < 32 + bits; shift += 8) {
            size_t hist[257] = {};
            for (uint64_t v : keys) ++hist[((v >> shift) & 255u) + 1];
            for (int d = 0; d < 256; ++d) hist[d + 1] += hist[d];
            for (uint64_t v : keys) tmp[hist[(v >> shift) & 255u]++] = v;
            keys.swap(tmp);
        }
        for (size_t j = 0; j < keys.size(); ++j) put(j, static_cast<size_t>(keys[j] & 0xFFFFFFFFu));
    }
    L.begin(s);  // the descriptor buffer's previous readers
    const bool waited = wait_patterns_for(c, L, max_pid, s);
    hipError_t e = hipSuccess;
    if (!inl) {
        if (!L.d_stripe_pat.reserve_on(desc_bytes, s)) return RS_ENOMEM;
        e = hipMemcpyAsync(L.d_stripe_pat.p, desc, desc_bytes, hipMemcpyHostToDevice, s);
        L.st_stripe.release_after(s);
        if (e != hipSuccess) return RS_EDEVICE;
    }
    const uint2* d_desc = inl ? nullptr : static_cast<const uint2*>(L.d_stripe_pat.p);
    if (count[0] > 0) {
        rsmi::MatArgs a = base_args(c, data, dss, parity, pss, pitch, len, count[0]);
        set_cache_patterns(c, a);
        a.stripe_desc = d_desc;
        if (inl) {
            a.n_inline = static_cast<uint32_t>(count[0]);
            std::copy(ldesc, ldesc + count[0], a.inl_desc);
        }
        a.shard_ptrs = shard_ptrs;
        e = rsmi::launch_matmul(a, max_lo, s);
    }
    size_t first = count[0];
    for (size_t kk = 1; kk < nk && e == hipSuccess; first += count[kk], ++kk) {
        if (!count[kk]) continue;
        // Generated bit-sliced reconstruct (syndromes through the fixed
        // encode network, bitslice.hpp): same descriptors and pattern cache.
        rsmi::MatArgs a = base_args(c, data, dss, parity, pss, pitch, len, count[kk]);
        set_cache_patterns(c, a);
        rsmi::BitsliceRecArgs b{};
        b.data = a.data;
        b.parity = a.parity;
        b.data_ss = a.data_ss;
        b.parity_ss = a.parity_ss;
        b.pitch = a.pitch;
        b.count = a.stripes;
        if (inl) {
            std::copy(ldesc + first, ldesc + first + count[kk], b.inl_desc);
            std::copy(lmask + first, lmask + first + count[kk], b.inl_mask);
        } else {
            b.stripe_desc = d_desc + first;
            b.stripe_mask = reinterpret_cast<const rsmi::BsStripeMask*>(
                                static_cast<const uint8_t*>(L.d_stripe_pat.p) + mask_off) + first;
        }
        b.coef = a.coef;
        b.src = a.src;
        b.dst = a.dst;
        b.dst_stride = a.dst_stride;
        b.ncols16 = a.ncols16;
        // 256 lanes x 2 columns per window, rec_iters windows per block
        const uint32_t windows = (a.ncols16 + 511u) / 512u, it = static_cast<uint32_t>(c->bitslice->rec_iters);
        b.blocks_per_stripe = (windows + it - 1u) / it;
        b.zpage = dev_zpage(c);
        b.shard_ptrs = shard_ptrs;
        b.xcd = c->xcd;
        e = kk <= static_cast<size_t>(T) ? c->bitslice->rec_top_launch[kk - 1](b, s) : c->bitslice->reconstruct(b, s);
    }
    L.end(s);  // under pat_mu: an eviction waits for these launches
    if (e == hipSuccess) {
        c->rec_stripes_table += static_cast<int64_t>(count[0]);
        c->rec_stripes_syndrome += static_cast<int64_t>(used - count[0]);
    }
    if (waited && e == hipSuccess) seen_patterns(c, L);
    return hip_status(e);
}

// Batched reconstruct on stream s with lease L: lookups and launches under
// a shared lock; only a call that meets new patterns takes it exclusively
// (to create, build and, past the cap, evict).
int reconstruct(rs_ctx* c, Lease& L, void* data, size_t dss, void* parity, size_t pss, size_t pitch,
                size_t len, size_t stripes, const uint8_t* erased, const uint64_t* shard_ptrs, hipStream_t s) {
    size_t missing = 0;
    uint64_t gen = 0;
    {
        std::shared_lock<std::shared_mutex> rl(c->pat_mu);
        const int rc = lookup_patterns(c, erased, stripes, L.pid, false, &missing, false, &L.miss_keys);
        if (rc != RS_OK) return rc;
        if (missing == 0) return launch_reconstruct(c, L, data, dss, parity, pss, pitch, len, stripes, shard_ptrs, s);
        gen = c->evictions;
    }
    std::unique_lock<std::shared_mutex> wl(c->pat_mu);
    // Only the stripes the shared pass missed are looked up again, unless
    // the cache was evicted meanwhile (ids found then are stale).  `missing`
    // counts distinct new patterns (an upper bound: another caller may have
    // created some of them since).
    bool stale = c->evictions != gen;
    if (c->pat_index.size() + missing > c->pat_cap) {
        evict_patterns(c);
        stale = true;
    }
    const int rc = lookup_patterns(c, erased, stripes, L.pid, true, nullptr, !stale);
    if (rc != RS_OK) return rc;
    const int st = flush_patterns(c, s, true);
    if (st != RS_OK) return st;
    return launch_reconstruct(c, L, data, dss, parity, pss, pitch, len, stripes, shard_ptrs, s);
}

// Pointer-mode reconstruct from a HOST table of shard addresses
// [stripes][n] (rs_reconstruct_spread: one member's stripes): the table goes
// through the lease's pinned staging into its device buffer on stream s,
// then the reconstruct reads it like rs_reconstruct_ptrs' device table.
int reconstruct_host_table(rs_ctx* c, const uint64_t* tab, size_t len, size_t stripes, const uint8_t* erased,
                           hipStream_t s) {
    const size_t bytes = stripes * static_cast<size_t>(c->n) * sizeof(uint64_t);
    for (size_t i = 0; i < stripes * static_cast<size_t>(c->n); ++i)
        if (tab[i] & 15u) return RS_EINVAL;  // the kernels move 16-byte vectors
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    Lease& L = *lg.L;
    L.begin(s);  // the lease's table buffer may last have been read on another stream
    if (!L.st_pieces.acquire(bytes) || !L.d_pieces.reserve_on(bytes, s)) return RS_ENOMEM;
    std::memcpy(L.st_pieces.p, tab, bytes);
    const hipError_t e = hipMemcpyAsync(L.d_pieces.p, L.st_pieces.p, bytes, hipMemcpyHostToDevice, s);
    L.st_pieces.release_after(s);
    if (e != hipSuccess) {
        L.end(s);
        return RS_EDEVICE;
    }
    const int rc = reconstruct(c, L, nullptr, 0, nullptr, 0, round_up(len, 16), len, stripes, erased,
                               static_cast<const uint64_t*>(L.d_pieces.p), s);
    L.end(s);  // also when nothing was launched: the table copy wrote d_pieces on s
    return rc;
}

// Holds the least busy member of a device set for one call.
struct SetPick {
    rsmi::DeviceSet* s;
    int i;
    explicit SetPick(rsmi::DeviceSet* set) : s(set), i(rsmi::set_acquire(set)) {}
    ~SetPick() { rsmi::set_release(s, i); }
    rs_ctx* member() const { return rsmi::set_member(s, i); }
};

// Member of a device set on the device holding p (nullptr: none).
rs_ctx* routed(rs_ctx* c, const void* p) {
    const int i = rsmi::set_route(c->set, p);
    return i < 0 ? nullptr : rsmi::set_member(c->set, i);
}

// Member i of c (c itself for a single-device context, i == 0).
rs_ctx* member_of(rs_ctx* c, int i) {
    if (c->set) return rsmi::set_member(c->set, i);
    return i == 0 ? c : nullptr;
}

int members_of(const rs_ctx* c) { return c->set ? rsmi::set_count(c->set) : 1; }

// Runs job(i) for every member of c: concurrently for a set, inline for a
// single-device context.
int run_members(rs_ctx* c, const std::function<int(int)>& job) {
    return c->set ? rsmi::set_run(c->set, job) : job(0);
}

// out_t = decode row (surv -> targets[t]) applied to the survivors, on the
// GPU through L's pinned host pipeline.  Runs on c->device.
int gpu_rows(rs_ctx* c, Lease& L, const std::vector<int>& surv, const std::vector<const uint8_t*>& surv_ptr,
             const std::vector<int>& targets, const std::vector<uint8_t*>& outs, size_t S,
             const std::function<void()>& while_gpu = nullptr) {
    const int k = c->k, e = static_cast<int>(targets.size());
    if (e == 0 || S == 0) {
        if (while_gpu) while_gpu();
        return RS_OK;
    }
    std::vector<uint8_t> rows;
    if (!rsmi::decode_rows(c->enc, k, c->n, surv, targets, rows)) return RS_ESINGULAR;
    rsmi::HostPipeline* pipe = L.pipeline();
    if (!pipe) return RS_ENOMEM;
    // A launch codes at most m rows per group of the one-pattern table; more
    // targets (possible when correcting) go in several passes.
    for (int t0 = 0; t0 < e; t0 += c->m) {
        const int et = std::min(c->m, e - t0);
        std::vector<uint8_t> coef(static_cast<size_t>(c->m) * k, 0);
        std::copy(rows.begin() + static_cast<size_t>(t0) * k,
                  rows.begin() + static_cast<size_t>(t0 + et) * k, coef.begin());
        std::vector<uint32_t> src(k), dstid(c->m, 0), cnt(1, static_cast<uint32_t>(et));
        for (int i = 0; i < k; ++i) src[i] = static_cast<uint32_t>(i);
        for (int t = 0; t < et; ++t) dstid[t] = static_cast<uint32_t>(k + t);
        const size_t pbytes = PatLayout(c, 1).total;
        const void* pat = nullptr;
        if (pipe->direct()) {
            // The kernel reads the one-pattern table straight from pinned
            // host memory (its device alias), like the survivors: no upload
            // and no stream sync before the launch.  The previous pass's
            // launches were drained by pipe->run.
            if (!L.st_onepat.acquire(pbytes)) return RS_ENOMEM;
            pack_patterns(c, 1, coef.data(), src.data(), dstid.data(), cnt.data(),
                          static_cast<uint8_t*>(L.st_onepat.p));
            pat = L.st_onepat.dev;
        } else {
            std::vector<uint8_t> hp(pbytes);
            pack_patterns(c, 1, coef.data(), src.data(), dstid.data(), cnt.data(), hp.data());
            if (!L.d_onepat.reserve_on(hp.size(), L.stream)) return RS_ENOMEM;
            if (hipMemcpyAsync(L.d_onepat.p, hp.data(), hp.size(), hipMemcpyHostToDevice, L.stream) != hipSuccess ||
                hipStreamSynchronize(L.stream) != hipSuccess)
                return RS_EDEVICE;
            pat = L.d_onepat.p;
        }
        auto launch = [c, et, pat](uint8_t* din, uint8_t* dout, size_t pitch, size_t w, hipStream_t st) {
            rsmi::MatArgs a = base_args(c, din, 0, dout, 0, pitch, w, 1);
            set_patterns(c, 1, pat, a);
            a.stripe_desc = first_stripe_desc(c, pat);  // et outputs, not m
            return rsmi::launch_matmul(a, et, st);
        };
        const hipError_t err = pipe->run(surv_ptr.data(), k, outs.data() + t0, et, S, launch,
                                         t0 == 0 ? while_gpu : std::function<void()>());
        if (err != hipSuccess) return RS_EDEVICE;
    }
    return RS_OK;
}

// rs_encode straight from / to engine-pinned memory (pinned.hpp): the
// split-table kernel reads the data shards and writes the parity over PCIe
// in place through a one-stripe shard table -- no staging copies, no DMA.
// Returns false (nothing done) unless the code is served by the split-table
// kernel and every shard is 16-byte aligned inside a registered range.
bool encode_in_place(rs_ctx* c, Lease& L, const uint8_t* input, size_t S, uint8_t* parity, int* rc) {
    const size_t k = c->k, m = c->m, n = c->n;
    if (c->bitslice || (S & 15u) || (reinterpret_cast<uintptr_t>(input) & 15u) ||
        (reinterpret_cast<uintptr_t>(parity) & 15u) || std::getenv("RSMI_NO_DIRECT"))
        return false;
    const uint64_t din = rsmi::pinned_device_address(input, k * S);
    const uint64_t dout = rsmi::pinned_device_address(parity, m * S);
    if (!din || !dout) return false;
    const hipStream_t s = L.stream;
    L.begin(s);
    // The input is one stripe in the strided layout (shard j at din + j*S,
    // parity t at dout + t*S): no shard table to upload, one launch, and a
    // polled completion (rsmi::wait_event).
    (void)n;
    rsmi::MatArgs a = base_args(c, reinterpret_cast<void*>(din), 0, reinterpret_cast<void*>(dout), 0, S, S, 1);
    set_patterns(c, 1, c->d_encpat.p, a);
    a.stripe_desc = nullptr;
    hipError_t e = launch_encode(c, a, s);
    L.end(s);
    const hipError_t sy = e == hipSuccess ? rsmi::wait_event(L.dev_done) : hipSuccess;
    *rc = (e == hipSuccess && sy == hipSuccess) ? RS_OK : RS_EDEVICE;
    ++c->encodes_in_place;
    return true;
}

// Output ranges [start, end) of a decode call (one dst, or every dst of a
// batch) and whether a share's S bytes meet any of them.
class OutRanges {
public:
    void add(const uint8_t* p, size_t len) {
        if (len) r_.push_back({reinterpret_cast<uintptr_t>(p), reinterpret_cast<uintptr_t>(p) + len});
    }
    void seal() {  // sorted by start, with the running maximum of the ends
        std::sort(r_.begin(), r_.end());
        uintptr_t mx = 0;
        for (auto& v : r_) v.second = mx = std::max(mx, v.second);
    }
    bool meets(const uint8_t* p, size_t S) const {
        if (!S || r_.empty()) return false;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + S;
        // the ranges starting before b; the largest end among them
        auto it = std::lower_bound(r_.begin(), r_.end(), std::make_pair(b, uintptr_t(0)));
        return it != r_.begin() && std::prev(it)->second > a;
    }

private:
    std::vector<std::pair<uintptr_t, uintptr_t>> r_;
};

// infectious lets shares alias dst (Decode(dst, shares) with dst holding
// received bytes).  The engine writes dst while its kernels still read the
// survivors, and moves present shares within dst, so every share that meets
// an output range is first copied aside (into `aside`) and its pointer in
// by_id replaced (a copy-after-the-kernel rule alone missed
// survivors stored in missing rows or one row below their own).  Returns the
// number of shares set aside.
size_t set_aside_aliases(const OutRanges& out, std::vector<const uint8_t*>& by_id, size_t S,
                         std::vector<uint8_t>& aside) {
    size_t cnt = 0;
    for (const uint8_t* p : by_id) cnt += p && out.meets(p, S);
    if (!cnt) return 0;
    aside.resize(cnt * S);
    size_t j = 0;
    for (const uint8_t*& p : by_id)
        if (p && out.meets(p, S)) {
            std::memcpy(aside.data() + j * S, p, S);
            p = aside.data() + j++ * S;
        }
    return cnt;
}

// Whether each column chunk of a single message records its own event
// (default: chunk c's rows are copied out while chunk c + 1 codes);
// RSMI_CHUNK_EVENTS=0 records only the last chunk's and copies every chunk
// out after it (A/B: whether the marker between the two kernels costs the
// 5.4-us gap of profiles/r06h/).
bool chunk_events() {
    static const bool on = [] {
        const char* e = std::getenv("RSMI_CHUNK_EVENTS");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// The lease's main stream waits for the chunks launched on stream2 (their
// events), so L.end(stream) orders the lease's next user after all of them.
void join_chunks(Lease& L, int launched) {
    for (int ch = launched - 1; ch >= 0; --ch)
        if (L.chunk_stream(ch) != L.stream) {
            (void)hipStreamWaitEvent(L.stream, L.ev[ch], 0);
            break;  // the last chunk on stream2 follows the earlier ones there
        }
}

// Mailbox grid for one staged message (rs_kernels.hpp MailboxHost): one
// launch before the first chunk is staged, then each chunk is a job posted
// through pinned memory and its completion a word the host polls -- the
// per-chunk launch (4.3 us), dispatch (5 us), gap between the chunks'
// kernels (5.4 us) and completion event of profiles/r06h/ go, and the
// chunks' PCIe reads overlap (a block group per chunk): config-1 decode
// 56.7-63.5 -> 47.6-48.9 us, encode 57.5-58.9 -> 50.0-50.8 us on one box
// (profiles/r06o/).  Off with RSMI_MAILBOX=0; only for the split-table
// variants that have a mailbox twin (RS(10,4), RS(4,2)).
bool mailbox_on() {
    static const bool on = [] {
        const char* e = std::getenv("RSMI_MAILBOX");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
// Calls of fewer chunks launch their kernel the ordinary way
// (RSMI_MAILBOX_MIN_JOBS, default 2; 1 also gives the one-launch decode of
// engine-pinned survivors a grid).
int mailbox_min_jobs() {
    static const int n = [] {
        const char* e = std::getenv("RSMI_MAILBOX_MIN_JOBS");
        const int v = e ? std::atoi(e) : 2;
        return v >= 1 && v <= rsmi::kMailboxJobs ? v : 2;
    }();
    return n;
}

// How long the grid's block 0 waits for a post (RSMI_MAILBOX_TIMEOUT_US,
// default 20 ms; tests shorten it to make grids give up); a waiting caller
// gives the grid 2.5x that (at least 1 ms) before it drains the stream and
// launches the undone chunks itself.
long mailbox_timeout_us() {
    static const long us = [] {
        const char* e = std::getenv("RSMI_MAILBOX_TIMEOUT_US");
        const long v = e ? std::atol(e) : 20000;
        return v > 0 ? v : 20000;
    }();
    return us;
}

// RSMI_MAILBOX_STAMPS=1 (diagnostics): every grid records device wall-clock
// stamps (rs_kernels.hpp MailboxDev::stamp) and the caller its own post and
// done times; medians go to stderr at exit.  Costs a synchronous copy per call.
struct MailboxStamps {
    std::mutex mu;
    std::vector<std::vector<double>> cols;  // per metric
    std::vector<std::string> names;
    static MailboxStamps& get() {
        static MailboxStamps* s = [] {
            auto* p = new MailboxStamps;
            std::atexit([] { get().print(); });
            return p;
        }();
        return *s;
    }
    void add(const std::string& name, double us) {
        std::lock_guard<std::mutex> lk(mu);
        size_t i = 0;
        while (i < names.size() && names[i] != name) ++i;
        if (i == names.size()) {
            names.push_back(name);
            cols.emplace_back();
        }
        cols[i].push_back(us);
    }
    void print() {
        std::lock_guard<std::mutex> lk(mu);
        if (names.empty()) return;
        std::fprintf(stderr, "RSMI_MAILBOX_STAMPS %zu calls, median us (host: from the launch call's return; device: from block 0's entry):\n",
                     cols[0].size());
        for (size_t i = 0; i < names.size(); ++i) {
            std::vector<double> v = cols[i];
            std::sort(v.begin(), v.end());
            std::fprintf(stderr, "  %-28s %8.2f\n", names[i].c_str(), v[v.size() / 2]);
        }
    }
};
bool mailbox_stamps() {
    static const bool on = [] {
        const char* e = std::getenv("RSMI_MAILBOX_STAMPS");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

class MailboxCall {
public:
    // Launches the grid for the chunks' launch arguments `args` (up to
    // max_e outputs per stripe) on L.stream (after L.begin), or leaves ok()
    // false: the caller launches its chunks itself.  `use` false: off.
    MailboxCall(rs_ctx* c, Lease& L, bool use, const std::vector<rsmi::MatArgs>& args, int max_e)
        : c_(c), L_(L), njobs_(static_cast<int>(args.size())), max_e_(max_e) {
        if (!use || !mailbox_on() || njobs_ < mailbox_min_jobs() || njobs_ > rsmi::kMailboxJobs ||
            !rsmi::mailbox_supported(c->k, max_e))
            return;
        uint32_t blocks = 1;
        for (int j = 0; j < njobs_; ++j) {
            rsmi::plan_mailbox_job(args[static_cast<size_t>(j)], max_e, &jobs_.job[j]);
            blocks = std::max(blocks, jobs_.job[j].blocks);
        }
        if (!L.mb) {
            void* h = nullptr;
            if (hipHostMalloc(&h, sizeof(rsmi::MailboxHost), hipHostMallocCoherent) != hipSuccess) return;
            void* hd = nullptr;
            void* dd = nullptr;
            if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess || hipMalloc(&dd, sizeof(rsmi::MailboxDev)) != hipSuccess ||
                hipMemset(dd, 0, sizeof(rsmi::MailboxDev)) != hipSuccess) {
                (void)hipGetLastError();
                (void)hipHostFree(h);
                if (dd) (void)hipFree(dd);
                return;
            }
            int khz = 0;
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0)
                khz = 100000;
            std::memset(h, 0, sizeof(rsmi::MailboxHost));
            L.mb = static_cast<rsmi::MailboxHost*>(h);
            L.mb_dev = static_cast<rsmi::MailboxHost*>(hd);
            L.mbd = static_cast<rsmi::MailboxDev*>(dd);
            L.mb_timeout = static_cast<uint64_t>(khz) * mailbox_timeout_us() / 1000;
        }
        // The previous call's grid reads the board no more (its jobs were
        // all waited for, or it was drained): reset it for this one.
        rsmi::MailboxHost* h = L.mb;
        __atomic_store_n(&h->quit, uint64_t(0), __ATOMIC_RELAXED);
        __atomic_store_n(&h->gave_up, uint64_t(0), __ATOMIC_RELAXED);
        for (uint64_t& d : h->done) __atomic_store_n(&d, uint64_t(0), __ATOMIC_RELAXED);
        __atomic_store_n(&h->posted, uint64_t(0), __ATOMIC_RELEASE);
        const uint32_t per_job = std::min<uint32_t>(blocks, 64);
        if (rsmi::launch_mailbox(L.mb_dev, L.mbd, jobs_, njobs_, c->k, max_e, per_job, L.mb_timeout, L.stream,
                                 mailbox_stamps()) != hipSuccess) {
            (void)hipGetLastError();
            return;
        }
        if (mailbox_stamps()) {
            t_launch_ = std::chrono::steady_clock::now();
            khz_ = static_cast<double>(L.mb_timeout) / mailbox_timeout_us() * 1000.0;
        }
        ok_ = true;
        ++c->mailbox_calls;
    }
    ~MailboxCall() {
        if (!ok_) return;
        if (waited_ < njobs_) {  // an early return: the grid leaves once it sees quit, then the stream drains
            __atomic_store_n(&L_.mb->quit, uint64_t(1), __ATOMIC_RELEASE);
            (void)hipStreamSynchronize(L_.stream);
        } else if (mailbox_stamps() && !recovered_) {
            record_stamps();
        }
    }
    bool ok() const { return ok_; }
    // Job j (0-based) is staged: its group may start.
    void post(int j) {
        __atomic_store_n(&L_.mb->posted, static_cast<uint64_t>(j + 1), __ATOMIC_RELEASE);
        posted_ = j + 1;
        if (mailbox_stamps()) t_post_[j] = std::chrono::steady_clock::now();
    }
    // Waits for job j.  A group that gave up (mailbox_timeout_us: the host
    // was slow to post) says so in gave_up, and one that could not run at
    // all leaves its job undone: then -- at once, or after 2.5x the timeout
    // -- the caller asks the grid to leave, drains the stream and launches
    // what is still undone itself.
    hipError_t wait(int j) {
        const uint64_t want = static_cast<uint64_t>(j + 1);
        const uint64_t* done = &L_.mb->done[j];
        if (__atomic_load_n(done, __ATOMIC_ACQUIRE) != want) {
            const auto t0 = std::chrono::steady_clock::now();
            for (unsigned spin = 0;; ++spin) {
                if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == want) break;
                if ((spin & 255u) != 255u) {
                    __builtin_ia32_pause();
                    continue;
                }
                if (__atomic_load_n(&L_.mb->gave_up, __ATOMIC_ACQUIRE)) return recover(j);
                const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
                if (us > std::max(1000L, mailbox_timeout_us() * 5 / 2)) return recover(j);
                if (us > 200) std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
        }
        waited_ = std::max(waited_, j + 1);
        if (mailbox_stamps()) t_done_[j] = std::chrono::steady_clock::now();
        return hipSuccess;
    }

private:
    void record_stamps() {
        uint64_t st[1 + 3 * rsmi::kMailboxJobs] = {};
        if (hipStreamSynchronize(L_.stream) != hipSuccess ||
            hipMemcpy(st, L_.mbd->stamp, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess)
            return;
        MailboxStamps& ms = MailboxStamps::get();
        auto host_us = [&](std::chrono::steady_clock::time_point t) {
            return std::chrono::duration<double, std::micro>(t - t_launch_).count();
        };
        auto dev_us = [&](uint64_t a, uint64_t b) { return (static_cast<double>(b) - static_cast<double>(a)) * 1000.0 / khz_; };
        for (int j = 0; j < njobs_; ++j) {
            const std::string p = "job" + std::to_string(j) + " ";
            ms.add(p + "host post", host_us(t_post_[j]));
            ms.add(p + "host sees done", host_us(t_done_[j]));
            ms.add(p + "dev seen posted", dev_us(st[0], st[1 + 3 * j]));
            ms.add(p + "dev args loaded", dev_us(st[0], st[2 + 3 * j]));
            ms.add(p + "dev done stored", dev_us(st[0], st[3 + 3 * j]));
        }
    }
    std::chrono::steady_clock::time_point t_launch_, t_post_[rsmi::kMailboxJobs], t_done_[rsmi::kMailboxJobs];
    double khz_ = 100000.0;

    hipError_t recover(int j) {
        __atomic_store_n(&L_.mb->quit, uint64_t(1), __ATOMIC_RELEASE);
        hipError_t e = hipStreamSynchronize(L_.stream);  // the grid has left
        for (int i = 0; i < posted_ && e == hipSuccess; ++i)
            if (__atomic_load_n(&L_.mb->done[i], __ATOMIC_ACQUIRE) != static_cast<uint64_t>(i + 1)) {
                e = rsmi::launch_matmul(jobs_.job[i].a, max_e_, L_.stream);
                if (e == hipSuccess) __atomic_store_n(&L_.mb->done[i], static_cast<uint64_t>(i + 1), __ATOMIC_RELAXED);
            }
        if (e == hipSuccess) e = hipStreamSynchronize(L_.stream);
        if (!recovered_) ++c_->mailbox_recovered;
        recovered_ = true;
        waited_ = std::max(waited_, j + 1);
        if (j >= posted_) return hipErrorInvalidValue;
        return e;
    }

    rs_ctx* c_;
    Lease& L_;
    int njobs_;
    bool ok_ = false, recovered_ = false;
    int max_e_;
    rsmi::MailboxJobs jobs_{};
    int posted_ = 0, waited_ = 0;
};

// The one-launch decode of decode_in_place / decode_staged: survivor j of
// Rebuild's choice `surv` is read at device address dev[j] (column chunk by
// column chunk when nch > 1, the copies `stage` lists filling each chunk's
// survivor columns first); the present data shares are copied into dst
// (unless present_done) while the kernel runs (no share overlaps dst:
// rs_decode set aliasing ones aside).  Chunk 0 is staged on the calling
// thread; the later chunks' staging and the present shares are handed to the
// copy pool at once (async_copies), so a worker awake in its spin window does
// them while the caller stages chunk 0 and launches -- the caller joins each
// before it needs it (finish), doing whatever no worker has claimed.
// Returns kDecodeNoStaging, having done nothing, when its pinned staging
// cannot be had (the caller falls back to the pipeline).
using StageFn = std::function<std::vector<rsmi::CopyPool::Piece>(size_t off, size_t w)>;

// The present data shares into dst while a single message's kernels run,
// on the calling thread: with streaming stores when the survivors were
// staged (the GPU is reading the staging meanwhile), with memcpy when the
// kernel reads engine-pinned survivors in place.  Config-1 decode, caller on
// the GPU's node (profiles/r06t/): handing the copy to the pool (a wake-up,
// parts claimed under its lock) 46.0-46.1 us, memcpy 44.8-46.2, streaming
// stores 44.2-44.8; the arena decode 1.02-1.04x one core with the pool,
// 1.05-1.06x with memcpy, 0.94-0.95x with streaming stores.
// RSMI_PRESENT_COPY=pool|inline|nt forces one way for both (A/B).
void copy_present_shares(const std::vector<rsmi::CopyPool::Piece>& v, size_t part, bool staged) {
    static const int forced = [] {
        const char* e = std::getenv("RSMI_PRESENT_COPY");
        if (!e) return -1;
        const std::string m(e);
        return m == "pool" ? 0 : m == "inline" ? 1 : m == "nt" ? 2 : -1;
    }();
    const int mode = forced >= 0 ? forced : staged ? 2 : 1;
    if (mode == 0) {
        rsmi::CopyPool& pool = rsmi::CopyPool::shared();
        pool.finish(pool.start(v, part));
        return;
    }
    for (const rsmi::CopyPool::Piece& q : v) {
        if (mode == 2) rsmi::stage_copy(q.dst, q.src, q.len);
        else std::memcpy(q.dst, q.src, q.len);
    }
    if (mode == 2) rsmi::stage_fence();
}
constexpr int kDecodeNoStaging = -1000;
int decode_launch(rs_ctx* c, Lease& L, const std::vector<uint8_t>& present, const std::vector<const uint8_t*>& by_id,
                  const std::vector<int>& surv, const std::vector<uint64_t>& dev, size_t S, uint8_t* dst,
                  bool present_done, int nch = 1, const StageFn& stage = nullptr);


// Where a staged message's column chunks split, as cumulative percentages
// of each shard: RSMI_CHUNK_SPLIT ("30,65" by default: three chunks of 30,
// 35 and 35 % -- the first staged soon, so the GPU starts reading early,
// each later one read by its own block group while the host stages the
// next).  Config-1 decode / encode, caller on the GPU's NUMA node, jobs'
// arguments in the kernel arguments (profiles/r06w/, three processes
// each): "30,65" 42.1-42.8 / 44.5-45.6 us, "25,60" 42.9-43.8 / 44.9-46.2,
// "25,55,80" 42.6-44.0 / 45.4-46.6, "20,50,80" 43.7-44.1 / 45.1-46.9;
// earlier, with the arguments on the job board (profiles/r06r/): "33"
// 46.8-47.4 / 50.4-51.0, "15,50" 47.3 / 49.6-49.9; an even split of two
// chunks 48.9-49.7 / 55.0-57.3 (profiles/r06o/).  A split of n cuts applies
// to calls of n + 1 chunks (RSMI_STAGE_CHUNKS forces another count, split
// evenly).
const std::vector<size_t>& chunk_split() {
    static const std::vector<size_t> cuts = [] {
        std::vector<size_t> v;
        const char* e = std::getenv("RSMI_CHUNK_SPLIT");
        const std::string str = e ? e : "30,65";
        size_t prev = 0;
        for (size_t i = 0; i < str.size();) {
            const size_t j = std::min(str.find(',', i), str.size());
            const long pct = std::atol(str.substr(i, j - i).c_str());
            if (pct <= static_cast<long>(prev) || pct >= 100) return std::vector<size_t>{30, 65};
            v.push_back(static_cast<size_t>(pct));
            prev = static_cast<size_t>(pct);
            i = j + 1;
        }
        if (v.empty() || v.size() > 3) return std::vector<size_t>{30, 65};
        return v;
    }();
    return cuts;
}
// Column chunks of a staged small message: chunk c covers bytes
// [off(c), off(c + 1)) of every shard, offsets multiples of 16.  Several
// chunks let the host stage the later ones while the kernel codes the first
// (and copy the first ones' outputs out while it codes the last): messages
// of >= 256 KiB take chunk_split()'s count, RSMI_STAGE_CHUNKS overrides
// (1..4).
int stage_chunks(size_t bytes) {
    static const int forced = [] {
        const char* e = std::getenv("RSMI_STAGE_CHUNKS");
        return e ? std::max(1, std::min(std::atoi(e), 4)) : 0;
    }();
    if (forced) return forced;
    return bytes >= (size_t(256) << 10) ? static_cast<int>(chunk_split().size()) + 1 : 1;
}
size_t chunk_off(size_t S, int c, int nch) {
    if (c >= nch) return S;
    const std::vector<size_t>& cuts = chunk_split();
    if (c > 0 && static_cast<size_t>(nch) == cuts.size() + 1) return (S * cuts[c - 1] / 100) & ~size_t(15);
    return (S * c / nch) & ~size_t(15);
}

// rs_decode of exactly k distinct shares that all lie in engine-pinned
// memory (pinned.hpp: an rs_arena / rs_pinned_alloc range, 16-byte aligned,
// readable up to round_up(S, 16)): the split-table kernel reads the
// survivors over PCIe where they are, through a one-stripe shard table that
// sits with the one-pattern table in the lease's pinned staging (read in
// place too: nothing is uploaded).  The regenerated data shares go straight
// into dst when dst is engine-pinned as well, else through pinned staging;
// the present ones are copied into dst on the host while the kernel runs.
// Returns false (nothing done) when the shares are not all engine-pinned.
bool decode_in_place(rs_ctx* c, Lease& L, const std::vector<uint8_t>& present,
                     const std::vector<const uint8_t*>& by_id, size_t S, uint8_t* dst, int* rc) {
    const int k = c->k;
    if (S == 0 || std::getenv("RSMI_NO_DIRECT")) return false;
    const size_t span = round_up(S, 16);
    std::vector<int> surv = rsmi::choose_survivors(present.data(), k, c->n);
    std::vector<uint64_t> dev(k);
    for (int j = 0; j < k; ++j) {
        const uint8_t* p = by_id[surv[j]];
        if (reinterpret_cast<uintptr_t>(p) & 15u) return false;
        dev[j] = rsmi::pinned_device_address(p, span);
        if (!dev[j]) return false;
    }
    // RSMI_INPLACE_CHUNKS=1 (A/B): the column chunks of a staged message
    // here too -- with the mailbox grid, a group per chunk and each chunk's
    // rows copied out while the later ones are read.
    static const bool chunked = [] {
        const char* e = std::getenv("RSMI_INPLACE_CHUNKS");
        return e && std::atoi(e) != 0;
    }();
    const int r = decode_launch(c, L, present, by_id, surv, dev, S, dst, false,
                                chunked ? stage_chunks(static_cast<size_t>(k) * S) : 1);
    if (r == kDecodeNoStaging) return false;
    *rc = r;
    ++c->decodes_in_place;
    return true;
}

// A message whose k survivors fit the one-shot staging (kStageSmall, the copy
// pool's inline threshold, host_pipeline.cpp): the survivors are copied into
// pinned staging and the one-launch decode reads the staging in place; the
// present data shares go to dst while the kernel runs (copying them in the
// same pass as the staging, before the launch, measured slower: 0.080 vs
// 0.073 ms per config-1 message, profiles/r04j/).  Larger messages take the
// chunked pipeline (host_pipeline.cpp), whose copies overlap its chunks.
constexpr size_t kStageSmall = size_t(2) << 20;

bool decode_staged(rs_ctx* c, Lease& L, const std::vector<uint8_t>& present, const std::vector<const uint8_t*>& by_id,
                   size_t S, uint8_t* dst, int* rc) {
    const int k = c->k;
    const size_t span = round_up(S, 16);
    if (S == 0 || static_cast<size_t>(k) * span > kStageSmall || std::getenv("RSMI_NO_STAGE_SMALL")) return false;
    if (!L.st_in.acquire(static_cast<size_t>(k) * span)) return false;
    void* alias = L.st_in.dev;
    std::vector<int> surv = rsmi::choose_survivors(present.data(), k, c->n);
    std::vector<uint64_t> dev(k);
    uint8_t* st = static_cast<uint8_t*>(L.st_in.p);
    for (int j = 0; j < k; ++j) dev[j] = reinterpret_cast<uint64_t>(alias) + static_cast<uint64_t>(j) * span;
    // survivors' columns [off, off + w) into staging (non-temporal), chunk by chunk
    auto stage = [&](size_t off, size_t w) {
        std::vector<rsmi::CopyPool::Piece> v;
        for (int j = 0; j < k; ++j) v.push_back({st + static_cast<size_t>(j) * span + off, by_id[surv[j]] + off, w, true});
        return v;
    };
    const int r = decode_launch(c, L, present, by_id, surv, dev, S, dst, false,
                                stage_chunks(static_cast<size_t>(k) * S), stage);
    if (r == kDecodeNoStaging) return false;
    *rc = r;
    return true;
}

int decode_launch(rs_ctx* c, Lease& L, const std::vector<uint8_t>& present, const std::vector<const uint8_t*>& by_id,
                  const std::vector<int>& surv, const std::vector<uint64_t>& dev, size_t S, uint8_t* dst,
                  bool present_done, int nch, const StageFn& stage) {
    const int k = c->k;
    const size_t span = round_up(S, 16);
    std::vector<int> missing;
    for (int i = 0; i < k; ++i)
        if (!present[i]) missing.push_back(i);
    const int e = static_cast<int>(missing.size());
    auto present_pieces = [&] {
        std::vector<rsmi::CopyPool::Piece> v;
        if (!present_done)
            for (int i = 0; i < k; ++i)
                if (present[i] && dst + static_cast<size_t>(i) * S != by_id[i]) v.push_back({dst + static_cast<size_t>(i) * S, by_id[i], S});
        return v;
    };
    if (e == 0) {  // every data share present: copies only
        copy_present_shares(present_pieces(), S, false);
        return RS_OK;
    }
    // dst never overlaps a share here: rs_decode sets aliasing shares aside
    // (set_aside_aliases), so present shares go to dst while the kernel runs.
    std::vector<uint8_t> rows;
    if (!rsmi::decode_rows(c->enc, k, c->n, surv, missing, rows)) return RS_ESINGULAR;
    nch = std::max(1, std::min(nch, static_cast<int>(std::min<size_t>(kBatchChunks, S / 4096))));  // >= 4 KiB a chunk
    // Outputs: dst's rows in place when dst is engine-pinned (and the rows
    // 16-byte aligned), else rows of the lease's pinned output staging.
    const bool dst_direct = !(S & 15u) && !(reinterpret_cast<uintptr_t>(dst) & 15u) &&
                            rsmi::pinned_device_address(dst, static_cast<size_t>(k) * S) != 0;
    if (!dst_direct && !L.st_out.acquire(static_cast<size_t>(e) * span)) return kDecodeNoStaging;
    // Pinned staging: [one-pattern table][nch shard tables: k survivors, e outputs]
    const size_t pbytes = PatLayout(c, 1).total, toff = round_up(pbytes, 16);
    const size_t n8 = static_cast<size_t>(c->n) * 8;
    if (!L.st_onepat.acquire(toff + nch * n8)) return kDecodeNoStaging;
    uint8_t* host = static_cast<uint8_t*>(L.st_onepat.p);
    std::vector<uint8_t> coef(static_cast<size_t>(c->m) * k, 0);
    std::copy(rows.begin(), rows.end(), coef.begin());
    std::vector<uint32_t> src(k), dstid(c->m, 0), cnt(1, static_cast<uint32_t>(e));
    for (int i = 0; i < k; ++i) src[i] = static_cast<uint32_t>(i);
    for (int t = 0; t < e; ++t) dstid[t] = static_cast<uint32_t>(k + t);
    pack_patterns(c, 1, coef.data(), src.data(), dstid.data(), cnt.data(), host);
    rsmi::trace_mark("rows+pattern");
    void* halias = L.st_onepat.dev;
    uint64_t oalias = 0;
    if (!dst_direct) oalias = reinterpret_cast<uint64_t>(L.st_out.dev);
    const void* pat = halias;
    // Survivors at a common pitch (decode_staged's staging) with outputs in
    // the output staging: the strided layout, no shard table.  The kernel's
    // first reads -- the pattern's coefficients and the survivors -- then go
    // out together (no descriptor, survivor-id or shard-table read before
    // them, each a PCIe round trip).
    bool strided = !dst_direct;
    for (int jj = 1; jj < k && strided; ++jj) strided = dev[jj] == dev[0] + static_cast<uint64_t>(jj) * span;
    const hipStream_t s = L.stream;
    rsmi::CopyPool& pool = rsmi::CopyPool::shared();
    // Helper jobs, oldest first: chunks 1.. of the staging (needed first),
    // then the present shares.  Parts of ~128 KiB let a worker and the caller
    // share a job.
    constexpr size_t kAsyncPart = size_t(128) << 10;
    // Off by default (RSMI_ASYNC_COPIES=1: on): on the GPU box the helper's
    // copies slowed the caller's own staging 2.3x (stage0 6.95 -> 16.3 us:
    // the two threads share the host's copy bandwidth) and the config-1
    // decode went 56.8 -> 64-66 us (profiles/r06g/).
    static const bool async_copies = [] {
        const char* v = std::getenv("RSMI_ASYNC_COPIES");
        return v && std::atoi(v) != 0;
    }();
    std::vector<rsmi::CopyPool::Async*> staged(static_cast<size_t>(nch), nullptr);
    rsmi::CopyPool::Async* present_job = nullptr;
    if (async_copies) {
        if (stage)
            for (int ch = 1; ch < nch; ++ch) {
                const size_t off = chunk_off(S, ch, nch), w = chunk_off(S, ch + 1, nch) - off;
                staged[ch] = pool.start(stage(off, w), kAsyncPart);
            }
        present_job = pool.start(present_pieces(), kAsyncPart);
    }
    L.begin(s);
    if (nch > 1 && L.chunk_stream(1) != s) L.begin(L.chunk_stream(1));
    // Every chunk's launch arguments (and shard table) up front: a staged
    // message's chunks go to a mailbox grid launched now, whose dispatch
    // overlaps the staging of chunk 0 (MailboxCall).
    std::vector<rsmi::MatArgs> args(static_cast<size_t>(nch));
    for (int ch = 0; ch < nch; ++ch) {
        const size_t off = chunk_off(S, ch, nch), w = chunk_off(S, ch + 1, nch) - off;
        rsmi::MatArgs& a = args[static_cast<size_t>(ch)];
        a = strided ? base_args(c, reinterpret_cast<void*>(dev[0] + off), 0, reinterpret_cast<void*>(oalias + off), 0,
                                span, w, 1)
                    : base_args(c, nullptr, 0, nullptr, 0, span, w, 1);
        set_patterns(c, 1, pat, a);
        a.src = nullptr;                    // survivor j is id j, output t is id k + t
        a.desc0 = static_cast<uint32_t>(e);  // pattern 0, e outputs
        if (!strided) {
            uint64_t* tab = reinterpret_cast<uint64_t*>(host + toff + ch * n8);
            for (int jj = 0; jj < k; ++jj) tab[jj] = dev[jj] + off;
            for (int t = 0; t < e; ++t)
                tab[k + t] = dst_direct ? rsmi::pinned_device_address(dst + static_cast<size_t>(missing[t]) * S, span) + off
                                        : oalias + static_cast<uint64_t>(t) * span + off;
            a.shard_ptrs = reinterpret_cast<const uint64_t*>(static_cast<const uint8_t*>(halias) + toff + ch * n8);
        }
    }
    MailboxCall mb(c, L, !async_copies && L.chunk_stream(1) == s, args, e);
    // every chunk records its event unless RSMI_CHUNK_EVENTS=0 on one stream
    const bool ev_each = mb.ok() || chunk_events() || (nch > 1 && L.chunk_stream(1) != s);
    hipError_t err = hipSuccess;
    int launched = 0;
    for (int ch = 0; ch < nch && err == hipSuccess; ++ch) {
        const size_t off = chunk_off(S, ch, nch), w = chunk_off(S, ch + 1, nch) - off;
        const hipStream_t cs = L.chunk_stream(ch);
        if (stage) {
            if (ch > 0 && async_copies) {
                pool.finish(staged[ch]);
                staged[ch] = nullptr;
            } else {
                const std::vector<rsmi::CopyPool::Piece> v = stage(off, w);
                for (const rsmi::CopyPool::Piece& q : v) rsmi::stage_copy(q.dst, q.src, q.len);
                rsmi::stage_fence();
            }
        }
        rsmi::trace_mark(ch ? "stage1" : "stage0");
        if (mb.ok()) {
            mb.post(ch);
        } else {
            err = rsmi::launch_matmul(args[static_cast<size_t>(ch)], e, cs);
            if (err == hipSuccess && (ev_each || ch == nch - 1)) err = hipEventRecord(L.ev[ch], cs);
        }
        if (err == hipSuccess) ++launched;
        rsmi::trace_mark(ch ? "launch1" : "launch0");
    }
    join_chunks(L, launched);
    L.end(s);
    for (rsmi::CopyPool::Async* j : staged) pool.finish(j);  // a failed launch left some unjoined
    if (async_copies) pool.finish(present_job);  // while the kernel runs
    else copy_present_shares(present_pieces(), S, stage != nullptr);
    rsmi::trace_mark("copy_present");
    for (int ch = 0; ch < launched; ++ch) {
        if (!ev_each && ch < nch - 1) continue;  // no event of its own: copied out with the last chunk
        const hipError_t w8 = mb.ok() ? mb.wait(ch) : rsmi::wait_event(L.ev[ch]);
        rsmi::trace_mark(ch ? "wait1" : "wait0");
        if (err == hipSuccess) err = w8;
        if (err != hipSuccess || dst_direct) continue;
        const int c0 = ev_each ? ch : 0;  // chunks [c0, ch] copied out now
        const size_t off = chunk_off(S, c0, nch), w = chunk_off(S, ch + 1, nch) - off;
        for (int t = 0; t < e; ++t)
            std::memcpy(dst + static_cast<size_t>(missing[t]) * S + off,
                        static_cast<uint8_t*>(L.st_out.p) + t * span + off, w);
        rsmi::trace_mark(ch ? "copyout1" : "copyout0");
    }
    if (launched < nch) (void)rsmi::wait_event(L.dev_done);  // a failed launch: drain what was queued
    return err == hipSuccess ? RS_OK : RS_EDEVICE;
}

// rs_encode of a small message (k shards within kStageSmall) from pageable
// buffers: the input is copied once into pinned staging in the strided
// layout (pitch round_up(S, 16)), one encode launch reads it and writes the
// parity into pinned staging over PCIe, and the parity rows are copied out.
bool encode_staged(rs_ctx* c, Lease& L, const uint8_t* input, size_t S, uint8_t* parity, int* rc) {
    const size_t k = c->k, m = c->m, span = round_up(S, 16);
    if (S == 0 || k * span > kStageSmall || std::getenv("RSMI_NO_STAGE_SMALL")) return false;
    if (!L.st_in.acquire(k * span) || !L.st_out.acquire(m * span)) return false;
    void *din = L.st_in.dev, *dout = L.st_out.dev;
    uint8_t* st = static_cast<uint8_t*>(L.st_in.p);
    const uint8_t* out = static_cast<const uint8_t*>(L.st_out.p);
    const int nch = std::max(1, std::min(stage_chunks(k * S), static_cast<int>(std::min<size_t>(kBatchChunks, S / 4096))));
    const hipStream_t s = L.stream;
    // chunk ch's columns of every data shard into staging (non-temporal):
    // chunk 0 on the calling thread, the others handed to the copy pool at
    // once and joined before their launch (decode_launch's async_copies)
    auto pieces = [&](int ch) {
        const size_t off = chunk_off(S, ch, nch), w = chunk_off(S, ch + 1, nch) - off;
        std::vector<rsmi::CopyPool::Piece> v;
        for (size_t j = 0; j < k; ++j) v.push_back({st + j * span + off, input + j * S + off, w, true});
        return v;
    };
    static const bool async_copies = [] {  // off by default, see decode_launch
        const char* v = std::getenv("RSMI_ASYNC_COPIES");
        return v && std::atoi(v) != 0;
    }();
    rsmi::CopyPool& pool = rsmi::CopyPool::shared();
    std::vector<rsmi::CopyPool::Async*> staged(static_cast<size_t>(nch), nullptr);
    if (async_copies)
        for (int ch = 1; ch < nch; ++ch) staged[ch] = pool.start(pieces(ch), size_t(128) << 10);
    L.begin(s);
    if (nch > 1 && L.chunk_stream(1) != s) L.begin(L.chunk_stream(1));
    std::vector<rsmi::MatArgs> args(static_cast<size_t>(nch));
    for (int ch = 0; ch < nch; ++ch) {
        const size_t off = chunk_off(S, ch, nch), w = chunk_off(S, ch + 1, nch) - off;
        rsmi::MatArgs& a = args[static_cast<size_t>(ch)];
        a = base_args(c, static_cast<uint8_t*>(din) + off, 0, static_cast<uint8_t*>(dout) + off, 0, span, w, 1);
        set_patterns(c, 1, c->d_encpat.p, a);
        a.stripe_desc = nullptr;
    }
    MailboxCall mb(c, L, !c->bitslice && !async_copies && L.chunk_stream(1) == s, args, static_cast<int>(m));
    const bool ev_each = mb.ok() || chunk_events() || (nch > 1 && L.chunk_stream(1) != s);
    hipError_t e = hipSuccess;
    int launched = 0;
    for (int ch = 0; ch < nch && e == hipSuccess; ++ch) {
        const hipStream_t cs = L.chunk_stream(ch);
        if (staged[ch]) {
            pool.finish(staged[ch]);
            staged[ch] = nullptr;
        } else {
            for (const rsmi::CopyPool::Piece& q : pieces(ch)) rsmi::stage_copy(q.dst, q.src, q.len);
            rsmi::stage_fence();
        }
        rsmi::trace_mark(ch ? "stage1" : "stage0");
        if (mb.ok()) {
            mb.post(ch);
        } else {
            e = launch_encode(c, args[static_cast<size_t>(ch)], cs);
            if (e == hipSuccess && (ev_each || ch == nch - 1)) e = hipEventRecord(L.ev[ch], cs);
        }
        if (e == hipSuccess) ++launched;
        rsmi::trace_mark(ch ? "launch1" : "launch0");
    }
    join_chunks(L, launched);
    L.end(s);
    for (rsmi::CopyPool::Async* j : staged) pool.finish(j);  // a failed launch left some unjoined
    for (int ch = 0; ch < launched; ++ch) {
        if (!ev_each && ch < nch - 1) continue;  // copied out with the last chunk
        const hipError_t w8 = mb.ok() ? mb.wait(ch) : rsmi::wait_event(L.ev[ch]);
        rsmi::trace_mark(ch ? "wait1" : "wait0");
        if (e == hipSuccess) e = w8;
        if (e != hipSuccess) continue;
        const int c0 = ev_each ? ch : 0;
        const size_t off = chunk_off(S, c0, nch), w = chunk_off(S, ch + 1, nch) - off;
        for (size_t t = 0; t < m; ++t) std::memcpy(parity + t * S + off, out + t * span + off, w);
        rsmi::trace_mark(ch ? "copyout1" : "copyout0");
    }
    if (launched < nch) (void)rsmi::wait_event(L.dev_done);
    *rc = e == hipSuccess ? RS_OK : RS_EDEVICE;
    return true;
}

// Rebuild from the present shares: data shares copied, missing ones
// regenerated from Rebuild's survivors.
int rebuild_into(rs_ctx* c, Lease& L, const std::vector<uint8_t>& present,
                 const std::vector<const uint8_t*>& by_id, size_t S, uint8_t* dst) {
    const int k = c->k;
    int rc_small = RS_OK;
    if (decode_staged(c, L, present, by_id, S, dst, &rc_small)) return rc_small;
    std::vector<int> surv = rsmi::choose_survivors(present.data(), k, c->n);
    std::vector<const uint8_t*> sp(k);
    for (int i = 0; i < k; ++i) sp[i] = by_id[surv[i]];
    std::vector<int> missing;
    std::vector<uint8_t*> outs;
    for (int i = 0; i < k; ++i)
        if (!present[i]) {
            missing.push_back(i);
            outs.push_back(dst + static_cast<size_t>(i) * S);
        }
    // The present data shares go to dst on the copy pool while the GPU
    // regenerates the missing ones (gpu_rows' overlap hook).
    auto copy_present = [&] {
        std::vector<rsmi::CopyPool::Piece> pieces;
        for (int i = 0; i < k; ++i)
            if (present[i] && dst + static_cast<size_t>(i) * S != by_id[i])
                pieces.push_back({dst + static_cast<size_t>(i) * S, by_id[i], S});
        rsmi::CopyPool::shared().run(pieces);
    };
    // (dst overlaps no share: rs_decode set aliasing shares aside.)
    return gpu_rows(c, L, surv, sp, missing, outs, S, copy_present);
}

// Columns where any of `outs` differs from the received shares `recv`.
std::vector<size_t> mismatched_columns(const std::vector<std::vector<uint8_t>>& outs,
                                       const std::vector<const uint8_t*>& recv, size_t S) {
    std::vector<uint8_t> bad(S, 0);
    for (size_t t = 0; t < outs.size(); ++t) {
        const uint8_t* a = outs[t].data();
        const uint8_t* b = recv[t];
        for (size_t o = 0; o < S; o += 4096) {
            const size_t w = std::min<size_t>(4096, S - o);
            if (std::memcmp(a + o, b + o, w) == 0) continue;
            for (size_t j = o; j < o + w; ++j) bad[j] |= a[j] != b[j];
        }
    }
    std::vector<size_t> cols;
    for (size_t j = 0; j < S; ++j)
        if (bad[j]) cols.push_back(j);
    return cols;
}

// infectious Decode with more than k distinct shares: Correct (consistency
// check + Berlekamp-Welch on inconsistent columns) then Rebuild.  The bulk
// work is GPU decodes; Berlekamp-Welch runs on the host for one column to
// locate the bad shares, which are then treated as erasures, and again only
// for columns that stay inconsistent.  Unlike infectious, the caller's share
// bytes are not modified (the corrected values only land in dst).  The
// result equals the oracle's Berlekamp-Welch restatement (oracle/rs_oracle.c
// orc_bw_column); parity against upstream infectious is unpinned.
int correct_decode(rs_ctx* c, Lease& L, std::vector<uint8_t> present, const std::vector<const uint8_t*>& by_id,
                   size_t S, uint8_t* dst) {
    const int k = c->k, n = c->n;
    std::vector<int> P;
    for (int i = 0; i < n; ++i)
        if (present[i]) P.push_back(i);
    const int r = static_cast<int>(P.size());
    // 1. are the shares one codeword?  predict the extras from Rebuild's k
    std::vector<int> base = rsmi::choose_survivors(present.data(), k, n);
    std::vector<uint8_t> in_base(n, 0);
    for (int v : base) in_base[v] = 1;
    std::vector<int> extras;
    for (int i : P)
        if (!in_base[i]) extras.push_back(i);
    std::vector<const uint8_t*> bp(k);
    for (int i = 0; i < k; ++i) bp[i] = by_id[base[i]];
    std::vector<std::vector<uint8_t>> pred(extras.size(), std::vector<uint8_t>(S));
    std::vector<uint8_t*> po;
    std::vector<const uint8_t*> rx;
    for (size_t t = 0; t < extras.size(); ++t) {
        po.push_back(pred[t].data());
        rx.push_back(by_id[extras[t]]);
    }
    int st = gpu_rows(c, L, base, bp, extras, po, S);
    if (st != RS_OK) return st;
    std::vector<size_t> bad = mismatched_columns(pred, rx, S);
    if (bad.empty()) return rebuild_into(c, L, present, by_id, S, dst);
    if ((r - k) / 2 <= 0) return RS_ENOT_ENOUGH;  // berlekampWelch: e <= 0
    // 2. locate the bad shares on the first inconsistent column
    std::vector<uint8_t> ys(r), cw(n);
    auto column = [&](size_t j) {
        for (int i = 0; i < r; ++i) ys[i] = by_id[P[i]][j];
        return rsmi::bw_column(k, n, P.data(), ys.data(), r, cw.data());
    };
    if (column(bad[0]) < 0) return RS_ETOO_MANY_ERRORS;
    std::vector<uint8_t> present2 = present;
    for (int i = 0; i < r; ++i)
        if (cw[P[i]] != ys[i]) present2[P[i]] = 0;  // treat as erased
    // 3. rebuild from the rest; shares outside its survivors must agree
    std::vector<int> base2 = rsmi::choose_survivors(present2.data(), k, n);
    std::vector<uint8_t> in_b2(n, 0);
    for (int v : base2) in_b2[v] = 1;
    std::vector<int> targets, others;
    std::vector<uint8_t*> outs;
    for (int i = 0; i < k; ++i)
        if (!in_b2[i]) {
            targets.push_back(i);
            outs.push_back(dst + static_cast<size_t>(i) * S);
        }
    for (int i : P)
        if (present2[i] && !in_b2[i]) others.push_back(i);
    std::vector<std::vector<uint8_t>> chk(others.size(), std::vector<uint8_t>(S));
    std::vector<const uint8_t*> rx2;
    for (size_t t = 0; t < others.size(); ++t) {
        targets.push_back(others[t]);
        outs.push_back(chk[t].data());
        rx2.push_back(by_id[others[t]]);
    }
    std::vector<const uint8_t*> bp2(k);
    for (int i = 0; i < k; ++i) bp2[i] = by_id[base2[i]];
    st = gpu_rows(c, L, base2, bp2, targets, outs, S);
    if (st != RS_OK) return st;
    for (int i = 0; i < k; ++i)
        if (in_b2[i]) std::memcpy(dst + static_cast<size_t>(i) * S, by_id[i], S);
    // 4. columns still inconsistent: full Berlekamp-Welch each
    for (size_t j : mismatched_columns(chk, rx2, S)) {
        if (column(j) < 0) return RS_ETOO_MANY_ERRORS;
        for (int i = 0; i < k; ++i) dst[static_cast<size_t>(i) * S + j] = cw[i];
    }
    return RS_OK;
}

// Reads the status words of patterns [0, npat) after s has built them
// (pat_mu held): RS_ESINGULAR if any survivor matrix was singular.
int pattern_status(rs_ctx* c, size_t first, size_t count, hipStream_t s) {
    if (count == 0) return RS_OK;
    std::vector<uint32_t> st(count);
    wait_patterns(c, s);
    if (hipMemcpyAsync(st.data(), static_cast<uint32_t*>(c->d_pstat.p) + first, count * 4, hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return RS_EDEVICE;
    for (uint32_t v : st)
        if (v) return RS_ESINGULAR;
    return RS_OK;
}

// CPUs this process may use: the affinity mask, then the cgroup v2 quota
// (a GPU box gives a job a share of a large host), at least 1.
int usable_cpus() {
    static const int n = [] {
        int cpus = static_cast<int>(std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        if (FILE* fh = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {};
            long period = 0;
            if (std::fscanf(fh, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
                cpus = std::min<int>(cpus, std::max<long>(1, std::atol(q) / period));
            std::fclose(fh);
        }
        return std::max(1, cpus);
    }();
    return n;
}

// Host/GPU crossover of the hash policy (rs_blake2b).  BLAKE2b's blocks
// chain, so the GPU kernel's time is one launch plus the longest message's
// chain (~1.76 us per 128-byte block on 4 lanes) plus the staging copies and
// its VALU-bound aggregate rate, while the host runs a message per thread at
// the rate measured once on this machine (1.73 GB/s per thread on the GPU
// box's EPYC 9575F, profiles/r03c/hash_policy.json), each extra thread
// costing ~25 us to start.  Both estimates are minimised over the host
// thread count; the host wins ties.  RSMI_HASH=host / gpu forces a side;
// RSMI_HASH_HOST_GBPS overrides the calibrated per-thread rate.
struct HashPlan {
    bool host;
    int threads;
};

double host_hash_rate() {
    static const double bps = [] {
        if (const char* v = std::getenv("RSMI_HASH_HOST_GBPS")) return std::max(0.01, std::atof(v)) * 1e9;
        std::vector<uint8_t> buf(size_t(128) << 10, 0x5A);
        uint8_t d[32];
        double best = 1e9;
        for (int r = 0; r < 3; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            rsmi::blake2b_host(buf.data(), buf.size(), 32, d);
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        return static_cast<double>(buf.size()) / std::max(best, 1e-6);
    }();
    return bps;
}

HashPlan plan_hash(int count, const size_t* lens) {
    static const int forced = [] {
        const char* v = std::getenv("RSMI_HASH");
        if (!v) return 0;
        return std::strcmp(v, "host") == 0 ? 1 : std::strcmp(v, "gpu") == 0 ? 2 : 0;
    }();
    double total = 0, longest = 0;
    for (int i = 0; i < count; ++i) {
        total += static_cast<double>(lens[i]);
        longest = std::max(longest, static_cast<double>(lens[i]));
    }
    const double h = host_hash_rate();
    constexpr double kThreadCost = 25e-6;
    const int tmax = std::max(1, std::min(count, usable_cpus()));
    int best_t = 1;
    double host_s = 1e30;
    for (int t = 1; t <= tmax; ++t) {
        const double est = std::max(longest / h, total / (h * t)) + kThreadCost * (t - 1);
        if (est < host_s) {
            host_s = est;
            best_t = t;
        }
    }
    if (forced) return {forced == 1, best_t};
    const double chain_blocks = std::ceil(std::max(longest, 1.0) / 128.0);
    const double gpu_s = 80e-6 + chain_blocks * 1.76e-6 + total / 50e9 + total / 1.0e12;
    return {host_s <= gpu_s, best_t};
}

}  // namespace

extern "C" {

const char* rs_strerror(int st) {
    switch (st) {
        case RS_OK: return "ok";
        case RS_EINVAL_KN: return "requires 1 <= k <= n <= 256";
        case RS_ELEN_NOT_MULTIPLE: return "input length must be a multiple of k";
        case RS_ENOT_ENOUGH: return "not enough shares";
        case RS_EBAD_SHARE_ID: return "invalid share id";
        case RS_ESINGULAR: return "singular matrix";
        case RS_ENO_SHARES: return "must specify at least one share";
        case RS_ESHARE_LEN: return "shares have different lengths";
        case RS_EINVAL: return "invalid argument";
        case RS_EDEVICE: return "HIP device error";
        case RS_ENOMEM: return "out of memory";
        case RS_ETOO_MANY_ERRORS: return "too many errors to reconstruct";
        default: return "unknown error";
    }
}

int rs_new_on_device(int k, int n, int device, rs_ctx** out) {
    if (!out) return RS_EINVAL;
    *out = nullptr;
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return RS_EINVAL_KN;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
        return RS_EDEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RS_EDEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RS_EDEVICE;
    DeviceGuard g(device);
    if (!g.ok) return RS_EDEVICE;
    rs_ctx* c = new (std::nothrow) rs_ctx;
    if (!c) return RS_ENOMEM;
    c->k = k;
    c->n = n;
    c->m = n - k;
    c->device = device;
    c->enc = rsmi::systematic_matrix(k, n);
    c->bitslice = pick_bitslice(c->enc, k, c->m);
    c->bitslice_rec = pick_bitslice_rec(c->bitslice);
    if (c->bitslice_rec) {
        // Row-subset syndrome kernels: opt-in (RSMI_BITSLICE_TOPS=1).  Same-box
        // A/B, 20 steps x 3 reps (profiles/r03i/): the full kernel for every
        // stripe is faster or tied on every config-5 mix (e = 1..4: 12.0 vs
        // 12.4 ms; pool of 256: 15.2 vs 15.5 ms; 1..8 and 1..16: tied).
        const char* tv = std::getenv("RSMI_BITSLICE_TOPS");
        c->n_tops = (tv && std::atoi(tv) != 0) ? c->bitslice->n_rec_tops : 0;
    }
    {
        // RS(64,16): with the network restricted to the rows a pattern uses,
        // the syndrome kernel beats the split-table kernel from e = 1
        // (profiles/r01e_ab_minrec.log); a threshold > 1 sends stripes with
        // fewer erasures to the split-table kernel.
        const char* ev = std::getenv("RSMI_BITSLICE_REC_MIN_E");
        c->bitslice_rec_min_e = ev ? std::max(1, std::atoi(ev)) : 1;
        if (c->bitslice_rec)
            c->rec_name = c->bitslice_rec_min_e <= 1
                              ? std::string(c->bitslice->rec_name)
                              : std::string(rsmi::variant_name(k, std::min(c->m, c->bitslice_rec_min_e - 1))) + " (e<" +
                                    std::to_string(c->bitslice_rec_min_e) + ") + " + c->bitslice->rec_name;
        for (int v = 0; v < c->n_tops; ++v)
            c->rec_name += std::string(v ? "," : " +t") + std::to_string(c->bitslice->rec_tops[v]);
    }
    {
        // XCD-aware block order (xcd.hpp) for the bit-sliced encode and both
        // reconstruct kernels; the split-table encode keeps the natural order
        // (profiles/r02ak/: RS(64,16) encode -10% time, reconstructs -2..3%,
        // RS(10,4) split-table encode +2%).  RSMI_XCD=0 / 1: off / on for
        // every kernel (A/B runs).
        const char* xv = std::getenv("RSMI_XCD");
        c->xcd = (xv && std::atoi(xv) == 0) ? 0u : 1u;
        c->xcd_split_enc = (xv && std::atoi(xv) == 1) ? ~0u : 0u;
        const char* rv = std::getenv("RSMI_XCD_ENC_REGION");  // A/B knob: blocks per XCD region
        if (rv) c->xcd_split_enc = static_cast<uint32_t>(std::min(std::max(0, std::atoi(rv)), 1 << 20));
        c->xcd_split_rec = c->xcd ? ~0u : 0u;
        const char* qv = std::getenv("RSMI_XCD_REC_REGION");  // A/B knob: blocks per XCD region
        if (qv) c->xcd_split_rec = static_cast<uint32_t>(std::min(std::max(0, std::atoi(qv)), 1 << 20));
        const char* bv = std::getenv("RSMI_XCD_BS_STRIPES");  // A/B knob: stripes per region (bit-sliced)
        if (bv && c->xcd) c->xcd = static_cast<uint32_t>(std::min(std::max(1, std::atoi(bv)), 64));
    }
    // Small reconstructs pass their descriptors in the kernel arguments
    // (launch_reconstruct); RSMI_NO_INLINE_DESC=1 uploads them always (A/B, tests).
    c->inline_desc = std::getenv("RSMI_NO_INLINE_DESC") == nullptr;
    {
        const char* ss = std::getenv("RSMI_SMALL_SPLIT");  // 0: never (A/B, tests)
        if (ss) c->small_split = static_cast<size_t>(std::max(0, std::atoi(ss)));
    }
    {
        // Pattern-cache bound (RSMI_PATTERN_CAP, for tests): 2^20 patterns,
        // 1.3 GiB of tables for RS(64,16).
        const char* pc = std::getenv("RSMI_PATTERN_CAP");
        c->pat_cap = pc ? static_cast<size_t>(std::max(1, std::atoi(pc))) : (size_t(1) << 20);
        const char* ff = std::getenv("RSMI_TEST_FAIL_FLUSH");
        c->test_fail_flush = ff ? std::atoi(ff) : 0;
        const char* ml = std::getenv("RSMI_MAX_LEASES");
        c->max_leases = ml ? static_cast<size_t>(std::max(1, std::atoi(ml))) : 16;
    }
    if (hipEventCreateWithFlags(&c->pat_ev, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return RS_EDEVICE;
    }
    if (hipEventCreateWithFlags(&c->caller_ev, hipEventDisableTiming) != hipSuccess) {
        rs_free(c);
        return RS_EDEVICE;
    }
    {
        const char* bo = std::getenv("RSMI_BUILD_OVERLAP");
        c->build_after_caller = !(bo && std::atoi(bo) != 0);
    }
    if (hipStreamCreateWithFlags(&c->build_stream, hipStreamNonBlocking) != hipSuccess) {
        rs_free(c);
        return RS_EDEVICE;
    }
    // Encode pattern: coef = bottom rows, src = 0..k-1, dst = k..n-1, cnt = m.
    std::vector<uint32_t> src(k), dst(c->m), cnt(1, static_cast<uint32_t>(c->m));
    for (int i = 0; i < k; ++i) src[i] = static_cast<uint32_t>(i);
    for (int t = 0; t < c->m; ++t) dst[t] = static_cast<uint32_t>(k + t);
    std::vector<uint8_t> pat(PatLayout(c, 1).total);
    pack_patterns(c, 1, c->enc.data() + static_cast<size_t>(k) * k, src.data(), dst.data(),
                  cnt.data(), pat.data());
    {
        const rsmi::Field& F = rsmi::field();
        const size_t nk = static_cast<size_t>(n) * k;
        // then a 2 KiB zero page (dev_zpage)
        std::vector<uint8_t> gf(round_up(nk + 768, 16) + 2048, 0);
        std::copy(c->enc.begin(), c->enc.end(), gf.begin());
        std::memcpy(gf.data() + nk, F.exp, 510);
        std::memcpy(gf.data() + nk + 510, F.exp, 2);
        std::memcpy(gf.data() + nk + 512, F.log, 256);
        if (!c->d_gf.reserve(gf.size()) ||
            hipMemcpy(c->d_gf.p, gf.data(), gf.size(), hipMemcpyHostToDevice) != hipSuccess) {
            rs_free(c);
            return RS_EDEVICE;
        }
    }
    if (!c->d_encpat.reserve(pat.size()) ||
        hipMemcpy(c->d_encpat.p, pat.data(), pat.size(), hipMemcpyHostToDevice) != hipSuccess) {
        rs_free(c);
        return RS_EDEVICE;
    }
    *out = c;
    return RS_OK;
}

int rs_new(int k, int n, rs_ctx** out) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return rs_new_on_device(k, n, dev, out);
}

int rs_new_devices(int k, int n, const int* devices, int count, rs_ctx** out) {
    if (!out) return RS_EINVAL;
    *out = nullptr;
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return RS_EINVAL_KN;
    if (!devices || count <= 0 || count > 256) return RS_EINVAL;
    rs_ctx* c = new (std::nothrow) rs_ctx;
    if (!c) return RS_ENOMEM;
    c->k = k;
    c->n = n;
    c->m = n - k;
    c->device = devices[0];
    c->enc = rsmi::systematic_matrix(k, n);
    const int st = rsmi::set_create(k, n, devices, count, &c->set);
    if (st != RS_OK) {
        delete c;
        return st;
    }
    for (int i = 0; i < rsmi::set_count(c->set); ++i) rsmi::set_member(c->set, i)->set_member = true;
    *out = c;
    return RS_OK;
}

int rs_member_count(const rs_ctx* c) { return c ? members_of(c) : RS_EINVAL; }

}  // extern "C"

namespace rsmi {
// device_set.cpp: frees a member context (rs_free ignores members).
void member_free(rs_ctx* c) {
    if (!c) return;
    c->set_member = false;
    rs_free(c);
}
}  // namespace rsmi

extern "C" {

rs_ctx* rs_member(rs_ctx* c, int i) { return c ? member_of(c, i) : nullptr; }

int rs_partition(size_t units, int parts, int part, size_t* first, size_t* count) {
    if (parts <= 0 || part < 0 || part >= parts || !first || !count) return RS_EINVAL;
    // units * part / parts without overflow for any size_t units
    auto at = [&](size_t p) {
        const size_t q = units / static_cast<size_t>(parts), r = units % static_cast<size_t>(parts);
        return q * p + r * p / static_cast<size_t>(parts);
    };
    *first = at(static_cast<size_t>(part));
    *count = at(static_cast<size_t>(part) + 1) - *first;
    return RS_OK;
}

void rs_free(rs_ctx* c) {
    if (!c || c->set_member) return;  // a set's member (rs_member) is freed with its set
    if (c->set) {
        rsmi::set_destroy(c->set);
        delete c;
        return;
    }
    {
        DeviceGuard g(c->device);
        (void)hipDeviceSynchronize();
        c->leases.clear();  // each lease syncs and frees its streams, staging and buffers
        c->free_leases.clear();
        c->st_pat.destroy();
        for (DevBuf* b : {&c->d_encpat, &c->d_gf}) b->release();
        for (GrowBuf* b : {&c->d_pcoef, &c->d_psrc, &c->d_pdst, &c->d_pcnt, &c->d_pstat, &c->d_pkey}) b->release();
        if (c->pat_ev) (void)hipEventDestroy(c->pat_ev);
        if (c->caller_ev) (void)hipEventDestroy(c->caller_ev);
        if (c->build_stream) (void)hipStreamDestroy(c->build_stream);
    }
    delete c;
}

int rs_k(const rs_ctx* c) { return c ? c->k : RS_EINVAL; }
int rs_n(const rs_ctx* c) { return c ? c->n : RS_EINVAL; }
int rs_device(const rs_ctx* c) { return c ? c->device : RS_EINVAL; }

int rs_encode_matrix(const rs_ctx* c, uint8_t* out) {
    if (!c || !out) return RS_EINVAL;
    std::memcpy(out, c->enc.data(), c->enc.size());
    return RS_OK;
}

const char* rs_kernel_name(const rs_ctx* c, int which) {
    if (!c) return "";
    if (c->set) return rs_kernel_name(rsmi::set_member(c->set, 0), which);
    if (which == 0 && c->bitslice) return c->bitslice->name;
    if (which == 1 && use_bitslice_rec(c)) return c->rec_name.c_str();
    return rsmi::variant_name(c->k, c->m);
}

int rs_pattern_count(const rs_ctx* c) {
    if (!c) return RS_EINVAL;
    if (c->set) {
        int sum = 0;
        for (int i = 0; i < rsmi::set_count(c->set); ++i) sum += rs_pattern_count(rsmi::set_member(c->set, i));
        return sum;
    }
    std::shared_lock<std::shared_mutex> rl(c->pat_mu);
    return static_cast<int>(c->pat_index.size());
}

int64_t rs_pattern_evictions(const rs_ctx* c) {
    if (!c) return RS_EINVAL;
    if (c->set) {
        int64_t sum = 0;
        for (int i = 0; i < rsmi::set_count(c->set); ++i) sum += rs_pattern_evictions(rsmi::set_member(c->set, i));
        return sum;
    }
    std::shared_lock<std::shared_mutex> rl(c->pat_mu);
    return static_cast<int64_t>(c->evictions);
}

int64_t rs_stat(const rs_ctx* c, int which) {
    if (!c) return RS_EINVAL;
    if (c->set) {
        int64_t sum = 0;
        for (int i = 0; i < rsmi::set_count(c->set); ++i) {
            const int64_t v = rs_stat(rsmi::set_member(c->set, i), which);
            if (v < 0) return v;
            sum += v;
        }
        return sum;
    }
    switch (which) {
        case RS_STAT_PATTERNS: return rs_pattern_count(c);
        case RS_STAT_EVICTIONS: return rs_pattern_evictions(c);
        case RS_STAT_BATCHES_IN_PLACE: return c->batches_in_place.load();
        case RS_STAT_BATCHES_STAGED: return c->batches_staged.load();
        case RS_STAT_ENCODES_IN_PLACE: return c->encodes_in_place.load();
        case RS_STAT_DECODES_IN_PLACE: return c->decodes_in_place.load();
        case RS_STAT_REC_STRIPES_TABLE: return c->rec_stripes_table.load();
        case RS_STAT_REC_STRIPES_SYNDROME: return c->rec_stripes_syndrome.load();
        case RS_STAT_ENCODE_BATCHES: return c->encode_batches.load();
        case RS_STAT_MAILBOX_CALLS: return c->mailbox_calls.load();
        case RS_STAT_MAILBOX_RECOVERED: return c->mailbox_recovered.load();
        case RS_STAT_LEASES: {
            std::lock_guard<std::mutex> lk(const_cast<rs_ctx*>(c)->lease_mu);
            return static_cast<int64_t>(c->leases.size());
        }
        default: return RS_EINVAL;
    }
}

int rs_pattern_rows(rs_ctx* c, const uint8_t* erased, uint8_t* rows, int* count) {
    if (!c || !erased || !rows || !count) return RS_EINVAL;
    if (c->set) return rs_pattern_rows(rsmi::set_member(c->set, 0), erased, rows, count);
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    const hipStream_t s = lg.L->stream;
    std::unique_lock<std::shared_mutex> wl(c->pat_mu);
    std::vector<uint32_t> pid;
    size_t missing = 0;
    int st = lookup_patterns(c, erased, 1, pid, false, &missing);
    if (st != RS_OK) return st;
    if (missing && c->pat_index.size() + 1 > c->pat_cap) evict_patterns(c);
    st = lookup_patterns(c, erased, 1, pid, true, nullptr);
    if (st != RS_OK) return st;
    st = flush_patterns(c);
    if (st != RS_OK) return st;
    const size_t id = pid[0], mk = static_cast<size_t>(c->m) * c->k;
    wait_patterns(c, s);
    if (hipMemcpyAsync(rows, static_cast<uint8_t*>(c->d_pcoef.p) + id * mk, mk, hipMemcpyDeviceToHost, s) !=
        hipSuccess)
        return RS_EDEVICE;
    *count = static_cast<int>(c->h_cnt[id]);
    return pattern_status(c, id, 1, s);  // synchronises s
}

int rs_prepare_patterns(rs_ctx* c, int max_e, void* stream) {
    if (!c || max_e < 0 || max_e > c->m) return RS_EINVAL;
    if (c->set) {  // every member, each on its own device's null stream
        if (stream) return RS_EINVAL;
        return rsmi::set_run(c->set, [&](int i) { return rs_prepare_patterns(rsmi::set_member(c->set, i), max_e, nullptr); });
    }
    // count = sum_{e=1..max_e} C(n, e)
    double total = 0, binom = 1;
    for (int e = 1; e <= max_e; ++e) {
        binom = binom * (c->n - e + 1) / e;
        total += binom;
    }
    if (total > double(1 << 20) || total > double(c->pat_cap)) return RS_EINVAL;
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    std::unique_lock<std::shared_mutex> wl(c->pat_mu);
    std::vector<uint8_t> er(c->n);
    std::vector<uint32_t> pid;
    std::vector<int> idx;
    // Every pattern of 1..max_e erasures, in lexicographic order of ids.
    auto for_each_pattern = [&](auto&& fn) -> int {
        for (int e = 1; e <= max_e; ++e) {
            idx.resize(e);
            for (int i = 0; i < e; ++i) idx[i] = i;
            while (true) {
                std::fill(er.begin(), er.end(), 0);
                for (int v : idx) er[v] = 1;
                const int err = fn();
                if (err != RS_OK) return err;
                int i = e - 1;
                while (i >= 0 && idx[i] == c->n - e + i) --i;
                if (i < 0) break;
                ++idx[i];
                for (int j = i + 1; j < e; ++j) idx[j] = idx[j - 1] + 1;
            }
        }
        return RS_OK;
    };
    // Evict only when the patterns not cached yet would pass the cap.
    size_t absent = 0;
    (void)for_each_pattern([&] {
        size_t miss = 0;
        const int err = lookup_patterns(c, er.data(), 1, pid, false, &miss);
        absent += miss;
        return err;
    });
    if (absent && c->pat_index.size() + absent > c->pat_cap) evict_patterns(c);
    const int err = for_each_pattern([&] { return lookup_patterns(c, er.data(), 1, pid, true, nullptr); });
    if (err != RS_OK) return err;
    const int st = flush_patterns(c);
    if (st != RS_OK) return st;
    return pattern_status(c, 0, c->h_cnt.size(), s);  // synchronises s
}

int rs_encode_stripes(rs_ctx* c, const void* data, size_t dss, void* parity, size_t pss,
                      size_t pitch, size_t len, size_t stripes, void* stream) {
    if (!c) return RS_EINVAL;
    if (c->m == 0 || stripes == 0 || len == 0) return RS_OK;
    if (!check_stripes_args(c, data, dss, parity, pss, pitch, len)) return RS_EINVAL;
    if (c->set) {
        rs_ctx* mc = routed(c, data);
        return mc ? rs_encode_stripes(mc, data, dss, parity, pss, pitch, len, stripes, stream) : RS_EINVAL;
    }
    // Reads only state that is immutable after rs_new: no lock, no lease.
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    rsmi::MatArgs a = base_args(c, const_cast<void*>(data), dss, parity, pss, pitch, len, stripes);
    set_patterns(c, 1, c->d_encpat.p, a);
    a.stripe_desc = nullptr;
    return hip_status(launch_encode(c, a, static_cast<hipStream_t>(stream)));
}

int rs_reconstruct_stripes(rs_ctx* c, void* data, size_t dss, void* parity, size_t pss,
                           size_t pitch, size_t len, size_t stripes, const uint8_t* erased,
                           void* stream) {
    if (!c || !erased) return RS_EINVAL;
    if (stripes == 0 || len == 0) return RS_OK;
    if (!check_stripes_args(c, data, dss, parity, pss, pitch, len)) return RS_EINVAL;
    if (c->set) {
        rs_ctx* mc = routed(c, data);
        return mc ? rs_reconstruct_stripes(mc, data, dss, parity, pss, pitch, len, stripes, erased, stream) : RS_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    return reconstruct(c, *lg.L, data, dss, parity, pss, pitch, len, stripes, erased, nullptr,
                       static_cast<hipStream_t>(stream));
}

int rs_reconstruct_ptrs(rs_ctx* c, const uint64_t* shard_ptrs, size_t len, size_t stripes, const uint8_t* erased,
                        void* stream) {
    if (!c || !erased || !shard_ptrs) return RS_EINVAL;
    if (stripes == 0 || len == 0) return RS_OK;
    if (round_up(len, 16) / 16 >= (size_t(1) << 28)) return RS_EINVAL;  // 32-bit column offsets
    if (reinterpret_cast<uintptr_t>(shard_ptrs) & 7u) return RS_EINVAL;
    if (c->set) {
        rs_ctx* mc = routed(c, shard_ptrs);
        return mc ? rs_reconstruct_ptrs(mc, shard_ptrs, len, stripes, erased, stream) : RS_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    return reconstruct(c, *lg.L, nullptr, 0, nullptr, 0, round_up(len, 16), len, stripes, erased, shard_ptrs,
                       static_cast<hipStream_t>(stream));
}

int rs_encode(rs_ctx* c, const uint8_t* input, size_t len, uint8_t* parity) {
    if (!c) return RS_EINVAL;
    rsmi::trace_begin();
    struct TraceEnd {
        ~TraceEnd() { rsmi::trace_end(); }
    } trace_end_at_exit;
    if (len % static_cast<size_t>(c->k) != 0) return RS_ELEN_NOT_MULTIPLE;
    const size_t S = len / static_cast<size_t>(c->k);
    if (S == 0 || c->m == 0) return RS_OK;
    if (!input || !parity) return RS_EINVAL;
    if (c->set) {
        const SetPick pk(c->set);
        return rs_encode(pk.member(), input, len, parity);
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    rsmi::trace_mark("validate+lease");
    int rc_in_place = RS_OK;
    if (encode_in_place(c, *lg.L, input, S, parity, &rc_in_place)) return rc_in_place;
    if (encode_staged(c, *lg.L, input, S, parity, &rc_in_place)) return rc_in_place;
    rsmi::HostPipeline* pipe = lg.L->pipeline();
    if (!pipe) return RS_ENOMEM;
    std::vector<const uint8_t*> srcs(c->k);
    std::vector<uint8_t*> dsts(c->m);
    for (int j = 0; j < c->k; ++j) srcs[j] = input + static_cast<size_t>(j) * S;
    for (int t = 0; t < c->m; ++t) dsts[t] = parity + static_cast<size_t>(t) * S;
    auto launch = [c](uint8_t* din, uint8_t* dout, size_t pitch, size_t w, hipStream_t st) {
        rsmi::MatArgs a = base_args(c, din, 0, dout, 0, pitch, w, 1);
        set_patterns(c, 1, c->d_encpat.p, a);
        return launch_encode(c, a, st);
    };
    return hip_status(pipe->run(srcs.data(), c->k, dsts.data(), c->m, S, launch));
}

int rs_decode(rs_ctx* c, int* numbers, const uint8_t** shares, int count, size_t share_len,
              uint8_t* dst) {
    if (!c) return RS_EINVAL;
    rsmi::trace_begin();
    struct TraceEnd {
        ~TraceEnd() { rsmi::trace_end(); }
    } trace_end_at_exit;
    const int k = c->k, n = c->n;
    if (count < k) return RS_ENOT_ENOUGH;  // Correct: NotEnoughShares comes first
    if (count <= 0) return RS_ENO_SHARES;
    if (!numbers || !shares || (!dst && share_len)) return RS_EINVAL;
    for (int i = 0; i < count; ++i)
        if (numbers[i] < 0 || numbers[i] >= n) return RS_EBAD_SHARE_ID;
    // sort.Sort(byNumber(shares)): in place on the caller's arrays.
    std::vector<int> order(count);
    for (int i = 0; i < count; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return numbers[a] < numbers[b]; });
    std::vector<int> nums(count);
    std::vector<const uint8_t*> ptrs(count);
    for (int i = 0; i < count; ++i) {
        nums[i] = numbers[order[i]];
        ptrs[i] = shares[order[i]];
    }
    std::copy(nums.begin(), nums.end(), numbers);
    std::copy(ptrs.begin(), ptrs.end(), shares);
    std::vector<uint8_t> present(n, 0);
    std::vector<const uint8_t*> by_id(n, nullptr);
    int distinct = 0;
    for (int i = 0; i < count; ++i)
        if (!present[nums[i]]) {
            present[nums[i]] = 1;
            by_id[nums[i]] = ptrs[i];
            ++distinct;
        }
    if (distinct < k) return RS_ESINGULAR;  // duplicate numbers: singular decode matrix
    if (share_len == 0) return RS_OK;
    for (int i = 0; i < n; ++i)
        if (present[i] && !by_id[i]) return RS_EINVAL;
    if (c->set) {  // numbers / shares are sorted already: the member sorts them again as a no-op
        const SetPick pk(c->set);
        return rs_decode(pk.member(), numbers, shares, count, share_len, dst);
    }
    std::vector<uint8_t> aside;  // shares that alias dst, set aside before anything is written
    {
        OutRanges out;
        out.add(dst, static_cast<size_t>(k) * share_len);
        out.seal();
        set_aside_aliases(out, by_id, share_len, aside);
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    rsmi::trace_mark("validate+lease");
    if (distinct > k) return correct_decode(c, *lg.L, present, by_id, share_len, dst);
    // Survivors in engine-pinned memory (an rs_arena, rs_pinned_alloc): one
    // launch reads them in place, no staging copies.
    int rc_in_place = RS_OK;
    if (decode_in_place(c, *lg.L, present, by_id, share_len, dst, &rc_in_place)) return rc_in_place;
    return rebuild_into(c, *lg.L, present, by_id, share_len, dst);
}

namespace {
// Pinned staging one batched host-API pass may use (rs_encode_batch: inputs +
// parity; rs_decode_batch: survivors + regenerated rows).  Larger batches go
// in groups of messages, so a lease's pinned memory stays bounded whatever the
// batch (RSMI_BATCH_STAGE_MB overrides, for tests).
size_t batch_stage_cap() {
    static const size_t cap = [] {
        const char* e = std::getenv("RSMI_BATCH_STAGE_MB");
        const long v = e ? std::atol(e) : 0;
        return (v > 0 ? static_cast<size_t>(v) : size_t(512)) << 20;
    }();
    return cap;
}

// Chunks of messages for the direct batch forms: one per 256 KiB of input
// bytes, at most kBatchChunks (their events) and one message each at least
// -- two config-1 messages already run as two chunks, the first coded while
// the second is staged (the single-message path's two-chunk overlap).
size_t direct_batch_chunks(size_t messages, size_t in_bytes) {
    static const size_t cap = [] {
        const char* e = std::getenv("RSMI_BATCH_CHUNKS");
        const long v = e ? std::atol(e) : static_cast<long>(kBatchChunks);
        return static_cast<size_t>(std::max(1L, std::min(v, static_cast<long>(kBatchChunksMax))));
    }();
    const size_t by_bytes = std::max<size_t>(1, in_bytes / (size_t(256) << 10));
    return std::max<size_t>(1, std::min({messages, cap, by_bytes}));
}
}  // namespace

int rs_decode_batch(rs_ctx* c, int batch, const int* counts, int* numbers, const uint8_t** shares,
                    size_t S, uint8_t** dsts, int* status) {
    if (!c || batch < 0 || (batch && (!counts || !numbers || !shares || !dsts || !status)))
        return RS_EINVAL;
    rsmi::trace_begin();
    struct TraceEnd {
        ~TraceEnd() { rsmi::trace_end(); }
    } trace_end_at_exit;
    if (c->set) return rsmi::set_decode_batch(c->set, batch, counts, numbers, shares, S, dsts, status);
    const int k = c->k, n = c->n;
    if (batch > 0 && S > 0) {
        // Shares that alias any message's dst (infectious lets shares alias
        // dst; a batch also lets message b's dst hold message b''s arena
        // survivors): the present shares go to the dsts and regenerated rows
        // come out while later chunks' kernels still read survivors, so those
        // shares are copied aside first and the batch runs on a pointer array
        // that names the copies; the caller's array is sorted like it.
        size_t total = 0;
        for (int b = 0; b < batch; ++b) total += static_cast<size_t>(std::max(counts[b], 0));
        OutRanges out;
        for (int b = 0; b < batch; ++b) out.add(dsts[b], static_cast<size_t>(k) * S);
        out.seal();
        std::vector<const uint8_t*> loc(shares, shares + total), orig(loc);
        std::vector<uint8_t> aside;
        if (set_aside_aliases(out, loc, S, aside)) {
            const int rc = rs_decode_batch(c, batch, counts, numbers, loc.data(), S, dsts, status);
            // loc was sorted with numbers; map copies back to the caller's pointers
            const uintptr_t a0 = reinterpret_cast<uintptr_t>(aside.data()), a1 = a0 + aside.size();
            std::vector<const uint8_t*> moved;  // orig pointers of the copies, in copy order
            for (const uint8_t* p : orig)
                if (p && out.meets(p, S)) moved.push_back(p);
            for (size_t j = 0; j < total; ++j) {
                const uintptr_t v = reinterpret_cast<uintptr_t>(loc[j]);
                shares[j] = (v >= a0 && v < a1) ? moved[(v - a0) / S] : loc[j];
            }
            return rc;
        }
    }
    {
        // Groups of messages within the staging cap (k survivors and at most
        // k regenerated rows each), in message order; the first failing
        // status of the whole batch is returned.
        const size_t per_msg = 2 * static_cast<size_t>(k) * round_up(std::max<size_t>(S, 1), 256);
        const size_t group = std::max<size_t>(1, batch_stage_cap() / per_msg);
        if (static_cast<size_t>(batch) > group) {
            int rc = RS_OK;
            size_t off = 0;
            for (int b0 = 0; b0 < batch;) {
                const int nb = static_cast<int>(std::min<size_t>(group, static_cast<size_t>(batch - b0)));
                size_t cnt = 0;
                for (int b = b0; b < b0 + nb; ++b) cnt += static_cast<size_t>(std::max(counts[b], 0));
                const int r = rs_decode_batch(c, nb, counts + b0, numbers + off, shares + off, S, dsts + b0, status + b0);
                if (r != RS_OK && rc == RS_OK) rc = r;
                off += cnt;
                b0 += nb;
            }
            return rc;
        }
    }
    // 1. validate + sort each message (rs_decode semantics); messages with
    //    exactly k distinct shares go to the batched launch.
    std::vector<size_t> first(batch + 1, 0);
    for (int b = 0; b < batch; ++b) first[b + 1] = first[b] + static_cast<size_t>(std::max(counts[b], 0));
    std::vector<int> fast;  // messages for the batched launch
    std::vector<std::vector<const uint8_t*>> by(batch);
    int rc = RS_OK;
    for (int b = 0; b < batch; ++b) {
        int* nb = numbers + first[b];
        const uint8_t** sb = shares + first[b];
        const int cnt = counts[b];
        status[b] = RS_OK;
        if (cnt < k) status[b] = RS_ENOT_ENOUGH;
        for (int i = 0; i < cnt && status[b] == RS_OK; ++i)
            if (nb[i] < 0 || nb[i] >= n) status[b] = RS_EBAD_SHARE_ID;
        if (status[b] != RS_OK) {
            if (rc == RS_OK) rc = status[b];
            continue;
        }
        std::vector<int> order(cnt);
        for (int i = 0; i < cnt; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return nb[x] < nb[y]; });
        std::vector<int> nums(cnt);
        std::vector<const uint8_t*> ptrs(cnt);
        for (int i = 0; i < cnt; ++i) {
            nums[i] = nb[order[i]];
            ptrs[i] = sb[order[i]];
        }
        std::copy(nums.begin(), nums.end(), nb);
        std::copy(ptrs.begin(), ptrs.end(), sb);
        by[b].assign(n, nullptr);
        int distinct = 0;
        for (int i = 0; i < cnt; ++i)
            if (!by[b][nums[i]]) {
                by[b][nums[i]] = ptrs[i];
                ++distinct;
            }
        if (distinct < k) {
            status[b] = RS_ESINGULAR;
            if (rc == RS_OK) rc = status[b];
        } else if (distinct > k) {
            status[b] = 1;  // Correct path, below
        } else if (S > 0) {
            fast.push_back(b);
        }
    }
    // 2. messages needing Correct: one by one
    for (int b = 0; b < batch; ++b) {
        if (status[b] != 1) continue;
        status[b] = rs_decode(c, numbers + first[b], shares + first[b], counts[b], S, dsts[b]);
        if (status[b] != RS_OK && rc == RS_OK) rc = status[b];
    }
    auto first_fail = [&] {  // the call's result: the first failing status in message order
        for (int b = 0; b < batch; ++b)
            if (status[b] != RS_OK) return status[b];
        return static_cast<int>(RS_OK);
    };
    (void)rc;
    if (fast.empty()) return first_fail();
    if (fast.size() == 1) {  // one message: the single-message path (two staged column chunks)
        const int b = fast[0];
        status[b] = rs_decode(c, numbers + first[b], shares + first[b], counts[b], S, dsts[b]);
        return first_fail();
    }
    auto fast_path = [&]() -> int {
        // 3. the rest: one pointer-mode reconstruct launch.  PCIe carries only
        //    the k survivors of each message in (packed [batch][k][pitch]) and
        //    only the regenerated data shards out; the kernel reads survivors
        //    where they landed and writes each erased shard to its own row of an
        //    output buffer (data rows first), through a [batch][n] shard-address
        //    table.  Present data shards go from the caller's buffers to dst on
        //    the host.
        const size_t pitch = round_up(S, 256);
        const size_t B = fast.size();
        std::vector<uint8_t> erased(B * static_cast<size_t>(n), 0);
        std::vector<rsmi::CopyPool::Piece> in, direct;
        std::vector<uint8_t*> regen;  // output row r (< E) -> caller destination
        size_t n_par_out = 0;
        for (size_t j = 0; j < B; ++j)
            for (int i = 0; i < n; ++i) {
                const uint8_t* p = by[fast[j]][i];
                if (p) {
                    if (i < k) direct.push_back({dsts[fast[j]] + static_cast<size_t>(i) * S, p, S});
                } else {
                    erased[j * n + i] = 1;
                    if (i < k) regen.push_back(dsts[fast[j]] + static_cast<size_t>(i) * S);
                    else ++n_par_out;
                }
            }
        const size_t E = regen.size();
        const size_t out_rows = E + n_par_out;
        // Zero-copy receive: when every survivor lies, 16-byte aligned, in
        // engine-pinned memory (rs_pinned_alloc / rs_arena), the kernel reads it
        // there over PCIe -- no staging copy, no H2D of survivors.
        const size_t sb = round_up(S, 16);
        std::vector<uint64_t> dev_of(B * static_cast<size_t>(n), 0);
        bool in_place = std::getenv("RSMI_NO_DIRECT") == nullptr;
        for (size_t j = 0; j < B && in_place; ++j)
            for (int i = 0; i < n && in_place; ++i)
                if (const uint8_t* p = by[fast[j]][i]) {
                    const uint64_t d = (reinterpret_cast<uintptr_t>(p) & 15u) ? 0 : rsmi::pinned_device_address(p, sb);
                    in_place = d != 0;
                    dev_of[j * n + i] = d;
                }
        const size_t packed = in_place ? 0 : B * static_cast<size_t>(k) * pitch;
        ++(in_place ? c->batches_in_place : c->batches_staged);
        DeviceGuard g(c->device);
        if (!g.ok) return RS_EDEVICE;
        LeaseGuard lg(c);
        if (!lg.L) return RS_ENOMEM;
        Lease& L = *lg.L;
        rsmi::HostPipeline* pipe = L.pipeline();
        if (!pipe) return RS_ENOMEM;
        const hipStream_t s = L.stream;
        static const bool batch_dma = [] {
            const char* e = std::getenv("RSMI_BATCH_DMA");  // 1: stage survivors by DMA (round 4; A/B)
            return e && std::atoi(e) != 0;
        }();
        if (!batch_dma) {
            // Survivors read by the kernel over PCIe where they are (engine-pinned,
            // in_place) or where the copy pool staged them (non-temporal stores),
            // in chunks of messages: chunk i is reconstructed while chunk i + 1
            // is staged and chunk i - 1's regenerated data shards -- written by
            // the kernel into pinned staging -- are copied out; erased parity (not
            // returned) goes to a device scratch row.  No DMA: the round-4 form
            // queued every chunk's H2D, then the kernel, then the D2H
            // (RSMI_BATCH_DMA=1).
            const size_t sp = round_up(S, 64);
            const size_t in_bytes = in_place ? 0 : B * static_cast<size_t>(k) * sp;
            const size_t tbl = B * static_cast<size_t>(n) * sizeof(uint64_t);
            // The lease's device buffers may last have been used on another
            // stream: order s after that before reserve_on may free them
            // (ADVICE r05), and release the staging after s on every exit.
            L.begin(s);
            struct StagingDone {
                Lease& L;
                hipStream_t s;
                ~StagingDone() {
                    L.st_batch.release_after(s);
                    L.end(s);
                }
            } staging_done{L, s};
            if (!L.st_batch.acquire(in_bytes + std::max<size_t>(E, 1) * sp) || !L.st_pieces.acquire(tbl) ||
                !L.d_pieces.reserve_on(tbl, s) || !L.d_batch.reserve_on(std::max<size_t>(n_par_out, 1) * sp, s))
                return RS_ENOMEM;
            uint8_t* h = static_cast<uint8_t*>(L.st_batch.p);
            uint8_t* hd = static_cast<uint8_t*>(L.st_batch.dev);
            uint8_t* h_out = h + in_bytes;
            uint8_t* d_out = hd + in_bytes;
            uint8_t* d_par = static_cast<uint8_t*>(L.d_batch.p);
            uint64_t* tab = static_cast<uint64_t*>(L.st_pieces.p);
            std::vector<rsmi::CopyPool::Piece> stage_in;
            stage_in.reserve(B * static_cast<size_t>(k));
            size_t r_data = 0, r_par = 0;
            for (size_t j = 0; j < B; ++j) {
                size_t q = 0;
                for (int i = 0; i < n; ++i) {
                    uint64_t& t = tab[j * n + i];
                    if (const uint8_t* p = by[fast[j]][i]) {
                        const size_t slot = j * k + q++;
                        if (in_place) {
                            t = dev_of[j * n + i];
                        } else {
                            stage_in.push_back({h + slot * sp, p, S, true});
                            t = reinterpret_cast<uint64_t>(hd + slot * sp);
                        }
                    } else if (i < k) {
                        t = reinterpret_cast<uint64_t>(d_out + r_data++ * sp);
                    } else {
                        t = reinterpret_cast<uint64_t>(d_par + r_par++ * sp);
                    }
                }
            }
            auto finish = [&](int code) {
                if (hipStreamSynchronize(s) != hipSuccess && code == RS_OK) code = RS_EDEVICE;
                return code;
            };
            if (hipMemcpyAsync(L.d_pieces.p, tab, tbl, hipMemcpyHostToDevice, s) != hipSuccess) return finish(RS_EDEVICE);
            L.st_pieces.release_after(s);
            const size_t moved = B * static_cast<size_t>(k) * sp;  // survivor bytes the kernels read
            const size_t nch = direct_batch_chunks(B, moved);
            std::vector<size_t> rows_before(B + 1, 0);  // regenerated data rows of messages [0, j)
            for (size_t j = 0; j < B; ++j) {
                size_t e_j = 0;
                for (int i = 0; i < k; ++i) e_j += by[fast[j]][i] == nullptr;
                rows_before[j + 1] = rows_before[j] + e_j;
            }
            size_t launched = 0;
            static const char* const kStage[] = {"stage0", "stage1", "stage2", "stage3", "stage4", "stage5", "stage6", "stage7"};
            static const char* const kLaunch[] = {"launch0", "launch1", "launch2", "launch3",
                                                  "launch4", "launch5", "launch6", "launch7"};
            static const char* const kWait[] = {"wait0", "wait1", "wait2", "wait3", "wait4", "wait5", "wait6", "wait7"};
            static const char* const kOut[] = {"copyout0", "copyout1", "copyout2", "copyout3",
                                               "copyout4", "copyout5", "copyout6", "copyout7"};
            static_assert(kBatchChunksMax == 8, "trace phase names");
            for (size_t ch = 0; ch < nch; ++ch) {
                const size_t j0 = B * ch / nch, j1 = B * (ch + 1) / nch;
                if (!in_place)
                    pipe->copy(std::vector<rsmi::CopyPool::Piece>(stage_in.begin() + j0 * k, stage_in.begin() + j1 * k));
                rsmi::trace_mark(kStage[ch]);
                const int st = reconstruct(c, L, nullptr, 0, nullptr, 0, sp, S, j1 - j0, erased.data() + j0 * n,
                                           static_cast<const uint64_t*>(L.d_pieces.p) + j0 * n, s);
                if (st != RS_OK || hipEventRecord(L.ev[ch], s) != hipSuccess) return finish(st != RS_OK ? st : RS_EDEVICE);
                rsmi::trace_mark(kLaunch[ch]);
                ++launched;
            }
            pipe->copy(direct);  // present data shards: no GPU, while it works
            rsmi::trace_mark("copy_present");
            for (size_t ch = 0; ch < launched; ++ch) {
                if (rsmi::wait_event(L.ev[ch]) != hipSuccess) return finish(RS_EDEVICE);
                rsmi::trace_mark(kWait[ch]);
                const size_t j0 = B * ch / nch, j1 = B * (ch + 1) / nch;
                std::vector<rsmi::CopyPool::Piece> out;
                for (size_t r = rows_before[j0]; r < rows_before[j1]; ++r) out.push_back({regen[r], h_out + r * sp, S});
                pipe->copy(out);
                rsmi::trace_mark(kOut[ch]);
            }
            return RS_OK;
        }
        L.begin(s);  // the lease's buffers may last have been read on another stream
        const size_t table_bytes = B * static_cast<size_t>(n) * sizeof(uint64_t);
        if (!L.st_batch.acquire(std::max<size_t>(std::max(packed, E * pitch), 16)) ||
            (packed && !L.d_pack.reserve_on(packed, s)) || !L.d_batch.reserve_on(std::max<size_t>(out_rows, 1) * pitch, s) ||
            !L.st_pieces.acquire(table_bytes) || !L.d_pieces.reserve_on(table_bytes, s))
            return RS_ENOMEM;
        // From the first async copy on, every exit waits for the stream: the
        // staging buffers may not be reused (or freed) while a DMA reads them.
        auto finish = [&](int code) {
            if (hipStreamSynchronize(s) != hipSuccess && code == RS_OK) code = RS_EDEVICE;
            L.end(s);
            return code;
        };
        uint8_t* h = static_cast<uint8_t*>(L.st_batch.p);
        uint8_t* dp = static_cast<uint8_t*>(L.d_pack.p);
        uint8_t* dout = static_cast<uint8_t*>(L.d_batch.p);
        uint64_t* tab = static_cast<uint64_t*>(L.st_pieces.p);
        size_t r_data = 0, r_par = E;
        for (size_t j = 0; j < B; ++j) {
            size_t q = 0;
            for (int i = 0; i < n; ++i) {
                uint64_t& t = tab[j * n + i];
                if (const uint8_t* p = by[fast[j]][i]) {
                    const size_t slot = j * k + q++;  // exactly k present (fast path)
                    if (in_place) {
                        t = dev_of[j * n + i];
                    } else {
                        in.push_back({h + slot * pitch, p, S});
                        t = reinterpret_cast<uint64_t>(dp + slot * pitch);
                    }
                } else {
                    t = reinterpret_cast<uint64_t>(dout + (i < k ? r_data++ : r_par++) * pitch);
                }
            }
        }
        if (hipMemcpyAsync(L.d_pieces.p, tab, table_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
            return finish(RS_EDEVICE);
        L.st_pieces.release_after(s);
        // Staged survivors go in chunks of messages: the host staging copy of
        // chunk i + 1 runs while chunk i crosses PCIe (the staging buffer is
        // pinned, so each hipMemcpyAsync returns at once).  `in` holds exactly k
        // pieces per message, in message order.
        const size_t chunks = in_place ? 0 : std::min<size_t>(B, packed >= kBatchChunkMin ? kBatchChunks : 1);
        for (size_t ch = 0; ch < chunks; ++ch) {
            const size_t j0 = B * ch / chunks, j1 = B * (ch + 1) / chunks;
            pipe->copy(std::vector<rsmi::CopyPool::Piece>(in.begin() + j0 * k, in.begin() + j1 * k));
            if (hipMemcpyAsync(dp + j0 * k * pitch, h + j0 * k * pitch, (j1 - j0) * k * pitch, hipMemcpyHostToDevice, s) !=
                hipSuccess)
                return finish(RS_EDEVICE);
        }
        const int st = reconstruct(c, L, nullptr, 0, nullptr, 0, pitch, S, B, erased.data(),
                                   static_cast<const uint64_t*>(L.d_pieces.p), s);
        if (st != RS_OK) return finish(st);
        // Regenerated data shards out, in chunks with an event each, so the host
        // copies chunk i into the callers' buffers while chunk i + 1 crosses.
        // (The D2H reuses the survivor staging: the stream orders it after the
        // H2D copies that read it.)
        const size_t ochunks = E == 0 ? 0 : std::min<size_t>(E, E * pitch >= kBatchChunkMin ? kBatchChunks : 1);
        int rc_dev = RS_OK;
        size_t queued = 0;
        for (size_t ch = 0; ch < ochunks && rc_dev == RS_OK; ++ch, ++queued) {
            const size_t r0 = E * ch / ochunks, r1 = E * (ch + 1) / ochunks;
            if (hipMemcpyAsync(h + r0 * pitch, dout + r0 * pitch, (r1 - r0) * pitch, hipMemcpyDeviceToHost, s) !=
                    hipSuccess ||
                hipEventRecord(L.ev[ch], s) != hipSuccess)
                rc_dev = RS_EDEVICE;
        }
        // present data shards need no GPU: copy them while the GPU works
        if (rc_dev == RS_OK) pipe->copy(direct);
        for (size_t ch = 0; ch < queued && rc_dev == RS_OK; ++ch) {
            const size_t r0 = E * ch / ochunks, r1 = E * (ch + 1) / ochunks;
            if (hipEventSynchronize(L.ev[ch]) != hipSuccess) {
                rc_dev = RS_EDEVICE;
                break;
            }
            std::vector<rsmi::CopyPool::Piece> out;
            out.reserve(r1 - r0);
            for (size_t r = r0; r < r1; ++r) out.push_back({regen[r], h + r * pitch, S});
            pipe->copy(out);
        }
        const int fin = finish(rc_dev);
        L.st_batch.release_after(s);
        return fin;
    };
    // A failure of the batched pass fails every message it carried (their
    // outputs were not all produced); the call returns the first failing
    // status in message order.
    const int fr = fast_path();
    if (fr != RS_OK)
        for (int b : fast) status[b] = fr;
    return first_fail();
}

int rs_encode_batch(rs_ctx* c, int batch, const uint8_t* const* inputs, size_t len, uint8_t* const* parities,
                    int* status) {
    if (!c || batch < 0 || (batch && (!inputs || !parities || !status))) return RS_EINVAL;
    rsmi::trace_begin();
    struct TraceEnd {
        ~TraceEnd() { rsmi::trace_end(); }
    } trace_end_at_exit;
    if (c->set) return rsmi::set_encode_batch(c->set, batch, inputs, len, parities, status);
    const size_t k = static_cast<size_t>(c->k), m = static_cast<size_t>(c->m);
    if (len % k != 0) {
        for (int b = 0; b < batch; ++b) status[b] = RS_ELEN_NOT_MULTIPLE;
        return batch ? RS_ELEN_NOT_MULTIPLE : RS_OK;
    }
    const size_t S = len / k;
    int rc = RS_OK;
    std::vector<int> todo;
    for (int b = 0; b < batch; ++b) {
        status[b] = RS_OK;
        if (S == 0 || m == 0) continue;
        if (!inputs[b] || !parities[b]) {
            status[b] = RS_EINVAL;
            if (rc == RS_OK) rc = RS_EINVAL;
            continue;
        }
        todo.push_back(b);
    }
    if (todo.empty()) return rc;
    // Messages stripe by stripe in the strided layout, [group][k][pitch] in
    // pinned staging followed by [group][m][pitch] of parity.
    const size_t pitch = round_up(S, 64);
    const size_t per_msg = (k + m) * pitch;
    // One message (it gets rs_encode's two-chunk staged path) or messages past
    // the staging cap / the kernels' column range: one rs_encode each.
    if (todo.size() == 1 || per_msg > batch_stage_cap() || round_up(S, 16) / 16 >= (size_t(1) << 28)) {
        for (int b : todo) status[b] = rs_encode(c, inputs[b], len, parities[b]);
        for (int b = 0; b < batch; ++b)  // the first failing status in message order
            if (status[b] != RS_OK) return status[b];
        return RS_OK;
    }
    // A message not coded gets the call's failure (never a stale RS_OK).
    auto fail_from = [&](size_t j0, int code) {
        for (size_t j = j0; j < todo.size(); ++j) status[todo[j]] = code;
        for (int b = 0; b < batch; ++b)
            if (status[b] != RS_OK) return status[b];
        return code;
    };
    DeviceGuard g(c->device);
    if (!g.ok) return fail_from(0, RS_EDEVICE);
    LeaseGuard lg(c);
    if (!lg.L) return fail_from(0, RS_ENOMEM);
    Lease& L = *lg.L;
    rsmi::HostPipeline* pipe = L.pipeline();
    if (!pipe) return fail_from(0, RS_ENOMEM);
    const hipStream_t s = L.stream;
    const size_t group = std::max<size_t>(1, batch_stage_cap() / per_msg);
    for (size_t g0 = 0; g0 < todo.size(); g0 += group) {
        const size_t B = std::min(group, todo.size() - g0);
        if (!L.st_batch.acquire(B * per_msg)) return fail_from(g0, RS_ENOMEM);
        uint8_t* h_in = static_cast<uint8_t*>(L.st_batch.p);
        uint8_t* h_out = h_in + B * k * pitch;
        uint8_t* d_in = static_cast<uint8_t*>(L.st_batch.dev);
        uint8_t* d_out = d_in + B * k * pitch;
        L.begin(s);
        // Chunks of messages: the staging copy of chunk i + 1 (copy pool,
        // non-temporal) runs while the kernel codes chunk i over PCIe, and
        // chunk i's parity is copied out while chunk i + 1's kernel runs.
        const size_t nch = direct_batch_chunks(B, B * k * pitch);
        hipError_t e = hipSuccess;
        size_t launched = 0;
        for (size_t ch = 0; ch < nch && e == hipSuccess; ++ch) {
            const size_t j0 = B * ch / nch, j1 = B * (ch + 1) / nch;
            std::vector<rsmi::CopyPool::Piece> in;
            in.reserve((j1 - j0) * k);
            for (size_t j = j0; j < j1; ++j)
                for (size_t i = 0; i < k; ++i)
                    in.push_back({h_in + (j * k + i) * pitch, inputs[todo[g0 + j]] + i * S, S, true});
            pipe->copy(in);
            rsmi::trace_mark(ch == 0 ? "stage0" : ch == 1 ? "stage1" : ch == 2 ? "stage2" : "stage3");
            rsmi::MatArgs a = base_args(c, d_in + j0 * k * pitch, k * pitch, d_out + j0 * m * pitch, m * pitch, pitch, S,
                                        j1 - j0);
            set_patterns(c, 1, c->d_encpat.p, a);
            a.stripe_desc = nullptr;
            e = launch_encode(c, a, s);
            if (e == hipSuccess) e = hipEventRecord(L.ev[ch], s);
            if (e == hipSuccess) ++launched;
            rsmi::trace_mark(ch == 0 ? "launch0" : ch == 1 ? "launch1" : ch == 2 ? "launch2" : "launch3");
        }
        L.end(s);
        for (size_t ch = 0; ch < launched && e == hipSuccess; ++ch) {
            e = rsmi::wait_event(L.ev[ch]);
            rsmi::trace_mark(ch == 0 ? "wait0" : ch == 1 ? "wait1" : ch == 2 ? "wait2" : "wait3");
            if (e != hipSuccess) break;
            const size_t j0 = B * ch / nch, j1 = B * (ch + 1) / nch;
            std::vector<rsmi::CopyPool::Piece> out;
            out.reserve((j1 - j0) * m);
            for (size_t j = j0; j < j1; ++j)
                for (size_t t = 0; t < m; ++t) out.push_back({parities[todo[g0 + j]] + t * S, h_out + (j * m + t) * pitch, S});
            pipe->copy(out);
            rsmi::trace_mark(ch == 0 ? "copyout0" : ch == 1 ? "copyout1" : ch == 2 ? "copyout2" : "copyout3");
        }
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(s);  // nothing may still read the staging
            for (size_t j = g0; j < todo.size(); ++j) status[todo[j]] = RS_EDEVICE;
            break;
        }
        c->encode_batches += 1;  // one per batched GPU pass (group)
    }
    (void)rc;
    for (int b = 0; b < batch; ++b)  // the first failing status in message order
        if (status[b] != RS_OK) return status[b];
    return RS_OK;
}

int rs_blake2b_device(rs_ctx* c, int count, const uint64_t* msg_ptrs, const uint64_t* lens, const uint32_t* order,
                      int digest_len, uint8_t* out, void* stream) {
    if (!c || count < 0 || digest_len < 1 || digest_len > 64) return RS_EINVAL;
    if (count == 0) return RS_OK;
    if (!msg_ptrs || !lens || !out) return RS_EINVAL;
    if (c->set) {
        rs_ctx* mc = routed(c, out);
        return mc ? rs_blake2b_device(mc, count, msg_ptrs, lens, order, digest_len, out, stream) : RS_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    rsmi::Blake2bArgs a{};
    a.ptrs = msg_ptrs;
    a.lens = lens;
    a.order = order;
    a.out = out;
    a.count = static_cast<uint32_t>(count);
    a.digest_len = static_cast<uint32_t>(digest_len);
    return hip_status(rsmi::launch_blake2b(a, static_cast<hipStream_t>(stream)));
}

int rs_blake2b_batch(rs_ctx* c, int count, const uint8_t* const* msgs, const size_t* lens, int digest_len,
                     uint8_t* out) {
    if (!c || count < 0 || digest_len < 1 || digest_len > 64) return RS_EINVAL;
    if (count == 0) return RS_OK;
    if (!msgs || !lens || !out) return RS_EINVAL;
    for (int i = 0; i < count; ++i)
        if (!msgs[i] && lens[i]) return RS_EINVAL;
    if (c->set) {
        const SetPick pk(c->set);
        return rs_blake2b_batch(pk.member(), count, msgs, lens, digest_len, out);
    }
    {
        // Consecutive groups of messages within the pinned-staging cap (a
        // message alone may exceed it: it is one group by itself).
        size_t total = 0;
        for (int i = 0; i < count; ++i) total += round_up(lens[i], 16);
        if (count > 1 && total > batch_stage_cap()) {
            for (int i0 = 0; i0 < count;) {
                int i1 = i0;
                size_t bytes = 0;
                while (i1 < count && (i1 == i0 || bytes + round_up(lens[i1], 16) <= batch_stage_cap()))
                    bytes += round_up(lens[i1++], 16);
                const int r = rs_blake2b_batch(c, i1 - i0, msgs + i0, lens + i0, digest_len,
                                               out + static_cast<size_t>(i0) * digest_len);
                if (r != RS_OK) return r;
                i0 = i1;
            }
            return RS_OK;
        }
    }
    // Longest messages first: the quads of one wave then run about the same
    // number of blocks.  Messages are packed 16-byte aligned in that order.
    std::vector<uint32_t> order(count);
    for (int i = 0; i < count; ++i) order[i] = static_cast<uint32_t>(i);
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return lens[x] > lens[y]; });
    std::vector<size_t> off(count);
    size_t total = 0;
    for (uint32_t i : order) {
        off[i] = total;
        total += round_up(lens[i], 16);
    }
    const size_t desc_bytes = round_up(static_cast<size_t>(count) * 20, 16);
    const size_t dig_bytes = static_cast<size_t>(count) * digest_len;
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    LeaseGuard lg(c);
    if (!lg.L) return RS_ENOMEM;
    Lease& L = *lg.L;
    rsmi::HostPipeline* pipe = L.pipeline();
    if (!pipe) return RS_ENOMEM;
    const hipStream_t s = L.stream;
    L.begin(s);
    if (!L.st_batch.acquire(std::max<size_t>(total, 16)) || !L.d_batch.reserve_on(std::max<size_t>(total, 16), s) ||
        !L.st_pieces.acquire(desc_bytes + dig_bytes) || !L.d_pieces.reserve_on(desc_bytes + dig_bytes, s))
        return RS_ENOMEM;
    auto finish = [&](int code) {
        if (hipStreamSynchronize(s) != hipSuccess && code == RS_OK) code = RS_EDEVICE;
        L.end(s);
        return code;
    };
    uint8_t* h = static_cast<uint8_t*>(L.st_batch.p);
    uint8_t* d = static_cast<uint8_t*>(L.d_batch.p);
    uint8_t* hd = static_cast<uint8_t*>(L.st_pieces.p);
    uint8_t* dd = static_cast<uint8_t*>(L.d_pieces.p);
    uint64_t* hptr = reinterpret_cast<uint64_t*>(hd);
    uint64_t* hlen = hptr + count;
    uint32_t* hord = reinterpret_cast<uint32_t*>(hlen + count);
    for (int i = 0; i < count; ++i) {
        hptr[i] = reinterpret_cast<uint64_t>(d + off[i]);
        hlen[i] = lens[i];
        hord[i] = order[i];
    }
    if (hipMemcpyAsync(dd, hd, desc_bytes, hipMemcpyHostToDevice, s) != hipSuccess) return finish(RS_EDEVICE);
    // Messages in, in up to kBatchChunks chunks (in packing order): the
    // staging copy of chunk i + 1 overlaps the DMA of chunk i.
    const size_t chunks = std::min<size_t>(count, total >= kBatchChunkMin ? kBatchChunks : 1);
    for (size_t ch = 0; ch < chunks; ++ch) {
        const size_t q0 = count * ch / chunks, q1 = count * (ch + 1) / chunks;
        std::vector<rsmi::CopyPool::Piece> in;
        for (size_t q = q0; q < q1; ++q)
            if (lens[order[q]]) in.push_back({h + off[order[q]], msgs[order[q]], lens[order[q]]});
        pipe->copy(in);
        const size_t b0 = off[order[q0]];
        const size_t b1 = q1 < static_cast<size_t>(count) ? off[order[q1]] : total;
        if (b1 > b0 && hipMemcpyAsync(d + b0, h + b0, b1 - b0, hipMemcpyHostToDevice, s) != hipSuccess)
            return finish(RS_EDEVICE);
    }
    rsmi::Blake2bArgs a{};
    a.ptrs = reinterpret_cast<const uint64_t*>(dd);
    a.lens = a.ptrs + count;
    a.order = reinterpret_cast<const uint32_t*>(a.lens + count);
    a.out = dd + desc_bytes;
    a.count = static_cast<uint32_t>(count);
    a.digest_len = static_cast<uint32_t>(digest_len);
    if (rsmi::launch_blake2b(a, s) != hipSuccess) return finish(RS_EDEVICE);
    if (hipMemcpyAsync(hd + desc_bytes, dd + desc_bytes, dig_bytes, hipMemcpyDeviceToHost, s) != hipSuccess)
        return finish(RS_EDEVICE);
    const int rc = finish(RS_OK);
    if (rc == RS_OK) std::memcpy(out, hd + desc_bytes, dig_bytes);
    L.st_batch.release_after(s);
    L.st_pieces.release_after(s);
    return rc;
}

int rs_blake2b_host(int count, const uint8_t* const* msgs, const size_t* lens, int digest_len, uint8_t* out,
                    int threads) {
    if (count < 0 || digest_len < 1 || digest_len > 64) return RS_EINVAL;
    if (count == 0) return RS_OK;
    if (!msgs || !lens || !out) return RS_EINVAL;
    for (int i = 0; i < count; ++i)
        if (!msgs[i] && lens[i]) return RS_EINVAL;
    rsmi::blake2b_host_batch(count, msgs, lens, digest_len, out, threads > 0 ? threads : usable_cpus());
    return RS_OK;
}

int rs_blake2b(rs_ctx* c, int count, const uint8_t* const* msgs, const size_t* lens, int digest_len, uint8_t* out,
               int* where) {
    if (!c || count < 0 || digest_len < 1 || digest_len > 64) return RS_EINVAL;
    if (where) *where = 0;
    if (count == 0) return RS_OK;
    if (!msgs || !lens || !out) return RS_EINVAL;
    const HashPlan hp = plan_hash(count, lens);
    if (hp.host) return rs_blake2b_host(count, msgs, lens, digest_len, out, hp.threads);
    if (where) *where = 1;
    return rs_blake2b_batch(c, count, msgs, lens, digest_len, out);  // a set picks its least busy member there
}

int rs_device_alloc(rs_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return RS_EINVAL;
    if (c->set) return rs_device_alloc(rsmi::set_member(c->set, 0), bytes, out);
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    return hipMalloc(out, bytes ? bytes : 1) == hipSuccess ? RS_OK : RS_ENOMEM;
}

int rs_device_free(rs_ctx* c, void* p) {
    if (!c) return RS_EINVAL;
    if (c->set) return rs_device_free(rsmi::set_member(c->set, 0), p);
    DeviceGuard g(c->device);
    return hip_status(hipFree(p));
}

int rs_stream_sync(rs_ctx* c, void* stream) {
    if (!c) return RS_EINVAL;
    if (c->set) return rs_stream_sync(rsmi::set_member(c->set, 0), stream);
    DeviceGuard g(c->device);
    return hip_status(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
}

int rs_encode_stripes_parts(rs_ctx* c, const rs_stripe_part* parts, size_t pitch, size_t len) {
    if (!c || !parts) return RS_EINVAL;
    return run_members(c, [&](int i) -> int {
        const rs_stripe_part& p = parts[i];
        if (!p.stripes) return RS_OK;
        return rs_encode_stripes(member_of(c, i), p.data, p.data_stripe_stride, p.parity, p.parity_stripe_stride, pitch,
                                 len, p.stripes, p.stream);
    });
}

int rs_reconstruct_stripes_parts(rs_ctx* c, const rs_stripe_part* parts, size_t pitch, size_t len,
                                 const uint8_t* erased) {
    if (!c || !parts || !erased) return RS_EINVAL;
    const int cnt = members_of(c);
    std::vector<size_t> first(static_cast<size_t>(cnt) + 1, 0);  // part i's stripes start at first[i]
    for (int i = 0; i < cnt; ++i) first[i + 1] = first[i] + parts[i].stripes;
    return run_members(c, [&](int i) -> int {
        const rs_stripe_part& p = parts[i];
        if (!p.stripes) return RS_OK;
        return rs_reconstruct_stripes(member_of(c, i), p.data, p.data_stripe_stride, p.parity, p.parity_stripe_stride,
                                      pitch, len, p.stripes, erased + first[i] * static_cast<size_t>(c->n), p.stream);
    });
}

int rs_reconstruct_spread(rs_ctx* c, const uint64_t* shard_ptrs, const int* owner, size_t len, size_t stripes,
                          const uint8_t* erased, void* const* streams) {
    if (!c || !shard_ptrs || !owner || !erased) return RS_EINVAL;
    if (stripes == 0 || len == 0) return RS_OK;
    if (round_up(len, 16) / 16 >= (size_t(1) << 28)) return RS_EINVAL;  // 32-bit column offsets
    const int cnt = members_of(c);
    for (size_t s = 0; s < stripes; ++s)
        if (owner[s] < 0 || owner[s] >= cnt) return RS_EINVAL;
    if (c->set && !rsmi::set_peer_ok(c->set)) return RS_EDEVICE;  // survivors on a GPU the owner cannot read
    const size_t n = static_cast<size_t>(c->n);
    return run_members(c, [&](int i) -> int {
        // Member i's stripes, in stripe order: their rows of the address
        // table and of the erasure flags.
        std::vector<uint64_t> tab;
        std::vector<uint8_t> er;
        for (size_t s = 0; s < stripes; ++s) {
            if (owner[s] != i) continue;
            tab.insert(tab.end(), shard_ptrs + s * n, shard_ptrs + (s + 1) * n);
            er.insert(er.end(), erased + s * n, erased + (s + 1) * n);
        }
        if (tab.empty()) return RS_OK;
        const hipStream_t st = streams ? static_cast<hipStream_t>(streams[i]) : nullptr;
        return reconstruct_host_table(member_of(c, i), tab.data(), len, tab.size() / n, er.data(), st);
    });
}

int rs_fill_splitmix(rs_ctx* c, void* dev, size_t len, uint64_t seed, void* stream) {
    if (!c || (!dev && len)) return RS_EINVAL;
    if (reinterpret_cast<uintptr_t>(dev) & 7u) return RS_EINVAL;
    if (c->set) {
        rs_ctx* mc = routed(c, dev);
        return mc ? rs_fill_splitmix(mc, dev, len, seed, stream) : RS_EINVAL;
    }
    DeviceGuard g(c->device);
    if (!g.ok) return RS_EDEVICE;
    return hip_status(rsmi::launch_fill_splitmix(dev, len, seed, static_cast<hipStream_t>(stream)));
}

}  // extern "C"
