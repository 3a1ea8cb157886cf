// host_pipeline.hpp -- the host-buffer path of the C ABI (rs_encode /
// rs_decode, i.e. the cgo calls replacing infectious Encode/Decode at
// main.go:262 / :77): caller bytes are streamed through pinned
// (hipHostMalloc) staging in column chunks.  Each chunk's kernel reads its
// survivors from the pinned staging and writes its outputs back into it
// over PCIe (direct mode: no copy-engine transfer, whose setup dominated a
// 1 MiB message), on one of three HIP streams so that chunk c's GPU work
// overlaps the staging copies of chunks c-1 and c+1.  Pageable <-> pinned
// copies are split over a process-wide worker pool.
//
// Every call on an rs_ctx leases its own HostPipeline (rsmi.cpp Lease), so
// concurrent Receive goroutines (main.go:49-52) each stream through their
// own slots; the copy pool takes jobs from any number of callers at once.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rsmi {

// Fixed set of worker threads running memcpy pieces for any number of
// concurrent callers.  Each run() is a job; workers take parts from the
// oldest unfinished job and the calling thread works on its own job.
class CopyPool {
public:
    explicit CopyPool(int threads);
    ~CopyPool();
    struct Piece {
        void* dst;
        const void* src;
        size_t len;
        bool nt = false;  // dst is pinned staging a kernel reads next: stage_copy (+ fence)
    };
    // Copies every piece (split further into <= 1 MiB parts); returns when done.
    void run(const std::vector<Piece>& pieces);
    // An asynchronous job: queued for the workers in parts of about
    // part_bytes, joined by finish(), which copies every part no worker has
    // claimed yet and waits for the claimed ones -- so a pool whose workers
    // are asleep costs the caller one wake-up call, and a spinning worker
    // takes the parts while the caller does other work (a single message's
    // second staging chunk and present shares, rsmi.cpp decode_launch).
    struct Async;
    Async* start(const std::vector<Piece>& pieces, size_t part_bytes);  // nullptr: nothing to copy
    void finish(Async* a);                                              // joins and frees a
    // Workers that run out of parts spin this long for the next job before
    // sleeping on the condition variable (RSMI_COPY_SPIN_US, default 0), at
    // most max_spinners of them at once (RSMI_COPY_SPINNERS, default 1): a
    // stream of messages then finds a helper awake, an idle process burns no
    // core after the window.
    int spin_us() const { return spin_us_; }
    // The process-wide pool (RSMI_COPY_THREADS workers, default min(8, cpus)).
    static CopyPool& shared();

private:
    // A job's pieces, big ones split at 1 MiB, are handed out in parts:
    // part i covers pieces [bounds[i], bounds[i + 1]) -- runs of small
    // pieces are grouped so that thousands of small messages do not cost a
    // lock round trip each.
    struct Job {
        std::vector<Piece> pieces;
        std::vector<size_t> bounds;
        size_t next = 0, finished = 0, parts = 0;
        std::condition_variable done_cv;
    };
    void worker();
    // Claims the next part of j (mu_ held); false once every part is claimed.
    static bool claim(Job* j, size_t* part);
    static void copy_part(const Job& j, size_t part);
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job*> jobs_;
    std::atomic<int> queued_{0};  // jobs in jobs_ (read without mu_ while spinning)
    std::atomic<int> spinners_{0};  // workers in their spin window
    int spin_us_ = 0;
    int max_spinners_ = 1;
    void split(const std::vector<Piece>& pieces, size_t group_bytes, Job& job) const;
    bool stop_ = false;
};

// Waits for ev on the host: polls it for up to RSMI_SYNC_SPIN_US
// microseconds (default 200) before blocking in hipEventSynchronize.  A
// 1 MiB message's kernel finishes within that window, and the blocking wait's
// wake-up was a fixed ~10 us of the host API's latency.
hipError_t wait_event(hipEvent_t ev);

// Copies caller bytes into pinned staging that a kernel is about to read over
// PCIe.  Non-temporal stores (then a store fence) leave the lines in DRAM
// rather than dirty in the CPU's caches, where every GPU read would have to
// snoop them out: one config-1 message's kernel reads its 1 MiB 4.7 us faster
// (tools/stream_probe.hip, profiles/r05j/).  RSMI_STAGE_NT=0: plain memcpy.
void stage_copy(void* dst, const void* src, size_t n);

// Phase trace of the single-message host calls (RSMI_TRACE=1, diagnostics
// only; one branch on a static flag otherwise): trace_begin() at a call's
// entry, trace_mark("name") after each phase, trace_end() at its exit; at
// process exit the mean microseconds of every phase (time since the previous
// mark) go to stderr.
void trace_begin();
void trace_mark(const char* phase);
void trace_end();
// The fence after a run of stage_copy calls (before the launch that reads them).
void stage_fence();

// Launches the GF kernel for one chunk: survivors at din + j*pitch (j < k),
// outputs at dout + t*pitch, w coded bytes per shard.
using ChunkLaunch = std::function<hipError_t(uint8_t* din, uint8_t* dout, size_t pitch,
                                             size_t w, hipStream_t stream)>;

class HostPipeline {
public:
    HostPipeline();
    ~HostPipeline();
    // out_t[0..S) = f(srcs[0..k)[0..S)) for t < e, streamed in chunks.
    // while_gpu (optional) runs on the calling thread once every chunk is
    // queued and before the last ones are drained: host work that overlaps
    // the GPU's (rs_decode copies the present data shares into dst there).
    hipError_t run(const uint8_t* const* srcs, int k, uint8_t* const* dsts, int e, size_t S,
                   const ChunkLaunch& launch, const std::function<void()>& while_gpu = nullptr);

    // Parallel pageable <-> pinned copies on the shared worker pool.
    void copy(const std::vector<CopyPool::Piece>& pieces) { pool_.run(pieces); }

    static constexpr int kSlots = 3;
    // Direct mode (default; RSMI_HOSTPIPE=dma selects the copy-engine path):
    // the kernel codes straight out of / into the pinned staging.
    bool direct() const { return direct_; }

private:
    struct Slot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        // d_in / d_out: device buffers (DMA mode) or the device aliases of
        // h_in / h_out (direct mode: the kernel reads and writes the pinned
        // staging over PCIe, no copy engine).
        uint8_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
        size_t cap_in = 0, cap_out = 0;
        bool pending = false;
        size_t c0 = 0, w = 0, pitch = 0;
        std::vector<uint8_t*> retired;  // outgrown pinned buffers, freed with the pipeline
    };
    bool ensure(Slot& s, size_t in_bytes, size_t out_bytes);
    bool grow(Slot& s, uint8_t** h, uint8_t** d, size_t* cap, size_t bytes);
    hipError_t drain(Slot& s, uint8_t* const* dsts, int e);
    Slot slots_[kSlots];
    CopyPool& pool_;
    bool direct_ = true;
};

}  // namespace rsmi
