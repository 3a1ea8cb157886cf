// host_pipeline.cpp -- see host_pipeline.hpp.
#include "host_pipeline.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <utility>
#include <vector>
#if defined(__x86_64__)
#include <emmintrin.h>
#endif

namespace rsmi {

namespace {
constexpr size_t kPart = size_t(1) << 20;          // memcpy split granularity
// Bytes a helper thread must get to be worth waking: handing a part to a
// sleeping worker costs tens of microseconds (futex wake, the queue lock), a
// 1 MiB memcpy on one core 12-60 us; jobs below 2 parts' worth run inline on
// the caller, larger ones are split in parts of at least this size
// (RSMI_COPY_PART_MIN overrides).
constexpr size_t kPartMin = size_t(1) << 20;
constexpr size_t kChunkBytes = size_t(8) << 20;    // survivor bytes staged per chunk
size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

int pool_threads() {
    const char* e = std::getenv("RSMI_COPY_THREADS");
    int t = e ? std::atoi(e) : static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, std::min(t, 8));
}
}  // namespace

namespace {
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#elif defined(__aarch64__)
    asm volatile("yield");
#endif
}
}  // namespace

namespace {
bool stage_nt() {
    static const bool on = [] {
        const char* e = std::getenv("RSMI_STAGE_NT");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
}  // namespace

void stage_copy(void* dst, const void* src, size_t n) {
#if defined(__x86_64__)
    if (stage_nt() && n >= 4096) {
        uint8_t* d = static_cast<uint8_t*>(dst);
        const uint8_t* s = static_cast<const uint8_t*>(src);
        const size_t head = (16u - (reinterpret_cast<uintptr_t>(d) & 15u)) & 15u;
        std::memcpy(d, s, head);
        d += head;
        s += head;
        n -= head;
        size_t i = 0;
        for (; i + 64 <= n; i += 64) {
            const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i));
            const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 16));
            const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 32));
            const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i + 48));
            _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), a);
            _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 16), b);
            _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 32), c);
            _mm_stream_si128(reinterpret_cast<__m128i*>(d + i + 48), e);
        }
        for (; i + 16 <= n; i += 16)
            _mm_stream_si128(reinterpret_cast<__m128i*>(d + i), _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + i)));
        std::memcpy(d + i, s + i, n - i);
        return;
    }
#endif
    std::memcpy(dst, src, n);
}

namespace {
bool trace_on() {
    static const bool on = [] {
        const char* e = std::getenv("RSMI_TRACE");
        return e && std::atoi(e) != 0;
    }();
    return on;
}
struct TraceCall {
    std::chrono::steady_clock::time_point t[24];
    const char* name[24];
    int n = 0;
};
thread_local TraceCall g_call;
struct TraceTotals {
    std::mutex mu;
    std::vector<std::pair<std::string, std::vector<double>>> phases;  // in first-seen order
    long calls = 0;
    ~TraceTotals() {
        if (!calls) return;
        std::fprintf(stderr, "RSMI_TRACE %ld calls, median / mean us per phase:\n", calls);
        double total = 0;
        for (auto& p : phases) {
            std::vector<double>& v = p.second;
            double sum = 0;
            for (double x : v) sum += x;
            std::sort(v.begin(), v.end());
            total += v[v.size() / 2];
            std::fprintf(stderr, "  %-28s %8.2f %8.2f  (%zu)\n", p.first.c_str(), v[v.size() / 2], sum / v.size(),
                         v.size());
        }
        std::fprintf(stderr, "  %-28s %8.2f (sum of medians)\n", "total", total);
    }
};
TraceTotals g_totals;
}  // namespace

void trace_begin() {
    if (!trace_on()) return;
    g_call.n = 0;
    trace_mark("begin");
}

void trace_mark(const char* phase) {
    if (!trace_on() || g_call.n >= 24) return;
    g_call.t[g_call.n] = std::chrono::steady_clock::now();
    g_call.name[g_call.n++] = phase;
}

void trace_end() {
    if (!trace_on() || g_call.n == 0) return;
    trace_mark("end");
    std::lock_guard<std::mutex> lk(g_totals.mu);
    ++g_totals.calls;
    for (int i = 1; i < g_call.n; ++i) {
        const double us = std::chrono::duration<double, std::micro>(g_call.t[i] - g_call.t[i - 1]).count();
        auto it = std::find_if(g_totals.phases.begin(), g_totals.phases.end(),
                               [&](const auto& p) { return p.first == g_call.name[i]; });
        if (it == g_totals.phases.end()) {
            g_totals.phases.push_back({g_call.name[i], {}});
            it = g_totals.phases.end() - 1;
        }
        it->second.push_back(us);
    }
    g_call.n = 0;
}

void stage_fence() {
#if defined(__x86_64__)
    if (stage_nt()) _mm_sfence();
#endif
}

// Polled completion, bounded: a thread polls only while its
// previous wait was short (at most the spin window: single-message calls),
// and at most max_spinners threads poll at once -- noise runs Receive once
// per peer connection, and each extra poller would burn a core for up to the
// window.  Everything else blocks in hipEventSynchronize.
hipError_t wait_event(hipEvent_t ev) {
    static const int spin_us = [] {
        const char* e = std::getenv("RSMI_SYNC_SPIN_US");
        return e ? std::max(0, std::min(std::atoi(e), 100000)) : 200;
    }();
    static const int max_spinners = [] {
        const char* e = std::getenv("RSMI_SYNC_SPINNERS");
        return e ? std::max(0, std::atoi(e)) : 2;
    }();
    static const bool adaptive = [] {
        const char* e = std::getenv("RSMI_SYNC_ADAPTIVE");  // 0: poll every wait (round 4; A/B)
        return !(e && std::atoi(e) == 0);
    }();
    static std::atomic<int> spinners{0};
    thread_local bool last_short = true;
    const auto t0 = std::chrono::steady_clock::now();
    if (spin_us > 0 && (last_short || !adaptive)) {
        if (spinners.fetch_add(1, std::memory_order_relaxed) < max_spinners) {
            const auto until = t0 + std::chrono::microseconds(spin_us);
            do {
                const hipError_t q = hipEventQuery(ev);
                if (q != hipErrorNotReady) {
                    spinners.fetch_sub(1, std::memory_order_relaxed);
                    return q;
                }
                cpu_relax();
            } while (std::chrono::steady_clock::now() < until);
        }
        spinners.fetch_sub(1, std::memory_order_relaxed);
    }
    const hipError_t r = hipEventSynchronize(ev);
    last_short = std::chrono::steady_clock::now() - t0 <= std::chrono::microseconds(spin_us);
    return r;
}

namespace {
void copy_pieces(const CopyPool::Piece* b, const CopyPool::Piece* e);
}  // namespace

// ------------------------------------------------------------ CopyPool ----
struct CopyPool::Async {
    Job job;
    bool queued = false;
};

// Pieces split at kPart and grouped into parts of about group_bytes.
void CopyPool::split(const std::vector<Piece>& pieces, size_t group_bytes, Job& job) const {
    size_t group = 0;  // bytes in the part being grouped
    job.bounds.push_back(0);
    for (const Piece& p : pieces)
        for (size_t o = 0; o < p.len; o += kPart) {
            const size_t len = std::min(kPart, p.len - o);
            job.pieces.push_back({static_cast<uint8_t*>(p.dst) + o, static_cast<const uint8_t*>(p.src) + o, len, p.nt});
            group += len;
            if (group >= group_bytes) {
                job.bounds.push_back(job.pieces.size());
                group = 0;
            }
        }
    if (job.bounds.back() != job.pieces.size()) job.bounds.push_back(job.pieces.size());
    job.parts = job.bounds.size() - 1;
}

CopyPool::Async* CopyPool::start(const std::vector<Piece>& pieces, size_t part_bytes) {
    Async* a = new (std::nothrow) Async;
    if (!a) {  // no handle: copy now
        copy_pieces(pieces.data(), pieces.data() + pieces.size());
        return nullptr;
    }
    split(pieces, std::max<size_t>(part_bytes, 1), a->job);
    if (a->job.parts == 0) {
        delete a;
        return nullptr;
    }
    if (threads_.empty()) return a;  // finish() copies it
    bool wake = false;
    {
        std::lock_guard<std::mutex> lk(mu_);
        jobs_.push_back(&a->job);
        a->queued = true;
        queued_.fetch_add(1, std::memory_order_release);
        wake = spinners_.load(std::memory_order_acquire) == 0;
    }
    if (wake) cv_.notify_one();  // a spinning worker sees queued_ without a wake-up
    return a;
}

void CopyPool::finish(Async* a) {
    if (!a) return;
    Job& job = a->job;
    size_t part = 0;
    if (!a->queued) {
        while (claim(&job, &part)) copy_part(job, part);
        delete a;
        return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    while (claim(&job, &part)) {
        lk.unlock();
        copy_part(job, part);
        lk.lock();
        ++job.finished;
    }
    job.done_cv.wait(lk, [&] { return job.finished == job.parts; });
    for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
        if (*it == &job) {
            jobs_.erase(it);
            queued_.fetch_sub(1, std::memory_order_release);
            break;
        }
    lk.unlock();
    delete a;
}

CopyPool::CopyPool(int threads) {
    const char* e = std::getenv("RSMI_COPY_SPIN_US");
    spin_us_ = e ? std::max(0, std::min(std::atoi(e), 10000)) : 0;
    const char* ms = std::getenv("RSMI_COPY_SPINNERS");
    max_spinners_ = ms ? std::max(0, std::atoi(ms)) : 1;
    for (int i = 0; i < threads - 1; ++i) threads_.emplace_back([this] { worker(); });
}

CopyPool::~CopyPool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : threads_) t.join();
}

CopyPool& CopyPool::shared() {
    // Leaked on purpose: worker threads must not be joined from a static
    // destructor after the runtime has started tearing down.
    static CopyPool* pool = new CopyPool(pool_threads());
    return *pool;
}

bool CopyPool::claim(Job* j, size_t* part) {
    if (j->next >= j->parts) return false;
    *part = j->next++;
    return true;
}

namespace {
// Copies pieces [b, e); non-temporal pieces are fenced before the copier
// reports them done (another thread's launch reads them next).
void copy_pieces(const CopyPool::Piece* b, const CopyPool::Piece* e) {
    bool nt = false;
    for (const CopyPool::Piece* p = b; p != e; ++p) {
        if (p->nt) {
            stage_copy(p->dst, p->src, p->len);
            nt = true;
        } else {
            std::memcpy(p->dst, p->src, p->len);
        }
    }
    if (nt) stage_fence();
}
}  // namespace

void CopyPool::copy_part(const Job& j, size_t part) {
    copy_pieces(j.pieces.data() + j.bounds[part], j.pieces.data() + j.bounds[part + 1]);
}

void CopyPool::worker() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        if (jobs_.empty() && spin_us_ > 0 && !stop_) {
            // Out of work: spin a while for the next job before sleeping
            // (at most max_spinners_ workers at once).
            if (spinners_.fetch_add(1, std::memory_order_acq_rel) < max_spinners_) {
                lk.unlock();
                const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us_);
                while (queued_.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
                    cpu_relax();
                lk.lock();
            }
            spinners_.fetch_sub(1, std::memory_order_acq_rel);
        }
        cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
        if (stop_) return;
        Job* j = jobs_.front();
        size_t part = 0;
        if (!claim(j, &part)) {  // every part handed out: the job leaves the queue
            jobs_.pop_front();
            queued_.fetch_sub(1, std::memory_order_release);
            continue;
        }
        lk.unlock();
        copy_part(*j, part);
        lk.lock();
        if (++j->finished == j->parts) j->done_cv.notify_all();
    }
}

void CopyPool::run(const std::vector<Piece>& pieces) {
    static const size_t part_min = [] {
        const char* e = std::getenv("RSMI_COPY_PART_MIN");
        const long long v = e ? std::atoll(e) : 0;
        return v > 0 ? static_cast<size_t>(v) : kPartMin;
    }();
    size_t total = 0;
    for (const Piece& p : pieces) total += p.len;
    if (total < 2 * part_min || threads_.empty()) {  // not worth a hand-off
        copy_pieces(pieces.data(), pieces.data() + pieces.size());
        return;
    }
    // Parts of about total / (2 x threads), at least part_min bytes.
    const size_t group_bytes = std::max(part_min, total / (2 * (threads_.size() + 1)));
    Job job;
    split(pieces, group_bytes, job);
    if (job.parts == 0) return;
    if (threads_.empty() || job.parts == 1) {
        for (size_t i = 0; i < job.parts; ++i) copy_part(job, i);
        return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    jobs_.push_back(&job);
    queued_.fetch_add(1, std::memory_order_release);
    cv_.notify_all();
    // The calling thread works on its own job.  Workers only touch `job`
    // under mu_ while it is queued or after claiming a part (finished <
    // parts), so it may live on this stack.
    size_t part = 0;
    while (claim(&job, &part)) {
        lk.unlock();
        copy_part(job, part);
        lk.lock();
        ++job.finished;
    }
    job.done_cv.wait(lk, [&] { return job.finished == job.parts; });
    for (auto it = jobs_.begin(); it != jobs_.end(); ++it)
        if (*it == &job) {
            jobs_.erase(it);
            queued_.fetch_sub(1, std::memory_order_release);
            break;
        }
}

// -------------------------------------------------------- HostPipeline ----
HostPipeline::HostPipeline() : pool_(CopyPool::shared()) {
    const char* e = std::getenv("RSMI_HOSTPIPE");
    direct_ = !(e && std::strcmp(e, "dma") == 0);
}

HostPipeline::~HostPipeline() {
    for (Slot& s : slots_) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (!direct_ && s.d_in) (void)hipFreeAsync(s.d_in, s.stream);
        if (!direct_ && s.d_out) (void)hipFreeAsync(s.d_out, s.stream);
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.h_in) (void)hipHostFree(s.h_in);
        if (s.h_out) (void)hipHostFree(s.h_out);
        for (uint8_t* r : s.retired) (void)hipHostFree(r);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
}

// Grows one side of a slot (its previous chunk was drained, and all its
// device work ran on s.stream): the device buffer is replaced in stream order
// (hipFreeAsync / hipMallocAsync, no sync), the pinned one is retired until
// the pipeline is destroyed (hipHostFree would sync the whole device).  x2
// growth bounds both the number of growths and the retired bytes.
bool HostPipeline::grow(Slot& s, uint8_t** h, uint8_t** d, size_t* cap, size_t bytes) {
    const size_t want = std::max(bytes, 2 * *cap);
    uint8_t* nh = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&nh), want, hipHostMallocDefault) != hipSuccess) return false;
    if (direct_) {
        // The kernel addresses the staging itself; the outgrown buffer may
        // still be read by the slot's previous chunk only if it was not
        // drained, and grow runs after drain.
        void* alias = nullptr;
        if (hipHostGetDevicePointer(&alias, nh, 0) != hipSuccess) alias = nh;
        if (*h) s.retired.push_back(*h);
        *h = nh;
        *d = static_cast<uint8_t*>(alias);
        *cap = want;
        return true;
    }
    if (*d && hipFreeAsync(*d, s.stream) != hipSuccess) {
        (void)hipHostFree(nh);
        return false;
    }
    *d = nullptr;
    if (*h) s.retired.push_back(*h);
    *h = nh;
    *cap = 0;
    if (hipMallocAsync(reinterpret_cast<void**>(d), want, s.stream) != hipSuccess) {
        *d = nullptr;
        return false;
    }
    *cap = want;
    return true;
}

bool HostPipeline::ensure(Slot& s, size_t in_bytes, size_t out_bytes) {
    if (!s.stream && hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) return false;
    if (!s.done && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return false;
    if (in_bytes > s.cap_in && !grow(s, &s.h_in, &s.d_in, &s.cap_in, in_bytes)) return false;
    if (out_bytes > s.cap_out && !grow(s, &s.h_out, &s.d_out, &s.cap_out, out_bytes)) return false;
    return true;
}

hipError_t HostPipeline::drain(Slot& s, uint8_t* const* dsts, int e) {
    if (!s.pending) return hipSuccess;
    s.pending = false;
    const hipError_t err = wait_event(s.done);
    if (err != hipSuccess) return err;
    std::vector<CopyPool::Piece> out;
    for (int t = 0; t < e; ++t) out.push_back({dsts[t] + s.c0, s.h_out + t * s.pitch, s.w});
    pool_.run(out);
    return hipSuccess;
}

hipError_t HostPipeline::run(const uint8_t* const* srcs, int k, uint8_t* const* dsts, int e,
                             size_t S, const ChunkLaunch& launch, const std::function<void()>& while_gpu) {
    if (S == 0 || e == 0) {
        if (while_gpu) while_gpu();
        return hipSuccess;
    }
    // Column chunk per shard: about kChunkBytes of survivors per chunk
    // (RSMI_HOSTPIPE_CHUNK overrides, for A/B runs).
    static const size_t chunk_bytes = [] {
        const char* e = std::getenv("RSMI_HOSTPIPE_CHUNK");
        const long long v = e ? std::atoll(e) : 0;
        return v > 0 ? static_cast<size_t>(v) : kChunkBytes;
    }();
    const size_t cb = round_up(std::min(S, std::max<size_t>(4096, chunk_bytes / k)), 256);
    const size_t nchunks = (S + cb - 1) / cb;
    hipError_t err = hipSuccess;
    size_t c = 0;
    for (; c < nchunks && err == hipSuccess; ++c) {
        Slot& s = slots_[c % kSlots];
        err = drain(s, dsts, e);  // results of chunk c - kSlots
        if (err != hipSuccess) break;
        if (!ensure(s, cb * static_cast<size_t>(k), cb * static_cast<size_t>(e))) {
            err = hipErrorOutOfMemory;
            break;
        }
        const size_t c0 = c * cb, w = std::min(cb, S - c0);
        std::vector<CopyPool::Piece> in;
        for (int j = 0; j < k; ++j) in.push_back({s.h_in + j * cb, srcs[j] + c0, w});
        pool_.run(in);
        if (direct_) {
            err = launch(s.d_in, s.d_out, cb, w, s.stream);
        } else {
            err = hipMemcpyAsync(s.d_in, s.h_in, cb * static_cast<size_t>(k), hipMemcpyHostToDevice, s.stream);
            if (err == hipSuccess) err = launch(s.d_in, s.d_out, cb, w, s.stream);
            if (err == hipSuccess)
                err = hipMemcpyAsync(s.h_out, s.d_out, cb * static_cast<size_t>(e), hipMemcpyDeviceToHost, s.stream);
        }
        if (err == hipSuccess) err = hipEventRecord(s.done, s.stream);
        if (err == hipSuccess) {
            s.pending = true;
            s.c0 = c0;
            s.w = w;
            s.pitch = cb;
        }
    }
    if (while_gpu) while_gpu();
    // Drain the last chunks in order (also after an error, so no slot is
    // left holding a pending copy into caller memory).
    for (size_t i = 0; i < kSlots; ++i) {
        Slot& s = slots_[(c + i) % kSlots];
        const hipError_t d = drain(s, dsts, e);
        if (err == hipSuccess) err = d;
    }
    return err;
}

}  // namespace rsmi
