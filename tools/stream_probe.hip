// stream_probe.hip -- one small pageable message through the GPU: can the
// host's staging copy overlap the kernel's PCIe reads at a finer grain than
// the engine's two launches (encode_staged, rsmi.cpp)?
//
// The message: k = 10 shards of S = 104,858 bytes (config 1), pageable; the
// outputs: 4 rows, pageable.  The "code" is movement-only (rows of XORs and
// shifts) so the probe measures the host/PCIe/launch pipeline, not GF.
//
//   serial   copy all into pinned staging, one launch, wait, copy the rows out
//   chunks2  the engine's shape: copy half, launch, copy half, launch, wait
//            each, copy each half's rows out
//   flags/B  ONE launch first; then the host copies the message B blocks' columns
//            at a time into staging and raises a ready flag per group (coherent
//            pinned memory); each block waits for its group's flag (system-scope
//            acquire), codes its 4 KiB columns, writes its rows, releases them at
//            system scope and raises a per-block done flag; the host copies each
//            group's rows out as soon as its blocks are done, and returns without
//            waiting for the kernel's completion signal.  Blocks give up waiting
//            after a timeout (every wave reaches the end).
//
// Every mode's output is checked against a host reference.  Medians of 300
// calls (after 30) in microseconds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <immintrin.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int K = 10, M = 4;
constexpr size_t S = 104858, SPAN = (S + 15) & ~size_t(15);
constexpr uint32_t NCOLS = SPAN / 16, NBLK = (NCOLS + 255) / 256;
constexpr uint64_t kTimeoutTicks = 2000000;  // 20 ms of the 100 MHz clock

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Args {
    const uint8_t* in;   // staging, shard j at j * SPAN
    uint8_t* out;        // staging, row t at t * SPAN
    const uint32_t* ready;
    uint32_t* done;
    uint32_t gen, bpf, flags, blk0;  // blk0: first block of this launch (its column base)
};

__device__ __forceinline__ bool wait_ready(const uint32_t* f, uint32_t gen) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
        if (v == gen) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

__global__ __launch_bounds__(256) void code(Args a) {
    const uint32_t blk = a.blk0 + blockIdx.x, col = blk * 256u + threadIdx.x;
    bool late = false;
    if (a.flags) late = !wait_ready(a.ready + blk / a.bpf, a.gen);
    const uint32_t c = col < NCOLS ? col : NCOLS - 1;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.in + j * SPAN) + c);
    u32x4 acc[M];
#pragma unroll
    for (int t = 0; t < M; ++t) {
        acc[t] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < K; ++j) acc[t] ^= x[j] << ((t + j) & 7);
    }
    if (col < NCOLS) {
#pragma unroll
        for (int t = 0; t < M; ++t) __builtin_nontemporal_store(acc[t], reinterpret_cast<u32x4*>(a.out + t * SPAN) + col);
    }
    if (a.flags) {
        __threadfence_system();
        const int any_late = __syncthreads_or(late);
        if (threadIdx.x == 0)
            __hip_atomic_store(a.done + blk, any_late ? ~a.gen : a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The same coding with BT-thread blocks (BT / 64 waves, BT x 16-byte columns
// per block): more blocks over more CUs for the same message.
template <int BT>
__global__ __launch_bounds__(BT) void code_bt(const uint8_t* in, uint8_t* out) {
    const uint32_t col = blockIdx.x * BT + threadIdx.x;
    const uint32_t c = col < NCOLS ? col : NCOLS - 1;
    u32x4 x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + j * SPAN) + c);
    u32x4 acc[M];
#pragma unroll
    for (int t = 0; t < M; ++t) {
        acc[t] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < K; ++j) acc[t] ^= x[j] << ((t + j) & 7);
    }
    if (col < NCOLS) {
#pragma unroll
        for (int t = 0; t < M; ++t) __builtin_nontemporal_store(acc[t], reinterpret_cast<u32x4*>(out + t * SPAN) + col);
    }
}

// Launch-latency probe: writes 1 to f[0] (system scope) as its first act and
// 2 as its last; the host times launch call -> start flag -> end flag -> event.
__global__ void stamp(uint32_t* f, uint32_t gen) {
    if (threadIdx.x == 0) __hip_atomic_store(f, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(f + 1, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static void reference(const uint8_t* msg, uint8_t* rows) {
    std::vector<uint8_t> pad(SPAN * K, 0);
    for (int j = 0; j < K; ++j) std::memcpy(pad.data() + j * SPAN, msg + j * S, S);
    for (int t = 0; t < M; ++t)
        for (size_t w = 0; w < SPAN / 4; ++w) {
            uint32_t acc = 0;
            for (int j = 0; j < K; ++j) {
                uint32_t v;
                std::memcpy(&v, pad.data() + j * SPAN + 4 * w, 4);
                acc ^= v << ((t + j) & 7);
            }
            if (4 * w < S) std::memcpy(rows + t * S + 4 * w, &acc, std::min<size_t>(4, S - 4 * w));
        }
}

int main() {
    std::vector<uint8_t> msg(K * S), rows(M * S), want(M * S);
    for (size_t i = 0; i < msg.size(); ++i) msg[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
    reference(msg.data(), want.data());
    uint8_t *st_in, *st_out;
    uint32_t* flags;
    CK(hipHostMalloc(&st_in, K * SPAN, hipHostMallocDefault));
    CK(hipHostMalloc(&st_out, M * SPAN, hipHostMallocDefault));
    CK(hipHostMalloc(&flags, 4096 * 4, hipHostMallocCoherent));
    std::memset(flags, 0, 4096 * 4);
    void *d_in, *d_out, *d_flags;
    CK(hipHostGetDevicePointer(&d_in, st_in, 0));
    CK(hipHostGetDevicePointer(&d_out, st_out, 0));
    CK(hipHostGetDevicePointer(&d_flags, flags, 0));
    uint32_t* ready = flags;
    uint32_t* done = flags + 1024;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev[2], fin;
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&fin, hipEventDisableTiming));
    auto wait = [](hipEvent_t e) {  // polled, like rsmi::wait_event
        for (int i = 0; i < 2000000; ++i) {
            const hipError_t q = hipEventQuery(e);
            if (q != hipErrorNotReady) return q;
        }
        return hipEventSynchronize(e);
    };
    uint32_t gen = 0;
    int timeouts = 0;
    auto launch = [&](uint32_t blk0, uint32_t nblk, bool fl, uint32_t bpf) {
        Args a{static_cast<const uint8_t*>(d_in), static_cast<uint8_t*>(d_out), static_cast<const uint32_t*>(d_flags),
               static_cast<uint32_t*>(d_flags) + 1024, gen, bpf, fl ? 1u : 0u, blk0};
        hipLaunchKernelGGL(code, dim3(nblk), dim3(256), 0, s, a);
    };
    bool nt_copy = false;  // stream the staging copy past the CPU caches (non-temporal stores)
    auto nt_memcpy = [](uint8_t* d, const uint8_t* src, size_t w) {
        size_t i = 0;
        while (i < w && (reinterpret_cast<uintptr_t>(d + i) & 31u)) { d[i] = src[i]; ++i; }
        for (; i + 32 <= w; i += 32)
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
        for (; i < w; ++i) d[i] = src[i];
    };
    auto copy_in = [&](size_t off, size_t w) {
        for (int j = 0; j < K; ++j) {
            if (nt_copy) nt_memcpy(st_in + j * SPAN + off, msg.data() + j * S + off, w);
            else std::memcpy(st_in + j * SPAN + off, msg.data() + j * S + off, w);
        }
        if (nt_copy) _mm_sfence();
    };
    auto copy_out = [&](size_t off, size_t w) {
        for (int t = 0; t < M; ++t) std::memcpy(rows.data() + t * S + off, st_out + t * SPAN + off, w);
    };
    auto serial = [&] {
        copy_in(0, S);
        launch(0, NBLK, false, 1);
        CK(hipEventRecord(fin, s));
        CK(wait(fin));
        copy_out(0, S);
    };
    auto chunks2 = [&] {
        const uint32_t b1 = NBLK / 2;
        const size_t o1 = size_t(b1) * 4096;
        copy_in(0, o1);
        launch(0, b1, false, 1);
        CK(hipEventRecord(ev[0], s));
        copy_in(o1, S - o1);
        launch(b1, NBLK - b1, false, 1);
        CK(hipEventRecord(ev[1], s));
        CK(wait(ev[0]));
        copy_out(0, o1);
        CK(wait(ev[1]));
        copy_out(o1, S - o1);
    };
    auto flagged = [&](uint32_t bpf) {
        ++gen;
        launch(0, NBLK, true, bpf);
        CK(hipEventRecord(fin, s));
        const uint32_t ng = (NBLK + bpf - 1) / bpf;
        for (uint32_t g = 0; g < ng; ++g) {
            const size_t off = size_t(g) * bpf * 4096, w = std::min(S, off + size_t(bpf) * 4096) - off;
            copy_in(off, w);
            std::atomic_thread_fence(std::memory_order_seq_cst);
            __atomic_store_n(ready + g, gen, __ATOMIC_RELEASE);
        }
        for (uint32_t g = 0; g < ng; ++g) {
            const uint32_t b0 = g * bpf, b1 = std::min(NBLK, b0 + bpf);
            for (uint32_t b = b0; b < b1; ++b) {
                uint32_t v;
                long spins = 0;
                while ((v = __atomic_load_n(done + b, __ATOMIC_ACQUIRE)) != gen && v != ~gen) {
                    __builtin_ia32_pause();
                    if (++spins == 200000000L) {
                        fprintf(stderr, "host gave up on block %u\n", b);
                        exit(3);
                    }
                }
                if (v == ~gen) ++timeouts;
            }
            const size_t off = size_t(g) * bpf * 4096, w = std::min(S, off + size_t(bpf) * 4096) - off;
            copy_out(off, w);
        }
    };
    auto time_mode = [&](const char* name, auto fn) {
        std::vector<double> t;
        bool ok = true;
        for (int r = 0; r < 330; ++r) {
            std::memset(rows.data(), 0, rows.size());
            const auto t0 = std::chrono::steady_clock::now();
            fn();
            const auto t1 = std::chrono::steady_clock::now();
            ok &= rows == want;
            if (r >= 30) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        CK(hipStreamSynchronize(s));
        std::sort(t.begin(), t.end());
        printf("%-12s median %7.1f us  p10 %7.1f  p90 %7.1f  %s\n", name, t[t.size() / 2], t[t.size() / 10],
               t[t.size() * 9 / 10], ok ? "ok" : "MISMATCH");
        fflush(stdout);
    };
    // one-core memcpy yardstick
    {
        std::vector<uint8_t> a(K * S), b(K * S, 1);
        std::vector<double> t;
        for (int r = 0; r < 200; ++r) {
            const auto t0 = std::chrono::steady_clock::now();
            std::memcpy(a.data(), b.data(), a.size());
            const auto t1 = std::chrono::steady_clock::now();
            t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("memcpy 1 MiB pageable->pageable median %.1f us\n", t[t.size() / 2]);
    }
    {  // launch latency as the host sees it
        uint32_t* f = flags + 2048;
        uint32_t* df = static_cast<uint32_t*>(d_flags) + 2048;
        std::vector<double> tc, ts, te, tq;
        for (uint32_t r = 1; r <= 220; ++r) {
            using clk = std::chrono::steady_clock;
            const auto t0 = clk::now();
            hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, s, df, r);
            CK(hipEventRecord(fin, s));
            const auto t1 = clk::now();
            while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != r) __builtin_ia32_pause();
            const auto t2 = clk::now();
            while (__atomic_load_n(f + 1, __ATOMIC_ACQUIRE) != r) __builtin_ia32_pause();
            const auto t3 = clk::now();
            CK(wait(fin));
            const auto t4 = clk::now();
            if (r > 20) {
                tc.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                ts.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
                te.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
                tq.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
            }
        }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        printf("launch+record call %.1f us; call start -> kernel's first store seen %.1f us; first -> last store %.1f us; "
               "last store -> event complete %.1f us\n", med(tc), med(ts), med(te), med(tq));
        fflush(stdout);
    }
    {  // the GPU side alone (HIP events around one launch; medians of 200)
        void *dev_in, *dev_out;
        CK(hipMalloc(&dev_in, K * SPAN));
        CK(hipMalloc(&dev_out, M * SPAN));
        CK(hipMemcpy(dev_in, st_in, K * SPAN, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto gpu_time = [&](const char* name, auto fn) {
            std::vector<float> t;
            for (int r = 0; r < 220; ++r) {
                CK(hipEventRecord(e0, s));
                fn();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 20) t.push_back(ms * 1000.f);
            }
            std::sort(t.begin(), t.end());
            printf("gpu %-44s median %6.1f us  p10 %6.1f\n", name, t[t.size() / 2], t[t.size() / 10]);
            fflush(stdout);
        };
        const uint8_t* hin = static_cast<const uint8_t*>(d_in);
        uint8_t* hout = static_cast<uint8_t*>(d_out);
        gpu_time("empty launch", [&] { hipLaunchKernelGGL(code_bt<64>, dim3(0 + 1), dim3(64), 0, s, (const uint8_t*)dev_in, (uint8_t*)dev_out); });
        gpu_time("BT256 (26 blocks) pinned in -> pinned out", [&] { hipLaunchKernelGGL(code_bt<256>, dim3((NCOLS + 255) / 256), dim3(256), 0, s, hin, hout); });
        gpu_time("BT128 pinned in -> pinned out", [&] { hipLaunchKernelGGL(code_bt<128>, dim3((NCOLS + 127) / 128), dim3(128), 0, s, hin, hout); });
        gpu_time("BT64 (103 blocks) pinned in -> pinned out", [&] { hipLaunchKernelGGL(code_bt<64>, dim3((NCOLS + 63) / 64), dim3(64), 0, s, hin, hout); });
        gpu_time("BT256 pinned in -> device out", [&] { hipLaunchKernelGGL(code_bt<256>, dim3((NCOLS + 255) / 256), dim3(256), 0, s, hin, (uint8_t*)dev_out); });
        gpu_time("BT64 pinned in -> device out", [&] { hipLaunchKernelGGL(code_bt<64>, dim3((NCOLS + 63) / 64), dim3(64), 0, s, hin, (uint8_t*)dev_out); });
        gpu_time("BT256 device in -> pinned out", [&] { hipLaunchKernelGGL(code_bt<256>, dim3((NCOLS + 255) / 256), dim3(256), 0, s, (const uint8_t*)dev_in, hout); });
        gpu_time("BT64 device in -> pinned out", [&] { hipLaunchKernelGGL(code_bt<64>, dim3((NCOLS + 63) / 64), dim3(64), 0, s, (const uint8_t*)dev_in, hout); });
        gpu_time("BT256 device in -> device out", [&] { hipLaunchKernelGGL(code_bt<256>, dim3((NCOLS + 255) / 256), dim3(256), 0, s, (const uint8_t*)dev_in, (uint8_t*)dev_out); });
        gpu_time("DMA 1 MiB pinned -> device", [&] { CK(hipMemcpyAsync(dev_in, st_in, K * SPAN, hipMemcpyHostToDevice, s)); });
        gpu_time("DMA 0.4 MiB device -> pinned", [&] { CK(hipMemcpyAsync(st_out, dev_out, M * SPAN, hipMemcpyDeviceToHost, s)); });
        CK(hipFree(dev_in));
        CK(hipFree(dev_out));
    }
    {  // serial, phase by phase
        std::vector<double> a1, a2, a3, a4;
        for (int ntc = 0; ntc < 2; ++ntc) {
            nt_copy = ntc;
            a1.clear(); a2.clear(); a3.clear(); a4.clear();
            for (int r = 0; r < 230; ++r) {
                using clk = std::chrono::steady_clock;
                const auto t0 = clk::now();
                copy_in(0, S);
                const auto t1 = clk::now();
                launch(0, NBLK, false, 1);
                CK(hipEventRecord(fin, s));
                const auto t2 = clk::now();
                CK(wait(fin));
                const auto t3 = clk::now();
                copy_out(0, S);
                const auto t4 = clk::now();
                if (r >= 30) {
                    a1.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                    a2.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
                    a3.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
                    a4.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
                }
            }
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
            printf("serial phases (%s copy): copy in %.1f, launch call %.1f, wait %.1f, copy out %.1f us\n",
                   ntc ? "nt" : "memcpy", med(a1), med(a2), med(a3), med(a4));
            fflush(stdout);
        }
        nt_copy = false;
    }
    for (int rep = 0; rep < 4; ++rep) {
        nt_copy = rep & 1;
        printf("-- staging copy: %s\n", nt_copy ? "non-temporal" : "memcpy");
        time_mode("serial", serial);
        time_mode("chunks2", chunks2);
        for (uint32_t bpf : {1u, 2u, 4u, 7u}) {
            char nm[32];
            snprintf(nm, sizeof nm, "flags/%u", bpf);
            time_mode(nm, [&] { flagged(bpf); });
        }
    }
    printf("blocks %u, flag timeouts %d\n", NBLK, timeouts);
    return 0;
}
