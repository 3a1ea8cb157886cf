// stage_copy.cpp -- host copy rates that bound a config-1 message's host
// path (host_pipeline.cpp stage_copy): 512 KiB pageable -> pinned
// (hipHostMalloc) with memcpy, SSE / AVX2 / AVX-512 non-temporal stores, and
// 800 KiB pageable -> pageable memcpy (the present shares into dst); medians
// of 2000 reps, one thread, sources warm like a just-received message.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__attribute__((target("sse2"))) static void nt_sse(void* d, const void* s, size_t n) {
    for (size_t i = 0; i < n; i += 64)
        for (int j = 0; j < 4; ++j)
            _mm_stream_si128((__m128i*)((char*)d + i) + j, _mm_loadu_si128((const __m128i*)((const char*)s + i) + j));
    _mm_sfence();
}
__attribute__((target("avx2"))) static void nt_avx2(void* d, const void* s, size_t n) {
    for (size_t i = 0; i < n; i += 64) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)((const char*)s + i));
        const __m256i b = _mm256_loadu_si256((const __m256i*)((const char*)s + i + 32));
        _mm256_stream_si256((__m256i*)((char*)d + i), a);
        _mm256_stream_si256((__m256i*)((char*)d + i + 32), b);
    }
    _mm_sfence();
}
__attribute__((target("avx512f"))) static void nt_avx512(void* d, const void* s, size_t n) {
    for (size_t i = 0; i < n; i += 64) _mm512_stream_si512((__m512i*)((char*)d + i), _mm512_loadu_si512((const char*)s + i));
    _mm_sfence();
}

template <class F>
static double med_us(F f) {
    std::vector<double> t;
    for (int r = 0; r < 2000; ++r) {
        const auto a = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t n = 512 << 10, p = 800 << 10;
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    // 64-byte aligned (the streaming stores need aligned destinations)
    char* srcp = static_cast<char*>(std::aligned_alloc(4096, 2 << 20));
    char* dstp = static_cast<char*>(std::aligned_alloc(4096, 2 << 20));
    std::memset(srcp, 1, 2 << 20);
    std::memset(dstp, 2, 2 << 20);
    struct Buf { char* p; char* data() { return p; } } src{srcp}, dst{dstp};
    void* pin = nullptr;
    if (hipHostMalloc(&pin, 2 << 20, hipHostMallocDefault) != hipSuccess) return 1;
    std::memset(pin, 0, 2 << 20);
    std::printf("pageable->pinned 512 KiB: memcpy %.2f us\n", med_us([&] { std::memcpy(pin, src.data(), n); }));
    std::printf("pageable->pinned 512 KiB: nt sse %.2f us\n", med_us([&] { nt_sse(pin, src.data(), n); }));
    std::printf("pageable->pinned 512 KiB: nt avx2 %.2f us\n", med_us([&] { nt_avx2(pin, src.data(), n); }));
    if (__builtin_cpu_supports("avx512f"))
        std::printf("pageable->pinned 512 KiB: nt avx512 %.2f us\n", med_us([&] { nt_avx512(pin, src.data(), n); }));
    std::printf("pageable->pageable 800 KiB: memcpy %.2f us\n", med_us([&] { std::memcpy(dst.data(), src.data() + (1 << 20), p); }));
    std::printf("pageable->pageable 800 KiB: nt avx2 %.2f us\n", med_us([&] { nt_avx2(dst.data(), src.data() + (1 << 20), p); }));
    std::printf("pinned->pageable 200 KiB: memcpy %.2f us (pinned not written by a GPU here: cached)\n",
                med_us([&] { std::memcpy(dst.data(), pin, 200 << 10); }));
    (void)hipHostFree(pin);
    return 0;
}
