// copypool_stress.cpp -- the shared host copy pool (csrc/host_pipeline.cpp,
// CopyPool::shared) under concurrent callers, built with ThreadSanitizer and
// AddressSanitizer on the host (GPU sanitizers are not available; the pool
// itself makes no HIP calls, so this runs on a CPU-only machine).
//
// Eight caller threads each submit random piece lists -- many small pieces,
// a few multi-MiB ones that the pool splits into parts -- at the same time,
// the way concurrent rs_encode/rs_decode/rs_decode_batch calls on one context
// (or on several contexts in one process) share the pool.  Every destination
// must equal its source byte for byte (starts misaligned on both sides, half
// the pieces through the non-temporal staging copy, guard bytes untouched);
// the sanitizers flag any data race on the job queue or out-of-bounds part
// split or copy.  Half the submissions are asynchronous jobs (start /
// finish, two in flight per caller) with the workers' spin window on or off.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "host_pipeline.hpp"

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
    const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
    rsmi::CopyPool& pool = rsmi::CopyPool::shared();
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            std::mt19937 rng(1234 + t);
            for (int it = 0; it < iters; ++it) {
                const int np = 1 + static_cast<int>(rng() % 64);
                std::vector<std::vector<unsigned char>> src(np), dst(np);
                std::vector<size_t> lens(np), soff(np), doff(np);
                std::vector<rsmi::CopyPool::Piece> pieces;
                for (int i = 0; i < np; ++i) {
                    const size_t len = rng() % 3 == 0 ? rng() % (3u << 20) : rng() % 70000;
                    // misaligned starts on both sides (the non-temporal copy's
                    // head / body / tail split), 32 guard bytes past the end
                    lens[i] = len;
                    soff[i] = rng() % 16;
                    doff[i] = rng() % 16;
                    src[i].resize(len + soff[i]);
                    for (size_t j = 0; j < src[i].size(); j += 997) src[i][j] = static_cast<unsigned char>(rng());
                    dst[i].assign(len + doff[i] + 32, 0xA5);
                    const bool nt = rng() % 2 == 0;  // staging-bound pieces (stage_copy + fence)
                    pieces.push_back({dst[i].data() + doff[i], src[i].data() + soff[i], len, nt});
                }
                // Odd iterations go through the asynchronous jobs (start, other
                // work, finish) that a single message's decode uses: two jobs in
                // flight at once, joined in either order.
                if (it % 2 == 0) {
                    pool.run(pieces);
                } else {
                    const size_t half = pieces.size() / 2;
                    std::vector<rsmi::CopyPool::Piece> a(pieces.begin(), pieces.begin() + half),
                        b(pieces.begin() + half, pieces.end());
                    rsmi::CopyPool::Async* ja = pool.start(a, 1 + rng() % (256u << 10));
                    rsmi::CopyPool::Async* jb = pool.start(b, 1 + rng() % (256u << 10));
                    if (rng() % 2) {
                        pool.finish(jb);
                        pool.finish(ja);
                    } else {
                        pool.finish(ja);
                        pool.finish(jb);
                    }
                }
                for (int i = 0; i < np; ++i) {
                    bool ok = std::equal(src[i].begin() + soff[i], src[i].end(), dst[i].begin() + doff[i]);
                    for (size_t j = 0; j < doff[i]; ++j) ok &= dst[i][j] == 0xA5;
                    for (size_t j = doff[i] + lens[i]; j < dst[i].size(); ++j) ok &= dst[i][j] == 0xA5;
                    if (!ok) bad.fetch_add(1);
                }
            }
        });
    for (auto& x : th) x.join();
    std::printf("copypool_stress: %s (%d mismatches, %d threads x %d submissions)\n",
                bad.load() ? "FAILED" : "ok", bad.load(), threads, iters);
    return bad.load() ? 1 : 0;
}
