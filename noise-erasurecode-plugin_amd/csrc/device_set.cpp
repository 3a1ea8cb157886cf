// device_set.cpp -- rs_new_devices: one context over several GPUs (see
// device_set.hpp).  Members are single-device contexts driven through the
// public C ABI; this file only decides which member does what and runs the
// members' parts concurrently, one host worker thread per member.
#include "device_set.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

namespace rsmi {

namespace {

// A member's host thread: runs the member's part of a set call (the
// members' parts of one call run at once, each thread issuing its own
// device's work -- SURVEY.md §7.5 "one host thread + stream per GPU").
class Worker {
public:
    Worker() : th_([this] { loop(); }) {}
    ~Worker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(f));
        }
        cv_.notify_one();
    }

private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;  // stop_ with nothing left
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace

struct DeviceSet {
    std::vector<rs_ctx*> members;
    std::vector<int> devices;
    std::vector<std::unique_ptr<Worker>> workers;  // [0] unused: member 0 runs on the caller
    std::unique_ptr<std::atomic<int>[]> inflight;
    std::atomic<unsigned> rotate{0};
    bool peer_ok = true;  // every pair of distinct member devices has peer access
};

int set_create(int k, int n, const int* devices, int count, DeviceSet** out) {
    *out = nullptr;
    if (!devices || count <= 0 || count > 256) return RS_EINVAL;
    std::unique_ptr<DeviceSet> s(new (std::nothrow) DeviceSet);
    if (!s) return RS_ENOMEM;
    s->inflight.reset(new (std::nothrow) std::atomic<int>[count]);
    if (!s->inflight) return RS_ENOMEM;
    for (int i = 0; i < count; ++i) s->inflight[i].store(0);
    for (int i = 0; i < count; ++i) {
        rs_ctx* c = nullptr;
        const int st = rs_new_on_device(k, n, devices[i], &c);
        if (st != RS_OK) {
            for (rs_ctx* m : s->members) rs_free(m);  // not yet marked as members
            return st;
        }
        s->members.push_back(c);
        s->devices.push_back(devices[i]);
    }
    // Peer access between distinct member devices: the shard-distributed
    // reconstruct reads survivors (and writes erased shards) in peer HBM.
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    for (int a : s->devices)
        for (int b : s->devices) {
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
                s->peer_ok = false;
                continue;
            }
            if (hipSetDevice(a) != hipSuccess) {
                s->peer_ok = false;
                continue;
            }
            const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
            if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            else if (e != hipSuccess) s->peer_ok = false;
        }
    if (prev >= 0) (void)hipSetDevice(prev);
    s->workers.resize(count);
    for (int i = 1; i < count; ++i) {
        s->workers[i].reset(new (std::nothrow) Worker);
        if (!s->workers[i]) {
            set_destroy(s.release());
            return RS_ENOMEM;
        }
    }
    *out = s.release();
    return RS_OK;
}

void set_destroy(DeviceSet* s) {
    if (!s) return;
    s->workers.clear();  // joins: no member work in flight on them
    for (rs_ctx* m : s->members) member_free(m);
    delete s;
}

int set_count(const DeviceSet* s) { return static_cast<int>(s->members.size()); }
rs_ctx* set_member(const DeviceSet* s, int i) {
    return i >= 0 && i < set_count(s) ? s->members[static_cast<size_t>(i)] : nullptr;
}
int set_device(const DeviceSet* s, int i) { return s->devices[static_cast<size_t>(i)]; }
bool set_peer_ok(const DeviceSet* s) { return s->peer_ok; }

namespace {
// Least busy member among those accepted by `ok`, ties rotating.
template <class Ok>
int pick(DeviceSet* s, Ok ok) {
    const int cnt = set_count(s);
    const unsigned r = s->rotate.fetch_add(1, std::memory_order_relaxed);
    int best = -1, best_load = 0;
    for (int j = 0; j < cnt; ++j) {
        const int i = static_cast<int>((r + static_cast<unsigned>(j)) % static_cast<unsigned>(cnt));
        if (!ok(i)) continue;
        const int load = s->inflight[i].load(std::memory_order_relaxed);
        if (best < 0 || load < best_load) {
            best = i;
            best_load = load;
        }
    }
    return best;
}
}  // namespace

int set_acquire(DeviceSet* s) {
    const int i = pick(s, [](int) { return true; });
    s->inflight[i].fetch_add(1, std::memory_order_relaxed);
    return i;
}

void set_release(DeviceSet* s, int member) { s->inflight[member].fetch_sub(1, std::memory_order_relaxed); }

int set_route(DeviceSet* s, const void* p) {
    hipPointerAttribute_t attr{};
    if (!p || hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;  // pageable host memory: no device owns it
    }
    if (attr.type != hipMemoryTypeDevice && attr.type != hipMemoryTypeArray) return 0;  // mapped host memory
    const int dev = attr.device;
    return pick(s, [&](int i) { return s->devices[static_cast<size_t>(i)] == dev; });
}

int set_run(DeviceSet* s, const std::function<int(int)>& job) {
    const int cnt = set_count(s);
    auto guarded = [&](int i) -> int {
        try {
            return job(i);
        } catch (const std::bad_alloc&) {
            return RS_ENOMEM;
        }
    };
    if (cnt == 1) return guarded(0);
    std::vector<int> rc(static_cast<size_t>(cnt), RS_OK);
    std::mutex mu;
    std::condition_variable cv;
    int left = cnt - 1;
    for (int i = 1; i < cnt; ++i)
        s->workers[static_cast<size_t>(i)]->post([&, i] {
            const int r = guarded(i);
            std::lock_guard<std::mutex> lk(mu);
            rc[static_cast<size_t>(i)] = r;
            --left;
            cv.notify_one();  // under the lock: the waiter may return (and destroy cv) once it sees left == 0
        });
    rc[0] = guarded(0);
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
    for (int r : rc)
        if (r != RS_OK) return r;
    return RS_OK;
}

int set_encode_batch(DeviceSet* s, int batch, const uint8_t* const* inputs, size_t len, uint8_t* const* parities,
                     int* status) {
    const int cnt = set_count(s);
    (void)set_run(s, [&](int i) -> int {
        size_t b0 = 0, nb = 0;
        (void)rs_partition(static_cast<size_t>(batch), cnt, i, &b0, &nb);
        if (!nb) return RS_OK;
        return rs_encode_batch(s->members[static_cast<size_t>(i)], static_cast<int>(nb), inputs + b0, len,
                               parities + b0, status + b0);
    });
    for (int b = 0; b < batch; ++b)  // the first failing status in message order
        if (status[b] != RS_OK) return status[b];
    return RS_OK;
}

int set_decode_batch(DeviceSet* s, int batch, const int* counts, int* numbers, const uint8_t** shares, size_t S,
                     uint8_t** dsts, int* status) {
    const int cnt = set_count(s);
    // Offsets of each message's shares in numbers[] / shares[].
    std::vector<size_t> first(static_cast<size_t>(batch) + 1, 0);
    for (int b = 0; b < batch; ++b) first[b + 1] = first[b] + static_cast<size_t>(std::max(counts[b], 0));
    (void)set_run(s, [&](int i) -> int {
        size_t b0 = 0, nb = 0;
        (void)rs_partition(static_cast<size_t>(batch), cnt, i, &b0, &nb);
        if (!nb) return RS_OK;
        return rs_decode_batch(s->members[static_cast<size_t>(i)], static_cast<int>(nb), counts + b0,
                               numbers + first[b0], shares + first[b0], S, dsts + b0, status + b0);
    });
    for (int b = 0; b < batch; ++b)
        if (status[b] != RS_OK) return status[b];
    return RS_OK;
}

}  // namespace rsmi
