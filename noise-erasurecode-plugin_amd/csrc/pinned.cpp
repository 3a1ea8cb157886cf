// pinned.cpp -- see pinned.hpp.  rs_pinned_alloc / rs_pinned_free and the
// rs_arena bump allocator of include/rsmi.h.
#include "pinned.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <new>
#include <shared_mutex>

#include "../../include/rsmi.h"
#include "host_pipeline.hpp"

namespace rsmi {
namespace {

struct Range {
    size_t len;
    uint64_t dev;  // device alias of the base (hipHostGetDevicePointer)
};

std::shared_mutex& reg_mu() {
    static std::shared_mutex mu;
    return mu;
}
std::map<uintptr_t, Range>& registry() {
    static std::map<uintptr_t, Range>* r = new std::map<uintptr_t, Range>();  // outlives static dtors
    return *r;
}

void* alloc_registered(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) d = p;
    std::unique_lock<std::shared_mutex> lk(reg_mu());
    registry()[reinterpret_cast<uintptr_t>(p)] = Range{bytes ? bytes : 1, reinterpret_cast<uint64_t>(d)};
    return p;
}

void free_registered(void* p) {
    if (!p) return;
    {
        std::unique_lock<std::shared_mutex> lk(reg_mu());
        registry().erase(reinterpret_cast<uintptr_t>(p));
    }
    (void)hipHostFree(p);
}

}  // namespace

uint64_t pinned_device_address(const void* p, size_t len) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::shared_lock<std::shared_mutex> lk(reg_mu());
    const std::map<uintptr_t, Range>& r = registry();
    auto it = r.upper_bound(a);
    if (it == r.begin()) return 0;
    --it;
    if (a + len > it->first + it->second.len || a + len < a) return 0;
    return it->second.dev + (a - it->first);
}

}  // namespace rsmi

struct rs_arena {
    uint8_t* base = nullptr;
    size_t cap = 0, used = 0;
};

extern "C" {

void* rs_pinned_alloc(size_t bytes) { return rsmi::alloc_registered(bytes); }

void rs_pinned_free(void* p) { rsmi::free_registered(p); }

rs_arena* rs_arena_new(size_t bytes) {
    rs_arena* a = new (std::nothrow) rs_arena;
    if (!a) return nullptr;
    a->base = static_cast<uint8_t*>(rsmi::alloc_registered(bytes));
    if (!a->base) {
        delete a;
        return nullptr;
    }
    a->cap = bytes;
    return a;
}

void* rs_arena_alloc(rs_arena* a, size_t bytes) {
    if (!a) return nullptr;
    // 256-byte slots: every slot is 16-byte aligned and can be read up to the
    // next multiple of 16 (the kernels code round_up(len, 16) bytes).
    const size_t want = (std::max<size_t>(bytes, 1) + 255) & ~size_t(255);
    if (want > a->cap - a->used) return nullptr;
    void* p = a->base + a->used;
    a->used += want;
    return p;
}

void* rs_arena_put(rs_arena* a, const void* data, size_t bytes) {
    if (bytes && !data) return nullptr;
    void* slot = rs_arena_alloc(a, bytes);
    if (slot && bytes) {
        rsmi::stage_copy(slot, data, bytes);
        rsmi::stage_fence();
    }
    return slot;
}

void rs_arena_reset(rs_arena* a) {
    if (a) a->used = 0;
}

size_t rs_arena_used(const rs_arena* a) { return a ? a->used : 0; }

void rs_arena_free(rs_arena* a) {
    if (!a) return;
    rsmi::free_registered(a->base);
    delete a;
}

}  // extern "C"
