// pinned.hpp -- engine-owned pinned host memory (rs_pinned_alloc, rs_arena)
// and the registry that lets a call recognise it without asking the HIP
// runtime about every pointer (hipPointerGetAttributes per shard cost what
// the staging copies saved, profiles/r01e_host_api_pinned_ab.json).
//
// Every range is hipHostMalloc memory mapped for the device, so a kernel can
// read it over PCIe in place: rs_decode_batch hands such survivors to the
// reconstruct kernel through its shard-address table (zero-copy receive,
// SURVEY.md §8f rank 1).
#pragma once

#include <cstddef>
#include <cstdint>

namespace rsmi {

// Device address of host range [p, p + len) if it lies inside one
// registered pinned range, else 0.
uint64_t pinned_device_address(const void* p, size_t len);

}  // namespace rsmi
