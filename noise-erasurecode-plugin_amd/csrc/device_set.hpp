// device_set.hpp -- a context over several GPUs (rs_new_devices, rsmi.h):
// north_star's stripe partition over the 8 GPUs of one node, behind the same
// C ABI the plugin's cgo shim calls.  A set owns one ordinary single-device
// context per member and one host worker thread per member; the entry points
// of rsmi.cpp forward a set context here, and everything below calls the
// members through the public C ABI -- the set adds no device code of its own.
//
// Placement rules:
//  - stripe-local (the headline): stripes / messages are split into
//    contiguous ranges, one per member, no collective;
//  - shard-distributed: the owner's reconstruct kernel reads its survivors
//    over xGMI where they lie (peer access), rs_reconstruct_spread.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>

#include "../../include/rsmi.h"

namespace rsmi {

struct DeviceSet;

// Members are created with rs_new_on_device; peer access is enabled between
// distinct member devices.  Returns an rs_status.
int set_create(int k, int n, const int* devices, int count, DeviceSet** out);
void set_destroy(DeviceSet* s);
// Frees a member context (rsmi.cpp; rs_free itself ignores a set's members).
void member_free(rs_ctx* c);

int set_count(const DeviceSet* s);
rs_ctx* set_member(const DeviceSet* s, int i);
int set_device(const DeviceSet* s, int i);
bool set_peer_ok(const DeviceSet* s);

// The member with the fewest calls in flight (ties rotate); the caller holds
// it until the matching set_release.
int set_acquire(DeviceSet* s);
void set_release(DeviceSet* s, int member);

// A member on the device that holds device (or mapped host) address p: the
// least busy of them; -1 if no member is on that device.  Host memory
// (pinned, mapped) routes to member 0.
int set_route(DeviceSet* s, const void* p);

// Runs job(i) for every member i at once -- member 0 on the calling thread,
// the others on their worker threads -- and returns the first failing status
// in member order (RS_OK if all succeed).  job(i) may skip a member by
// returning RS_OK.
int set_run(DeviceSet* s, const std::function<int(int)>& job);

// Batched host API over the set: messages in contiguous ranges per member.
int set_encode_batch(DeviceSet* s, int batch, const uint8_t* const* inputs, size_t len, uint8_t* const* parities,
                     int* status);
int set_decode_batch(DeviceSet* s, int batch, const int* counts, int* numbers, const uint8_t** shares, size_t S,
                     uint8_t** dsts, int* status);

}  // namespace rsmi
