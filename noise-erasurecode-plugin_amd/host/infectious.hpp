// infectious.hpp -- C++ host API over the engine's C ABI (include/rsmi.h)
// with the names and contracts of the github.com/vivint/infectious calls the
// reference plugin makes (/root/reference/main.go:24 import):
//   NewFEC(k, n)                 main.go:73, :248
//   (*FEC).Encode(input, output) main.go:262
//   (*FEC).Decode(dst, shares)   main.go:77
//   Share{Number, Data}, DeepCopy main.go:57-69, :254-258
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

struct rs_ctx;

namespace rsmi_host {

// Go `error`: code is an rs_status value (rsmi.h / rsmi_wire.h), 0 = nil.
struct Status {
    int code = 0;
    std::string msg;
    bool ok() const { return code == 0; }
    static Status Ok() { return {}; }
    static Status Err(int c, std::string m) { return {c, std::move(m)}; }
};

// infectious.Share.  Data is owned here; Encode's callback receives a
// ShareView whose bytes are only valid during the callback (data shares
// alias the input, the parity buffer is reused), hence DeepCopy.
struct Share {
    int Number = 0;
    std::vector<uint8_t> Data;
    Share DeepCopy() const { return *this; }
};

struct ShareView {
    int Number = 0;
    const uint8_t* Data = nullptr;
    size_t Len = 0;
    Share DeepCopy() const { return Share{Number, std::vector<uint8_t>(Data, Data + Len)}; }
};

class FEC {
public:
    ~FEC();
    FEC(const FEC&) = delete;
    FEC& operator=(const FEC&) = delete;

    int Required() const { return k_; }
    int Total() const { return n_; }
    rs_ctx* ctx() const { return ctx_; }

    // Calls output for shares 0..n-1 in order (data shares first).
    Status Encode(const uint8_t* input, size_t len,
                  const std::function<void(const ShareView&)>& output);
    // The parity of many messages of len bytes each in one GPU pass
    // (rs_encode_batch): (*parity)[b] = the m * len / k parity bytes of
    // inputs[b] (rs_encode's layout), (*st)[b] its status.
    Status EncodeBatch(const std::vector<const uint8_t*>& inputs, size_t len,
                       std::vector<std::vector<uint8_t>>* parity, std::vector<Status>* st);
    // Sorts `shares` by Number in place; *dst receives k * len(share) bytes.
    Status Decode(std::vector<uint8_t>* dst, std::vector<Share>& shares);
    // Decode of many messages (same share length) in one GPU pass
    // (rs_decode_batch); (*out)[b] / (*st)[b] per message.
    Status DecodeBatch(std::vector<std::vector<Share>>& msgs, std::vector<std::vector<uint8_t>>* out,
                       std::vector<Status>* st);
    // The same over shares held by shared ownership (the plugin's mempool
    // snapshots, ShardPlugin::Receive): nothing is copied in, and the
    // caller's order is left alone (the pool's order carries no meaning).
    Status DecodeShared(std::vector<uint8_t>* dst, const std::vector<std::shared_ptr<const Share>>& shares);
    Status DecodeBatchShared(const std::vector<std::vector<std::shared_ptr<const Share>>>& msgs,
                             std::vector<std::vector<uint8_t>>* out, std::vector<Status>* st);

private:
    friend Status NewFEC(int k, int n, std::shared_ptr<FEC>* out);
    FEC(int k, int n, rs_ctx* c) : k_(k), n_(n), ctx_(c) {}
    int k_, n_;
    rs_ctx* ctx_;
    std::mutex mu_;                // guards parity_ (a cached FEC is shared between threads)
    std::vector<uint8_t> parity_;  // reused between calls like infectious's fec_buf
};

// infectious.NewFEC: errors with RS_EINVAL_KN unless 1 <= k <= n <= 256.
Status NewFEC(int k, int n, std::shared_ptr<FEC>* out);

// Cached FEC per (k, n): the plugin calls NewFEC for every message
// (main.go:73, :248); the engine's construction uploads tables, so callers on
// a hot path share one per code.
Status CachedFEC(int k, int n, std::shared_ptr<FEC>* out);

std::string StatusText(int code);

}  // namespace rsmi_host
