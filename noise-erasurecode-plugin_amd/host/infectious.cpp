// infectious.cpp -- see infectious.hpp.
#include "infectious.hpp"

#include <algorithm>
#include <map>
#include <mutex>

#include "../../include/rsmi.h"

namespace rsmi_host {

std::string StatusText(int code) { return rs_strerror(code); }

static Status from(int code, const char* what) {
    if (code == RS_OK) return Status::Ok();
    return Status::Err(code, std::string(what) + ": " + rs_strerror(code));
}

FEC::~FEC() {
    if (ctx_) rs_free(ctx_);
}

Status NewFEC(int k, int n, std::shared_ptr<FEC>* out) {
    rs_ctx* c = nullptr;
    const int rc = rs_new(k, n, &c);
    if (rc != RS_OK) return from(rc, "NewFEC");
    out->reset(new FEC(k, n, c));
    return Status::Ok();
}

Status CachedFEC(int k, int n, std::shared_ptr<FEC>* out) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::shared_ptr<FEC>> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({k, n});
    if (it != cache.end()) {
        *out = it->second;
        return Status::Ok();
    }
    Status st = NewFEC(k, n, out);
    if (st.ok()) cache[{k, n}] = *out;
    return st;
}

Status FEC::Encode(const uint8_t* input, size_t len,
                   const std::function<void(const ShareView&)>& output) {
    if (len % static_cast<size_t>(k_) != 0)
        return from(RS_ELEN_NOT_MULTIPLE, "Encode");
    const size_t S = len / static_cast<size_t>(k_);
    const int m = n_ - k_;
    std::lock_guard<std::mutex> lk(mu_);
    parity_.resize(static_cast<size_t>(m) * S);
    if (S && m) {
        const int rc = rs_encode(ctx_, input, len, parity_.data());
        if (rc != RS_OK) return from(rc, "Encode");
    }
    for (int i = 0; i < k_; ++i) output(ShareView{i, input + static_cast<size_t>(i) * S, S});
    for (int i = 0; i < m; ++i) output(ShareView{k_ + i, parity_.data() + static_cast<size_t>(i) * S, S});
    return Status::Ok();
}

Status FEC::EncodeBatch(const std::vector<const uint8_t*>& inputs, size_t len,
                        std::vector<std::vector<uint8_t>>* parity, std::vector<Status>* st) {
    const int B = static_cast<int>(inputs.size());
    parity->assign(B, {});
    st->assign(B, Status::Ok());
    if (B == 0) return Status::Ok();
    const size_t P = len % static_cast<size_t>(k_) == 0 ? len / static_cast<size_t>(k_) * (n_ - k_) : 0;
    std::vector<uint8_t*> outs(B);
    for (int b = 0; b < B; ++b) {
        (*parity)[b].resize(P);
        outs[b] = (*parity)[b].data();
    }
    std::vector<int> codes(B, RS_OK);
    const int rc = rs_encode_batch(ctx_, B, inputs.data(), len, outs.data(), codes.data());
    for (int b = 0; b < B; ++b)
        if (codes[b] != RS_OK) {
            (*st)[b] = from(codes[b], "Encode");
            (*parity)[b].clear();
        }
    return rc == RS_OK ? Status::Ok() : from(rc, "EncodeBatch");
}

Status FEC::Decode(std::vector<uint8_t>* dst, std::vector<Share>& shares) {
    const int cnt = static_cast<int>(shares.size());
    const size_t S = cnt ? shares[0].Data.size() : 0;
    for (const Share& s : shares)
        if (s.Data.size() != S) return from(RS_ESHARE_LEN, "Decode");
    std::vector<int> nums(cnt);
    std::vector<const uint8_t*> ptrs(cnt);
    for (int i = 0; i < cnt; ++i) {
        nums[i] = shares[i].Number;
        ptrs[i] = shares[i].Data.data();
    }
    std::vector<uint8_t> out(static_cast<size_t>(k_) * S);
    const int rc = rs_decode(ctx_, nums.data(), ptrs.data(), cnt, S, out.data());
    if (rc != RS_OK) return from(rc, "Decode");
    // mirror infectious's in-place sort of the caller's slice
    std::stable_sort(shares.begin(), shares.end(),
                     [](const Share& a, const Share& b) { return a.Number < b.Number; });
    *dst = std::move(out);
    return Status::Ok();
}

Status FEC::DecodeBatch(std::vector<std::vector<Share>>& msgs, std::vector<std::vector<uint8_t>>* out,
                        std::vector<Status>* st) {
    const int B = static_cast<int>(msgs.size());
    out->assign(B, {});
    st->assign(B, Status::Ok());
    if (B == 0) return Status::Ok();
    const size_t S = msgs[0].empty() ? 0 : msgs[0][0].Data.size();
    std::vector<int> counts(B), nums;
    std::vector<const uint8_t*> ptrs;
    for (int b = 0; b < B; ++b) {
        counts[b] = static_cast<int>(msgs[b].size());
        for (const Share& s : msgs[b]) {
            if (s.Data.size() != S) return from(RS_ESHARE_LEN, "DecodeBatch");
            nums.push_back(s.Number);
            ptrs.push_back(s.Data.data());
        }
    }
    std::vector<uint8_t*> dsts(B);
    for (int b = 0; b < B; ++b) {
        (*out)[b].resize(static_cast<size_t>(k_) * S);
        dsts[b] = (*out)[b].data();
    }
    std::vector<int> codes(B, 0);
    const int rc = rs_decode_batch(ctx_, B, counts.data(), nums.data(), ptrs.data(), S, dsts.data(),
                                   codes.data());
    for (int b = 0; b < B; ++b) {
        if (codes[b] != RS_OK) {
            (*st)[b] = from(codes[b], "Decode");
            (*out)[b].clear();
        }
        std::stable_sort(msgs[b].begin(), msgs[b].end(),
                         [](const Share& x, const Share& y) { return x.Number < y.Number; });
    }
    return rc == RS_OK ? Status::Ok() : from(rc, "DecodeBatch");
}

Status FEC::DecodeShared(std::vector<uint8_t>* dst, const std::vector<std::shared_ptr<const Share>>& shares) {
    const int cnt = static_cast<int>(shares.size());
    const size_t S = cnt ? shares[0]->Data.size() : 0;
    std::vector<int> nums(cnt);
    std::vector<const uint8_t*> ptrs(cnt);
    for (int i = 0; i < cnt; ++i) {
        if (shares[i]->Data.size() != S) return from(RS_ESHARE_LEN, "Decode");
        nums[i] = shares[i]->Number;
        ptrs[i] = shares[i]->Data.data();
    }
    // Decoded straight into the caller's vector: a caller that reuses it
    // (a receive loop's ReceiveEvent) reuses its capacity -- no fresh 1 MiB
    // allocation and zero-fill per message.
    dst->resize(static_cast<size_t>(k_) * S);
    const int rc = rs_decode(ctx_, nums.data(), ptrs.data(), cnt, S, dst->data());
    if (rc != RS_OK) {
        dst->clear();
        return from(rc, "Decode");
    }
    return Status::Ok();
}

Status FEC::DecodeBatchShared(const std::vector<std::vector<std::shared_ptr<const Share>>>& msgs,
                              std::vector<std::vector<uint8_t>>* out, std::vector<Status>* st) {
    const int B = static_cast<int>(msgs.size());
    out->assign(B, {});
    st->assign(B, Status::Ok());
    if (B == 0) return Status::Ok();
    const size_t S = msgs[0].empty() ? 0 : msgs[0][0]->Data.size();
    std::vector<int> counts(B), nums;
    std::vector<const uint8_t*> ptrs;
    for (int b = 0; b < B; ++b) {
        counts[b] = static_cast<int>(msgs[b].size());
        for (const std::shared_ptr<const Share>& s : msgs[b]) {
            if (s->Data.size() != S) return from(RS_ESHARE_LEN, "DecodeBatch");
            nums.push_back(s->Number);
            ptrs.push_back(s->Data.data());
        }
    }
    std::vector<uint8_t*> dsts(B);
    for (int b = 0; b < B; ++b) {
        (*out)[b].resize(static_cast<size_t>(k_) * S);
        dsts[b] = (*out)[b].data();
    }
    std::vector<int> codes(B, 0);
    const int rc = rs_decode_batch(ctx_, B, counts.data(), nums.data(), ptrs.data(), S, dsts.data(),
                                   codes.data());
    for (int b = 0; b < B; ++b)
        if (codes[b] != RS_OK) {
            (*st)[b] = from(codes[b], "Decode");
            (*out)[b].clear();
        }
    return rc == RS_OK ? Status::Ok() : from(rc, "DecodeBatch");
}

}  // namespace rsmi_host
