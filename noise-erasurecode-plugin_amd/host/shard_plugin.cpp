// shard_plugin.cpp -- see shard_plugin.hpp.
#include "shard_plugin.hpp"

#include <algorithm>
#include <future>
#include <map>
#include <tuple>

#include "../../include/rsmi.h"
#include "../../include/rsmi_wire.h"

namespace rsmi_host {

// ---------------------------------------------------------------- Shard ----
static rs_shard_view view_of(const Shard& s) {
    rs_shard_view v{};
    v.file_signature = s.FileSignature.data();
    v.file_signature_len = s.FileSignature.size();
    v.shard_data = s.ShardData.data();
    v.shard_data_len = s.ShardData.size();
    v.shard_number = s.ShardNumber;
    v.total_shards = s.TotalShards;
    v.minimum_needed_shards = s.MinimumNeededShards;
    return v;
}

size_t Shard::Size() const {
    const rs_shard_view v = view_of(*this);
    return rs_shard_size(&v);
}

std::vector<uint8_t> Shard::Marshal() const {
    const rs_shard_view v = view_of(*this);
    std::vector<uint8_t> out(rs_shard_size(&v));
    size_t w = 0;
    rs_shard_marshal(&v, out.data(), out.size(), &w);
    out.resize(w);
    return out;
}

Status Shard::Unmarshal(const uint8_t* data, size_t len) {
    rs_shard_view v{};
    const int rc = rs_shard_unmarshal(data, len, &v);
    if (rc != 0) {
        const char* what = rc == RS_EWIRE_EOF        ? "unexpected EOF"
                           : rc == RS_EWIRE_OVERFLOW ? "proto: integer overflow"
                           : rc == RS_EWIRE_LENGTH   ? "proto: negative length found during unmarshaling"
                                                     : "proto: Shard: bad wire type or tag";
        return Status::Err(rc, what);
    }
    FileSignature.assign(v.file_signature, v.file_signature + v.file_signature_len);
    ShardData.assign(v.shard_data, v.shard_data + v.shard_data_len);
    ShardNumber = v.shard_number;
    TotalShards = v.total_shards;
    MinimumNeededShards = v.minimum_needed_shards;
    return Status::Ok();
}

// ---------------------------------------------------------------- helpers --
std::vector<uint8_t> serializeMessage(const PeerID& id, const std::vector<uint8_t>& message) {
    std::vector<uint8_t> out;
    out.reserve(8 + id.Address.size() + id.Id.size() + message.size());
    auto put32 = [&](uint32_t v) {
        for (int i = 0; i < 4; ++i) out.push_back(static_cast<uint8_t>(v >> (8 * i)));
    };
    put32(static_cast<uint32_t>(id.Address.size()));
    out.insert(out.end(), id.Address.begin(), id.Address.end());
    put32(static_cast<uint32_t>(id.Id.size()));
    out.insert(out.end(), id.Id.begin(), id.Id.end());
    out.insert(out.end(), message.begin(), message.end());
    return out;
}

int largestPrimeFactors(int n) {
    int result = -1;
    while (n > 0 && n % 2 == 0) {
        result = 2;
        n /= 2;
    }
    for (int i = 3; i * i <= n; i += 2)
        while (n % i == 0) {
            result = std::max(result, i);
            n /= i;
        }
    if (n > 2) result = std::max(result, n);
    return result;
}

std::string HexString(const std::vector<uint8_t>& b) {
    static const char* d = "0123456789abcdef";
    std::string s(b.size() * 2, '0');
    for (size_t i = 0; i < b.size(); ++i) {
        s[2 * i] = d[b[i] >> 4];
        s[2 * i + 1] = d[b[i] & 15];
    }
    return s;
}

// ----------------------------------------------------------- ShardPlugin ---
ShardPlugin::ShardPlugin(int k, int n, Signer sign, Verifier verify, int hashLen)
    : MinimumNeededShards(k), TotalShards(n), HashLen(hashLen), sign_(std::move(sign)), verify_(std::move(verify)) {}

std::unique_ptr<ShardPlugin> NewShardPlugin(Signer sign, Verifier verify, int k, int n, int hashLen) {
    return std::make_unique<ShardPlugin>(k, n, std::move(sign), std::move(verify), hashLen);
}

Status ShardPlugin::HashBytes(const std::vector<std::vector<uint8_t>>& msgs,
                              std::vector<std::vector<uint8_t>>* out) const {
    if (HashLen <= 0) {
        *out = msgs;
        return Status::Ok();
    }
    out->assign(msgs.size(), std::vector<uint8_t>(static_cast<size_t>(HashLen)));
    if (msgs.empty()) return Status::Ok();
    // Any context on the device serves the hash; use this plugin's code.
    std::shared_ptr<FEC> f;
    Status st = CachedFEC(MinimumNeededShards, TotalShards, &f);
    if (!st.ok()) return st;
    std::vector<const uint8_t*> ptrs(msgs.size());
    std::vector<size_t> lens(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) {
        ptrs[i] = msgs[i].data();
        lens[i] = msgs[i].size();
    }
    std::vector<uint8_t> dig(msgs.size() * static_cast<size_t>(HashLen));
    // The engine's policy: host CPU for one message or a batch whose longest
    // chain dominates, the GPU kernel for many messages in flight.
    const int rc = rs_blake2b(f->ctx(), static_cast<int>(msgs.size()), ptrs.data(), lens.data(), HashLen,
                              dig.data(), nullptr);
    if (rc != RS_OK) return Status::Err(rc, std::string("blake2b: ") + rs_strerror(rc));
    for (size_t i = 0; i < msgs.size(); ++i)
        std::copy(dig.begin() + i * HashLen, dig.begin() + (i + 1) * HashLen, (*out)[i].begin());
    return Status::Ok();
}

size_t ShardPlugin::PoolSize(const std::vector<uint8_t>& sig) const {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = shards_.find(HexString(sig));
    return it == shards_.end() ? 0 : it->second.size();
}

Status ShardPlugin::shardInput(const std::vector<uint8_t>& input, std::vector<Share>* out) {
    std::shared_ptr<FEC> f;
    Status st = CachedFEC(MinimumNeededShards, TotalShards, &f);
    if (!st.ok()) return st;
    std::vector<Share> shares(static_cast<size_t>(TotalShards));
    st = f->Encode(input.data(), input.size(), [&](const ShareView& s) {
        shares[static_cast<size_t>(s.Number)] = s.DeepCopy();  // main.go:255-258
    });
    if (!st.ok()) return st;
    *out = std::move(shares);
    return Status::Ok();
}

// The signature hash (main.go:219-223) and the encode (main.go:225) are
// independent: a helper thread hashes (one message: host CPU, no HIP calls)
// while this thread, whose HIP state is warm, drives the GPU encode, so the
// call costs about the longer of the two, not their sum.  The signer itself
// runs here, after both.
Status ShardPlugin::sign_input(const PeerID& self, const std::vector<uint8_t>& input, std::vector<uint8_t>* sig,
                               const std::function<Status()>& encode) {
    std::vector<std::vector<uint8_t>> h;
    std::future<Status> hashed;
    if (sign_) {
        std::vector<std::vector<uint8_t>> ser{serializeMessage(self, input)};
        hashed = std::async(std::launch::async, [this, ser = std::move(ser), &h] { return HashBytes(ser, &h); });
    }
    Status st = encode();
    Status hs = sign_ ? hashed.get() : Status::Ok();
    if (!hs.ok()) return hs;
    if (!st.ok()) return st;
    if (sign_) *sig = sign_(h[0]);
    return Status::Ok();
}

Status ShardPlugin::prepareShards(const PeerID& self, const std::vector<uint8_t>* input,
                                  std::vector<Shard>* out) {
    if (input == nullptr) return Status::Err(RS_EINVAL, "network: input is null");
    std::vector<Share> shares;
    std::vector<uint8_t> sig;
    Status st = sign_input(self, *input, &sig, [&] { return shardInput(*input, &shares); });
    if (!st.ok()) return st;
    out->clear();
    for (Share& s : shares) {
        Shard m;
        m.FileSignature = sig;
        m.ShardData = std::move(s.Data);
        m.ShardNumber = static_cast<uint64_t>(s.Number);
        m.TotalShards = static_cast<uint64_t>(TotalShards);
        m.MinimumNeededShards = static_cast<uint64_t>(MinimumNeededShards);
        out->push_back(std::move(m));
    }
    return Status::Ok();
}

void ShardPlugin::prepareShardsBatch(const PeerID& self, const std::vector<std::vector<uint8_t>>& inputs,
                                     std::vector<std::vector<Shard>>* out, std::vector<Status>* sts) {
    out->assign(inputs.size(), {});
    sts->assign(inputs.size(), Status::Ok());
    std::vector<std::vector<uint8_t>> sigs(inputs.size());
    if (sign_) {
        std::vector<std::vector<uint8_t>> ser, h;
        ser.reserve(inputs.size());
        for (const std::vector<uint8_t>& in : inputs) ser.push_back(serializeMessage(self, in));
        Status hs = HashBytes(ser, &h);
        if (!hs.ok()) {
            sts->assign(inputs.size(), hs);
            return;
        }
        for (size_t i = 0; i < inputs.size(); ++i) sigs[i] = sign_(h[i]);
    }
    // The encodes: messages of equal length go through one rs_encode_batch
    // pass each (send-side batching); then shardInput's shares per message
    // (data shares copied out of the input, main.go:255-258).
    std::shared_ptr<FEC> f;
    Status fs = CachedFEC(MinimumNeededShards, TotalShards, &f);
    if (!fs.ok()) {
        sts->assign(inputs.size(), fs);
        return;
    }
    std::map<size_t, std::vector<size_t>> by_len;
    for (size_t i = 0; i < inputs.size(); ++i) by_len[inputs[i].size()].push_back(i);
    const size_t k = static_cast<size_t>(MinimumNeededShards), m = static_cast<size_t>(TotalShards) - k;
    for (const auto& [len, idx] : by_len) {
        std::vector<const uint8_t*> ptrs;
        for (size_t i : idx) ptrs.push_back(inputs[i].data());
        std::vector<std::vector<uint8_t>> parity;
        std::vector<Status> est;
        f->EncodeBatch(ptrs, len, &parity, &est);
        for (size_t q = 0; q < idx.size(); ++q) {
            const size_t i = idx[q];
            if (!est[q].ok()) {
                (*sts)[i] = est[q];
                continue;
            }
            const size_t S = len / k;
            for (size_t sn = 0; sn < k + m; ++sn) {
                Shard sh;
                sh.FileSignature = sigs[i];
                const uint8_t* src = sn < k ? inputs[i].data() + sn * S : parity[q].data() + (sn - k) * S;
                sh.ShardData.assign(src, src + S);
                sh.ShardNumber = static_cast<uint64_t>(sn);
                sh.TotalShards = static_cast<uint64_t>(TotalShards);
                sh.MinimumNeededShards = static_cast<uint64_t>(MinimumNeededShards);
                (*out)[i].push_back(std::move(sh));
            }
        }
    }
}

Status ShardPlugin::ShardAndBroadcast(const PeerID& self, const std::vector<uint8_t>* input,
                                      const std::function<void(const Shard&)>& broadcast) {
    std::vector<Shard> shards;
    Status st = prepareShards(self, input, &shards);
    if (!st.ok()) return st;
    for (const Shard& s : shards) broadcast(s);
    return Status::Ok();
}

Status ShardPlugin::ShardAndBroadcastWire(const PeerID& self, const std::vector<uint8_t>* input,
                                          const std::function<void(const uint8_t*, size_t)>& broadcast) {
    if (input == nullptr) return Status::Err(RS_EINVAL, "network: input is null");
    std::shared_ptr<FEC> f;
    Status st = CachedFEC(MinimumNeededShards, TotalShards, &f);
    if (!st.ok()) return st;
    const size_t k = static_cast<size_t>(MinimumNeededShards), n = static_cast<size_t>(TotalShards);
    if (input->size() % k != 0)
        return Status::Err(RS_ELEN_NOT_MULTIPLE, std::string("Encode: ") + rs_strerror(RS_ELEN_NOT_MULTIPLE));
    const size_t S = input->size() / k;
    std::lock_guard<std::mutex> lk(wire_mu_);
    wire_parity_.resize((n - k) * S);
    // The parity goes into this plugin's buffer while the signature hash
    // runs (sign_input); nothing is marshalled before the signature exists.
    std::vector<uint8_t> sig;
    st = sign_input(self, *input, &sig, [&] {
        if (S == 0 || n == k) return Status::Ok();
        const int rc = rs_encode(f->ctx(), input->data(), input->size(), wire_parity_.data());
        return rc == RS_OK ? Status::Ok() : Status::Err(rc, std::string("Encode: ") + rs_strerror(rc));
    });
    if (!st.ok()) return st;
    for (size_t i = 0; i < n; ++i) {
        rs_shard_view v{};
        v.file_signature = sig.data();
        v.file_signature_len = sig.size();
        v.shard_data = i < k ? input->data() + i * S : wire_parity_.data() + (i - k) * S;
        v.shard_data_len = S;
        v.shard_number = i;
        v.total_shards = n;
        v.minimum_needed_shards = k;
        const size_t need = rs_shard_size(&v);
        if (wire_.size() < need) wire_.resize(need);
        size_t w = 0;
        rs_shard_marshal(&v, wire_.data(), wire_.size(), &w);
        broadcast(wire_.data(), w);
    }
    return Status::Ok();
}

Status ShardPlugin::Receive(const PeerID& sender, const Shard& msg, ReceiveEvent* ev) {
    return receive(sender, msg, nullptr, ev);
}

Status ShardPlugin::Receive(const PeerID& sender, Shard&& msg, ReceiveEvent* ev) {
    return receive(sender, msg, &msg.ShardData, ev);
}

// take: the message's bytes may be moved into the pool (Receive(Shard&&)).
Status ShardPlugin::receive(const PeerID& sender, const Shard& msg, std::vector<uint8_t>* take, ReceiveEvent* ev) {
    ReceiveEvent local;
    ReceiveEvent& e = ev ? *ev : local;
    // Reset, keeping e.message's capacity for the decode (a caller that
    // reuses its event decodes into the same buffer every time).
    e.pooled = e.decoded = e.verified = false;
    e.decode_status = Status::Ok();
    e.message.clear();
    const std::string key = HexString(msg.FileSignature);
    std::vector<PoolEntry> pool;
    PoolEntry mine;  // this shard as a pool entry, built outside the lock
    {
        std::unique_lock<std::mutex> lk(mu_);
        auto it = shards_.find(key);
        const bool pools = it == shards_.end() ||
                           static_cast<int64_t>(it->second.size()) < static_cast<int64_t>(msg.MinimumNeededShards);
        if (pools) {
            // main.go:56-62 / :65-71: the share joins the pool.  Its bytes are
            // copied with the lock released; the pool is looked up again after
            // (another Receive may have changed it meanwhile, as the
            // reference's Load/Delete/Store sequence allows).
            lk.unlock();
            mine = take ? std::make_shared<const Share>(Share{static_cast<int>(msg.ShardNumber), std::move(*take)})
                        : std::make_shared<const Share>(Share{static_cast<int>(msg.ShardNumber), msg.ShardData});
            lk.lock();
            it = shards_.find(key);
            if (it == shards_.end() ||
                static_cast<int64_t>(it->second.size()) < static_cast<int64_t>(msg.MinimumNeededShards)) {
                shards_[key].push_back(std::move(mine));
                e.pooled = true;
                return Status::Ok();
            }
        }
        std::vector<PoolEntry>& p = it->second;
        const int64_t len = static_cast<int64_t>(p.size());
        if (!(len >= static_cast<int64_t>(msg.MinimumNeededShards) &&
              len <= static_cast<int64_t>(msg.TotalShards)))  // main.go:100-101
            return Status::Err(RS_EINVAL, "Shards mempool is larger than maximum size");
        pool = p;  // k shared pointers: the decode reads the bytes outside the lock
    }
    // main.go:72-99: k and n come from the message.
    e.decoded = true;
    std::shared_ptr<FEC> f;
    e.decode_status = CachedFEC(static_cast<int>(msg.MinimumNeededShards),
                                static_cast<int>(msg.TotalShards), &f);
    if (e.decode_status.ok()) e.decode_status = f->DecodeShared(&e.message, pool);
    if (!e.decode_status.ok()) e.message.clear();
    if (e.decode_status.ok() && verify_) {
        std::vector<std::vector<uint8_t>> h;
        if (HashBytes({serializeMessage(sender, e.message)}, &h).ok()) e.verified = verify_(h[0], msg.FileSignature);
    }
    if (e.verified) {  // main.go:90-92
        std::lock_guard<std::mutex> lk(mu_);
        shards_.erase(key);
        return Status::Ok();
    }
    if (pool.size() == msg.TotalShards)  // main.go:96-98
        return Status::Err(RS_ESINGULAR, "Could not put together the message due to corruption");
    return Status::Ok();
}

void ShardPlugin::ReceiveBatch(const std::vector<std::pair<PeerID, Shard>>& msgs,
                               std::vector<ReceiveEvent>* evs, std::vector<Status>* sts) {
    evs->assign(msgs.size(), ReceiveEvent{});
    sts->assign(msgs.size(), Status::Ok());
    struct Job {
        size_t msg;
        std::string key;
        std::vector<PoolEntry> pool;
    };
    std::vector<size_t> pending(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) pending[i] = i;
    while (!pending.empty()) {
        std::vector<size_t> deferred;
        std::vector<Job> jobs;
        std::unordered_map<std::string, bool> busy;  // key has a decode this phase
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (size_t i : pending) {
                const Shard& msg = msgs[i].second;
                ReceiveEvent& e = (*evs)[i];
                const std::string key = HexString(msg.FileSignature);
                if (busy.count(key)) {
                    deferred.push_back(i);
                    continue;
                }
                auto it = shards_.find(key);
                if (it == shards_.end()) {
                    shards_[key].push_back(
                        std::make_shared<const Share>(Share{static_cast<int>(msg.ShardNumber), msg.ShardData}));
                    e.pooled = true;
                    continue;
                }
                std::vector<PoolEntry>& p = it->second;
                const int64_t len = static_cast<int64_t>(p.size());
                if (len < static_cast<int64_t>(msg.MinimumNeededShards)) {
                    p.push_back(std::make_shared<const Share>(Share{static_cast<int>(msg.ShardNumber), msg.ShardData}));
                    e.pooled = true;
                    continue;
                }
                if (!(len >= static_cast<int64_t>(msg.MinimumNeededShards) &&
                      len <= static_cast<int64_t>(msg.TotalShards))) {
                    (*sts)[i] = Status::Err(RS_EINVAL, "Shards mempool is larger than maximum size");
                    continue;
                }
                busy[key] = true;
                jobs.push_back(Job{i, key, p});
            }
        }
        // A decoded (or failed) job: drop the pool once verified, else the
        // reference's corruption error when every shard was pooled.
        auto settle = [&](size_t j) {
            const Job& jb = jobs[j];
            const ReceiveEvent& e = (*evs)[jb.msg];
            const Shard& msg = msgs[jb.msg].second;
            if (e.verified) {
                std::lock_guard<std::mutex> lk(mu_);
                shards_.erase(jb.key);
            } else if (jb.pool.size() == msg.TotalShards) {
                (*sts)[jb.msg] = Status::Err(RS_ESINGULAR, "Could not put together the message due to corruption");
            }
        };
        std::vector<size_t> verify_jobs;
        // Decode the phase's pools, grouped by (k, n, share length).
        std::map<std::tuple<uint64_t, uint64_t, size_t>, std::vector<size_t>> groups;
        for (size_t j = 0; j < jobs.size(); ++j) {
            const Shard& m = msgs[jobs[j].msg].second;
            const size_t S = jobs[j].pool.empty() ? 0 : jobs[j].pool[0]->Data.size();
            groups[{m.MinimumNeededShards, m.TotalShards, S}].push_back(j);
        }
        for (auto& g : groups) {
            std::vector<size_t>& ids = g.second;
            for (size_t j : ids) (*evs)[jobs[j].msg].decoded = true;
            std::shared_ptr<FEC> f;
            Status fs = CachedFEC(static_cast<int>(std::get<0>(g.first)),
                                  static_cast<int>(std::get<1>(g.first)), &f);
            std::vector<std::vector<PoolEntry>> pools;
            std::vector<std::vector<uint8_t>> outs;
            std::vector<Status> st;
            bool uniform = true;  // a pool with mixed share lengths goes alone
            for (size_t j : ids)
                for (const PoolEntry& s : jobs[j].pool) uniform &= s->Data.size() == std::get<2>(g.first);
            if (fs.ok() && uniform) {
                for (size_t j : ids) pools.push_back(jobs[j].pool);
                f->DecodeBatchShared(pools, &outs, &st);
            } else {
                for (size_t j : ids) {
                    std::vector<uint8_t> o;
                    Status s1 = fs.ok() ? f->DecodeShared(&o, jobs[j].pool) : fs;
                    outs.push_back(std::move(o));
                    st.push_back(s1);
                }
            }
            for (size_t q = 0; q < ids.size(); ++q) {
                const Job& jb = jobs[ids[q]];
                ReceiveEvent& e = (*evs)[jb.msg];
                e.decode_status = st[q];
                if (st[q].ok()) e.message = std::move(outs[q]);
                if (st[q].ok() && verify_) verify_jobs.push_back(ids[q]);
                else settle(ids[q]);
            }
        }
        // Verify every decoded message of the phase: one GPU hash launch for
        // all of them (hp.HashBytes of serializeMessage, main.go:82-89).
        if (!verify_jobs.empty()) {
            std::vector<std::vector<uint8_t>> ser, h;
            ser.reserve(verify_jobs.size());
            for (size_t j : verify_jobs) ser.push_back(serializeMessage(msgs[jobs[j].msg].first, (*evs)[jobs[j].msg].message));
            const Status hs = HashBytes(ser, &h);
            for (size_t v = 0; v < verify_jobs.size(); ++v) {
                const size_t j = verify_jobs[v];
                ReceiveEvent& e = (*evs)[jobs[j].msg];
                e.verified = hs.ok() && verify_(h[v], msgs[jobs[j].msg].second.FileSignature);
                settle(j);
            }
        }
        pending.swap(deferred);
    }
}

}  // namespace rsmi_host
