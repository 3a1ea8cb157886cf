// shard_plugin.hpp -- C++ mirror of the reference plugin's shard path
// (/root/reference/main.go), on top of the engine (infectious.hpp):
//   ShardPlugin{MinimumNeededShards, TotalShards, Shards}  main.go:43-50
//   Receive (decode branch)                                main.go:52-107
//   NewShardPlugin                                         main.go:108-115
//   ShardAndBroadcast                                      main.go:201-210
//   prepareShards                                          main.go:211-241
//   shardInput                                             main.go:243-267
//   serializeMessage                                       main.go:276-302
//   largestPrimeFactors (CLI k/n re-derivation)            main.go:303-335
//   erasurecode.Shard + Marshal/Unmarshal/Size             protobuf/shard.proto:21-27
// Networking, ed25519 signing and discovery are out of scope:
// the signature scheme is a caller-supplied callback and "broadcast" is a
// callback receiving each Shard.  The hash policy (blake2b, main.go:38-41)
// applies when HashLen > 0: noise's Sign(sp, hp, msg) is
// sp.Sign(hp.HashBytes(msg)), so the callbacks then receive the BLAKE2b
// digest of serializeMessage(...) instead of the message itself.  Hashing
// goes through the engine's host/GPU crossover (rs_blake2b): the
// single-message paths (prepareShards, Receive) hash on the host CPU --
// prepareShards overlapping the GPU encode -- and ReceiveBatch /
// prepareShardsBatch hash a whole batch in one GPU launch when it holds
// enough messages.
#pragma once

#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "infectious.hpp"

namespace rsmi_host {

// erasurecode.Shard (protobuf/shard.pb.go:29-37).
struct Shard {
    std::vector<uint8_t> FileSignature;
    std::vector<uint8_t> ShardData;
    uint64_t ShardNumber = 0;
    uint64_t TotalShards = 0;
    uint64_t MinimumNeededShards = 0;

    size_t Size() const;                                   // shard.pb.go:355
    std::vector<uint8_t> Marshal() const;                  // shard.pb.go:209
    Status Unmarshal(const uint8_t* data, size_t len);     // shard.pb.go:413
    bool operator==(const Shard& o) const {
        return FileSignature == o.FileSignature && ShardData == o.ShardData &&
               ShardNumber == o.ShardNumber && TotalShards == o.TotalShards &&
               MinimumNeededShards == o.MinimumNeededShards;
    }
};

// peer.ID as serializeMessage uses it: Address string + Id bytes.
struct PeerID {
    std::string Address;
    std::vector<uint8_t> Id;
};

// [u32le len(Address)][Address][u32le len(Id)][Id][message]  (main.go:276-302)
std::vector<uint8_t> serializeMessage(const PeerID& id, const std::vector<uint8_t>& message);

// main.go:303-335; -1 for n < 2 (the reference's initial value).
int largestPrimeFactors(int n);

// keys.Sign(policy, hash, msg) stand-in and crypto.Verify stand-in.  With
// HashLen > 0 `msg` is blake2b-(8*HashLen)(serializeMessage(...)).
using Signer = std::function<std::vector<uint8_t>(const std::vector<uint8_t>& msg)>;
using Verifier = std::function<bool(const std::vector<uint8_t>& msg,
                                    const std::vector<uint8_t>& signature)>;

// What Receive did with one message (the reference only logs it).
struct ReceiveEvent {
    bool pooled = false;      // shard appended to / created the mempool
    bool decoded = false;     // decode branch ran (main.go:72-99)
    bool verified = false;    // signature check passed; pool deleted
    Status decode_status;     // NewFEC / Decode error (logged by the reference)
    std::vector<uint8_t> message;  // completeMessage
};

class ShardPlugin {
public:
    int MinimumNeededShards;
    int TotalShards;

    // 0: sign/verify callbacks see the serialized message (no hash policy);
    // 1..64: they see its BLAKE2b digest of that many bytes (rs_blake2b policy).
    int HashLen = 0;

    ShardPlugin(int minimumNeededShards, int totalShards, Signer sign, Verifier verify, int hashLen = 0);

    // main.go:52-107.  `sender` = ctx.Sender().  The mempool update is done
    // under one lock (the reference's Load->Delete->Store on sync.Map is not
    // atomic); the pooling rules are unchanged: shards are
    // appended until MinimumNeededShards are held, the next shard triggers
    // the decode of the pool (without itself being added), a pool holding
    // more than TotalShards is an error.
    Status Receive(const PeerID& sender, const Shard& msg, ReceiveEvent* ev = nullptr);
    // The same for a message the caller hands over: a pooled shard keeps the
    // message's ShardData (moved, not copied), as the reference's Share
    // aliases shard.ShardData (main.go:57-69).
    Status Receive(const PeerID& sender, Shard&& msg, ReceiveEvent* ev = nullptr);

    // Receive for a batch of arrivals (receive-side batching, SURVEY.md §8f
    // rank 3): the same pooling rules and per-key order as calling Receive on
    // each message in turn, but every pool that triggers in a phase is
    // decoded in one GPU pass (FEC::DecodeBatch per (k, n, share length)).
    // Arrivals for a key whose decode is in flight wait for the next phase.
    // (*evs)[i] / (*sts)[i] correspond to msgs[i].
    void ReceiveBatch(const std::vector<std::pair<PeerID, Shard>>& msgs,
                      std::vector<ReceiveEvent>* evs, std::vector<Status>* sts);

    // main.go:201-210 with net.Broadcast replaced by `broadcast`.
    Status ShardAndBroadcast(const PeerID& self, const std::vector<uint8_t>* input,
                             const std::function<void(const Shard&)>& broadcast);
    // ShardAndBroadcast with the Shards marshalled (what net.Broadcast sends,
    // shard.pb.go:219-252) straight from the encode's output -- the data
    // shares from the input, the parity from the plugin's parity buffer --
    // into one reused wire buffer: each share byte is copied once, where the
    // reference copies it twice (DeepCopy main.go:255-258, then Marshal).
    // broadcast gets each message's wire bytes, valid during the call; calls
    // on one plugin serialise on the buffers, so broadcast must not call
    // ShardAndBroadcastWire on the same plugin (Receive is fine).
    Status ShardAndBroadcastWire(const PeerID& self, const std::vector<uint8_t>* input,
                                 const std::function<void(const uint8_t* wire, size_t len)>& broadcast);
    // main.go:211-241 (input == nullptr -> "network: input is null").
    Status prepareShards(const PeerID& self, const std::vector<uint8_t>* input,
                         std::vector<Shard>* out);
    // prepareShards for many inputs: every input's signature hash in one
    // rs_blake2b call (HashLen > 0), and the encodes of equal-length inputs
    // in one rs_encode_batch pass each (send-side batching); shares as
    // shardInput makes them.  (*out)[i] / (*sts)[i] correspond to inputs[i].
    void prepareShardsBatch(const PeerID& self, const std::vector<std::vector<uint8_t>>& inputs,
                            std::vector<std::vector<Shard>>* out, std::vector<Status>* sts);
    // main.go:243-267
    Status shardInput(const std::vector<uint8_t>& input, std::vector<Share>* out);

    size_t PoolSize(const std::vector<uint8_t>& fileSignature) const;

    // hp.HashBytes over many messages (BLAKE2b, HashLen bytes, rs_blake2b);
    // with HashLen == 0 the messages are returned unchanged.
    Status HashBytes(const std::vector<std::vector<uint8_t>>& msgs, std::vector<std::vector<uint8_t>>* out) const;

private:
    Status sign_input(const PeerID& self, const std::vector<uint8_t>& input, std::vector<uint8_t>* sig,
                      const std::function<Status()>& encode);
    Status receive(const PeerID& sender, const Shard& msg, std::vector<uint8_t>* take, ReceiveEvent* ev);
    Signer sign_;
    Verifier verify_;
    mutable std::mutex mu_;
    // key: hex(signature).  Shares are held by shared ownership: a decode
    // snapshots the pool (k pointer copies) under mu_ and reads the bytes
    // after releasing it, like the Go slice the reference stores
    // (main.go:72-77 decodes the pool's own backing array).
    using PoolEntry = std::shared_ptr<const Share>;
    std::unordered_map<std::string, std::vector<PoolEntry>> shards_;
    std::mutex wire_mu_;
    std::vector<uint8_t> wire_;         // ShardAndBroadcastWire's marshal buffer (grown, never shrunk)
    std::vector<uint8_t> wire_parity_;  // ... and its parity shares
};

// NewShardPlugin(signaturePolicy, hashPolicy, k, n)  main.go:108-115;
// hashLen > 0 selects the BLAKE2b hash policy.
std::unique_ptr<ShardPlugin> NewShardPlugin(Signer sign, Verifier verify, int minimumNeededShards,
                                            int totalShards, int hashLen = 0);

std::string HexString(const std::vector<uint8_t>& b);  // fmt.Sprintf("%x", ...)

}  // namespace rsmi_host
