/*
 * rsmi.h -- C ABI of the MI355X-native Reed-Solomon engine that replaces the
 * github.com/vivint/infectious calls on the shard encode/reconstruct path of
 * da-moon/noise-erasurecode-plugin.
 *
 * Every entry point names the reference call site it replaces.  The Go side
 * of the plugin (ShardPlugin, main.go:43-115/201-267) and the protobuf Shard
 * message (protobuf/shard.proto:21-27) stay unchanged; a cgo package exposing
 * NewFEC / (*FEC).Encode / (*FEC).Decode / Share on top of this header (see
 * INTEGRATION.md) is the only change the plugin needs (its import at
 * main.go:24).
 *
 * Conventions
 *  - k = MinimumNeededShards (data shards), n = TotalShards, m = n - k.
 *  - All arithmetic is GF(2^8), polynomial 0x11D, systematic Vandermonde code
 *    with evaluation points {0, 2^1, ..., 2^(n-1)} (infectious NewFEC).
 *  - Status codes are ints: RS_OK (0) or a negative rs_status.
 *  - Host pointers are never retained past a call (cgo rule).
 *  - Device pointers / streams are HIP device pointers / hipStream_t passed
 *    as void*; the stream may be NULL (legacy default stream).
 *  - An rs_ctx is bound to one HIP device (or to several: a device set,
 *    rs_new_devices below) and may be shared between threads
 *    (noise calls Receive concurrently, once per peer connection,
 *    main.go:49-52).  Each call leases its own stream, pinned staging and
 *    device workspace from a pool inside the ctx (RSMI_MAX_LEASES, default
 *    16, concurrent calls; more wait for a lease), so concurrent calls run
 *    concurrently.  The only shared state is the decode-pattern cache,
 *    guarded by a reader/writer lock: lookups and launches share it, only a
 *    call that meets a new erasure pattern takes it exclusively.
 *  - There is no CPU fallback: without a usable gfx950 device rs_new returns
 *    RS_EDEVICE.
 */
#ifndef RSMI_H
#define RSMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    RS_OK = 0,
    RS_EINVAL_KN = -1,         /* NewFEC: "requires 1 <= k <= n <= 256"            */
    RS_ELEN_NOT_MULTIPLE = -2, /* Encode: "input length must be a multiple of k"   */
    RS_ENOT_ENOUGH = -3,       /* Decode/Rebuild: NotEnoughShares                  */
    RS_EBAD_SHARE_ID = -4,     /* Rebuild: "invalid share id"                      */
    RS_ESINGULAR = -5,         /* invertMatrix: "singular matrix" (duplicate ids)  */
    RS_ENO_SHARES = -6,        /* Decode: "must specify at least one share"        */
    RS_ESHARE_LEN = -7,        /* shares of unequal length                         */
    RS_EINVAL = -8,            /* bad argument (NULL, misaligned device buffer...) */
    RS_EDEVICE = -9,           /* HIP runtime error or no gfx950 device            */
    RS_ENOMEM = -10,           /* host or device allocation failed                 */
    RS_ETOO_MANY_ERRORS = -16, /* Correct: TooManyErrors (Berlekamp-Welch failed)  */
} rs_status;

typedef struct rs_ctx rs_ctx;

/* ---- construction: replaces infectious.NewFEC(k, n) ---------------------
 * main.go:73 (receive side, k/n from the message) and main.go:248 (send
 * side, shardInput).  Builds the n x k systematic matrix once and uploads it;
 * the plugin re-creating a ctx per message is cheap but a cached ctx per
 * (k, n) is what INTEGRATION.md recommends. */
int rs_new(int k, int n, rs_ctx **out);                 /* current HIP device */
int rs_new_on_device(int k, int n, int device, rs_ctx **out);
void rs_free(rs_ctx *ctx);
int rs_k(const rs_ctx *ctx);
int rs_n(const rs_ctx *ctx);
int rs_device(const rs_ctx *ctx);
/* Copy of the n x k row-major encode matrix (infectious FEC.enc_matrix). */
int rs_encode_matrix(const rs_ctx *ctx, uint8_t *out);
const char *rs_strerror(int status);
/* Diagnostics: name of the kernel that serves encode (which = 0) or
 * reconstruct (which = 1) for this ctx, e.g. "bitslice_k64_m16" or
 * "K10_MG4_B256" (no reference counterpart). */
const char *rs_kernel_name(const rs_ctx *ctx, int which);

/* ---- host-buffer API (the cgo path) -------------------------------------
 * rs_encode replaces (*FEC).Encode(input, output) at main.go:262.
 * input: len bytes, len % k == 0 (else RS_ELEN_NOT_MULTIPLE), S = len / k.
 * Data shares 0..k-1 are views input[i*S, (i+1)*S) (systematic, exactly as
 * infectious emits them); parity shares k..n-1 are written to
 * parity[(i-k)*S, (i-k+1)*S).  len == 0 is allowed (empty shares).
 * When input and parity are engine-pinned (rs_pinned_alloc / rs_arena),
 * 16-byte aligned with S % 16 == 0, and the code uses the split-table
 * kernel, the kernel reads and writes them in place over PCIe; rs_decode
 * likewise reads exactly k engine-pinned survivors in place (one launch, no
 * staging; dst written in place too when it is engine-pinned).  Pageable
 * buffers are staged through the lease's pinned memory, which the kernel
 * reads and writes over PCIe. */
int rs_encode(rs_ctx *ctx, const uint8_t *input, size_t len, uint8_t *parity);

/* rs_decode replaces (*FEC).Decode(dst, shares) at main.go:77: Correct, then
 * Rebuild.  numbers[count] / shares[count] describe the received
 * infectious.Share values; both arrays are sorted in place by number, like
 * infectious sorts the caller's slice.  Each share holds share_len bytes.
 * dst receives k * share_len bytes = the original input.
 * With exactly k distinct shares (the only case the plugin produces,
 * main.go:65) Correct has nothing to check.  With more, shares inconsistent
 * with one codeword are corrected by Berlekamp-Welch (up to
 * floor((count-k)/2) bad shares per byte column); the corrections go to dst
 * only -- unlike infectious, the caller's share bytes are not modified.
 * Errors: count < k -> RS_ENOT_ENOUGH; number outside [0, n) ->
 * RS_EBAD_SHARE_ID; fewer than k distinct numbers -> RS_ESINGULAR;
 * inconsistent shares with count - k < 2 -> RS_ENOT_ENOUGH; no codeword
 * within the correction radius -> RS_ETOO_MANY_ERRORS. */
int rs_decode(rs_ctx *ctx, int *numbers, const uint8_t **shares, int count,
              size_t share_len, uint8_t *dst);

/* rs_decode_batch: receive-side batching -- Decode
 * for `batch` messages of this code in one GPU pass.  Message b has
 * counts[b] shares; their numbers / pointers are consecutive in numbers[] /
 * shares[] (message b starts at sum(counts[0..b))), each share_len bytes;
 * dsts[b] receives k * share_len bytes.  Per-message results go to
 * status[b] (rs_decode's codes; each message's slice of numbers/shares is
 * sorted in place).  Messages with more than k distinct shares take the
 * rs_decode path (Correct); the rest are staged through pinned memory and
 * regenerated by rs_reconstruct_stripes launches that read the survivors over
 * PCIe where they lie (engine-pinned) or where they were staged, in chunks.
 * Batches beyond the pinned-staging cap (512 MiB; RSMI_BATCH_STAGE_MB) go in
 * groups of messages.  Returns RS_OK if every message decoded, else the first
 * failing status (in message order). */
int rs_decode_batch(rs_ctx *ctx, int batch, const int *counts, int *numbers,
                    const uint8_t **shares, size_t share_len, uint8_t **dsts, int *status);

/* rs_encode_batch: send-side batching, the counterpart of rs_decode_batch --
 * Encode (main.go:262, once per message in shardInput main.go:243-267) for
 * `batch` messages of this code in one GPU pass.  inputs[b] holds len bytes
 * (len % k == 0, else every status is RS_ELEN_NOT_MULTIPLE); parities[b]
 * receives (n - k) * len / k bytes laid out as rs_encode's parity.  The
 * messages are staged through pinned memory in chunks (the staging copy of
 * one chunk overlaps the kernel of the previous one, which reads and writes
 * the staging over PCIe), in groups of messages within the pinned-staging cap
 * (512 MiB; RSMI_BATCH_STAGE_MB).  status[b] gets each message's code;
 * returns RS_OK if every message encoded, else the first failing status. */
int rs_encode_batch(rs_ctx *ctx, int batch, const uint8_t *const *inputs, size_t len,
                    uint8_t *const *parities, int *status);

/* ---- device-resident batched API (many stripes per launch) ---------------
 * Stripe s, shard i lives at
 *     i <  k:  data   + s * data_stripe_stride   + i       * shard_pitch
 *     i >= k:  parity + s * parity_stripe_stride + (i - k) * shard_pitch
 * shard_len bytes are coded per shard; shard_pitch, both stripe strides and
 * both base pointers must be multiples of 16 and shard_pitch >=
 * round_up(shard_len, 16) (bytes between shard_len and the next multiple of
 * 16 are coded too: padding, never read back by the host API).
 *
 * rs_encode_stripes: parity of every stripe (stripe-batched (*FEC).Encode).
 * Enqueued on stream; returns when the launch is queued. */
int rs_encode_stripes(rs_ctx *ctx, const void *data, size_t data_stripe_stride,
                      void *parity, size_t parity_stripe_stride, size_t shard_pitch,
                      size_t shard_len, size_t stripes, void *stream);

/* rs_reconstruct_stripes: erased is a HOST array of stripes * n flags
 * (non-zero = shard i of stripe s is missing).  Every erased shard, data or
 * parity, is regenerated in place from k survivors chosen like infectious
 * Rebuild (data shares first, then the highest-numbered parity).  Per-pattern
 * decode matrices are inverted once and cached in the ctx.  A stripe with
 * more than m erasures -> RS_ENOT_ENOUGH (nothing is launched).  Enqueued on
 * stream (the small pattern tables are staged through pinned memory). */
int rs_reconstruct_stripes(rs_ctx *ctx, void *data, size_t data_stripe_stride,
                           void *parity, size_t parity_stripe_stride, size_t shard_pitch,
                           size_t shard_len, size_t stripes, const uint8_t *erased,
                           void *stream);

/* rs_reconstruct_ptrs: rs_reconstruct_stripes with shards anywhere in
 * device memory.  shard_ptrs is a DEVICE array [stripes][n] of device
 * addresses (16-byte aligned): shard i of stripe s is read (survivor) or
 * written (erased) at shard_ptrs[s * n + i]; entries of present shards that
 * Rebuild does not choose are never dereferenced.  shard_len bytes per
 * shard (round_up(shard_len, 16) are coded).  The survivor gather of the
 * shard-distributed placement reconstructs straight out of its receive
 * buffers with it, and rs_decode_batch out of its packed
 * staging.  Enqueued on stream. */
int rs_reconstruct_ptrs(rs_ctx *ctx, const uint64_t *shard_ptrs, size_t shard_len, size_t stripes,
                        const uint8_t *erased, void *stream);

/* Cached decode patterns held by the ctx (diagnostics / tests).  The cache
 * holds at most 2^20 patterns (RSMI_PATTERN_CAP); a call that would exceed
 * that evicts it whole, with no host synchronisation (the rebuilt rows wait
 * on the device for the launches that read the old ones).
 * rs_pattern_evictions counts those evictions. */
int rs_pattern_count(const rs_ctx *ctx);
int64_t rs_pattern_evictions(const rs_ctx *ctx);

/* Counters of a ctx (diagnostics / tests). */
enum {
    RS_STAT_PATTERNS = 0,          /* cached decode patterns                          */
    RS_STAT_EVICTIONS = 1,         /* pattern-cache evictions                         */
    RS_STAT_BATCHES_IN_PLACE = 2,  /* rs_decode_batch calls that read survivors in place */
    RS_STAT_BATCHES_STAGED = 3,    /* ... that staged them through pinned copies      */
    RS_STAT_LEASES = 4,            /* leases created (peak concurrent calls)          */
    RS_STAT_ENCODES_IN_PLACE = 5,  /* rs_encode calls served from engine-pinned memory */
    RS_STAT_DECODES_IN_PLACE = 6,  /* rs_decode calls that read engine-pinned survivors in place */
    RS_STAT_REC_STRIPES_TABLE = 7,  /* stripes reconstructed by the split-table kernel (batched API) */
    RS_STAT_REC_STRIPES_SYNDROME = 8, /* ... by the bit-sliced syndrome kernels                     */
    RS_STAT_ENCODE_BATCHES = 9,    /* rs_encode_batch GPU passes (one per staging group) */
    RS_STAT_MAILBOX_CALLS = 10,    /* rs_encode / rs_decode calls whose chunks went to a mailbox grid */
    RS_STAT_MAILBOX_RECOVERED = 11, /* ... of them with a chunk the grid left undone (launched by the caller) */
};
int64_t rs_stat(const rs_ctx *ctx, int which);

/* Diagnostics: the decode rows the engine uses for one erasure pattern
 * (erased = n flags).  rows receives m*k bytes: row t (t < *count) is the
 * combination of the k survivors (Rebuild's choice) that regenerates the
 * t-th erased shard in increasing id order; built on the GPU like every
 * batched pattern.  Synchronises the ctx's device. */
int rs_pattern_rows(rs_ctx *ctx, const uint8_t *erased, uint8_t *rows, int *count);

/* Precompute (invert and upload) the decode patterns of every erasure set of
 * 1..max_erasures shards (max_erasures <= m), e.g. the 1,470 patterns of
 * RS(10,4) with <= 4 erasures, so later rs_reconstruct_stripes calls only
 * index them.  RS_EINVAL if that would exceed 2^20 patterns. */
int rs_prepare_patterns(rs_ctx *ctx, int max_erasures, void *stream);

/* ---- signature hashing: batched BLAKE2b -----------
 * The plugin signs and verifies blake2b(serializeMessage(id, message)):
 * defaultHashPolicy = blake2b.New() (main.go:38-41), keys.Sign at
 * main.go:219-223 on the send side, crypto.Verify at main.go:82-89 after
 * every decode; the framing is serializeMessage (main.go:276-302).  These
 * hash many messages per launch (RFC 7693 BLAKE2b, unkeyed, digest_len 1..64
 * bytes; noise's policy is recalled to use the 32-byte digest, which is not
 * BLAKE2b-512 truncated: the digest length is part of the parameter block).
 * BLAKE2b chains a message's 128-byte blocks sequentially, so one message
 * runs on 4 lanes; batches of hundreds of messages or more pay off.
 *
 * rs_blake2b_batch: host messages msgs[i] of lens[i] bytes (any alignment)
 * -> out[i * digest_len ...].  Staged through pinned memory like
 * rs_decode_batch; returns when out is written. */
int rs_blake2b_batch(rs_ctx *ctx, int count, const uint8_t *const *msgs, const size_t *lens,
                     int digest_len, uint8_t *out);
/* rs_blake2b_device: device-resident messages.  msg_ptrs[count] (device
 * addresses, any alignment) and lens[count] are device arrays; order
 * (device, may be NULL) lists the messages longest first; out is device
 * memory of count * digest_len bytes.  Enqueued on stream. */
int rs_blake2b_device(rs_ctx *ctx, int count, const uint64_t *msg_ptrs, const uint64_t *lens,
                      const uint32_t *order, int digest_len, uint8_t *out, void *stream);
/* rs_blake2b: the hash policy the plugin uses (hp.HashBytes, main.go:38-41,
 * :219-223, :82-89) with a host/GPU crossover.  A single message, or a batch
 * whose longest chain dominates, is hashed on the host CPU (C BLAKE2b, one
 * thread per message up to the CPUs this process may use); a batch with
 * many messages in flight goes to the GPU kernel (rs_blake2b_batch).  The
 * choice compares the two paths' estimated times; the
 * digests are identical either way.  RSMI_HASH=host / gpu forces a side.
 * *where (may be NULL) reports the side taken: 0 host, 1 GPU.
 * Replaces: hp.HashBytes(serializeMessage(...)) at main.go:219-223 (sign) and
 * main.go:82-89 (verify). */
int rs_blake2b(rs_ctx *ctx, int count, const uint8_t *const *msgs, const size_t *lens, int digest_len,
               uint8_t *out, int *where);
/* rs_blake2b_host: host-only BLAKE2b of host messages on `threads` threads
 * (<= 0: the CPUs this process may use).  Needs no context and no GPU. */
int rs_blake2b_host(int count, const uint8_t *const *msgs, const size_t *lens, int digest_len, uint8_t *out,
                    int threads);

/* ---- memory helpers ------------------------------------------------------
 * Engine-pinned host memory (hipHostMalloc, mapped for the device).  The
 * engine keeps a registry of these ranges: rs_decode_batch recognises
 * survivors that lie in them (and are 16-byte aligned) without querying the
 * runtime, and its reconstruct kernel reads them over PCIe in place -- no
 * staging memcpy, no per-shard DMA (zero-copy receive, SURVEY.md §8f rank 1;
 * the reference copies every ShardData at Unmarshal, shard.pb.go:468-503,
 * and DeepCopy's every share, main.go:255-258). */
void *rs_pinned_alloc(size_t bytes); /* NULL on failure */
void rs_pinned_free(void *p);
/* Receive arena: one pinned range carved into 256-byte aligned slots by a
 * bump pointer (rs_shard_unmarshal_arena places ShardData in it).  Reset
 * recycles every slot; not thread-safe (one arena per receiving thread).
 * rs_arena_put copies bytes into a fresh slot with streaming stores, as
 * rs_shard_unmarshal_arena does: the lines go to DRAM instead of staying
 * dirty in the CPU's caches, where each of the kernel's PCIe reads would
 * have to snoop them out. */
typedef struct rs_arena rs_arena;
rs_arena *rs_arena_new(size_t bytes);            /* NULL on failure */
void *rs_arena_alloc(rs_arena *a, size_t bytes); /* NULL when full */
void *rs_arena_put(rs_arena *a, const void *data, size_t bytes); /* the slot, NULL when full */
void rs_arena_reset(rs_arena *a);
size_t rs_arena_used(const rs_arena *a);
void rs_arena_free(rs_arena *a);
int rs_device_alloc(rs_ctx *ctx, size_t bytes, void **out);
int rs_device_free(rs_ctx *ctx, void *p);
int rs_stream_sync(rs_ctx *ctx, void *stream);

/* ---- device sets: one context over several GPUs ---------------------------
 * north_star: "stripes are independent, so they are partitioned across the 8
 * GPUs of one node with no collectives on the encode path"; SURVEY.md §8e and
 * §7.5 ("one host thread + stream per GPU").  The plugin process that loads
 * this library (through the Go shim's NewFECOnDevices) uses every GPU of the
 * node through one context:
 *
 * rs_new_devices builds a context over `count` HIP devices (devices[i];
 * repeats allowed -- two members on one GPU).  Member i is an ordinary
 * single-device context on devices[i] (rs_member; owned by the set, never
 * freed by the caller) with one host worker thread of its own.  Peer access
 * is enabled between every pair of distinct member devices that supports it.
 * Every entry point above accepts a device-set context:
 *  - rs_encode / rs_decode (one message) run on the member with the fewest
 *    calls in flight (concurrent Receive goroutines spread over the GPUs);
 *  - rs_encode_batch / rs_decode_batch split the messages into `count`
 *    contiguous ranges (rs_partition), each range on its member's thread, all
 *    members at once; per-message status and the return value as on one GPU;
 *  - the device-resident calls (rs_encode_stripes, rs_reconstruct_stripes,
 *    rs_reconstruct_ptrs, rs_fill_splitmix, rs_blake2b_device) run on a
 *    member on the device that holds their (first) device buffer, RS_EINVAL
 *    if no member is on it; rs_prepare_patterns (stream must be NULL) runs
 *    on every member; rs_blake2b* on the least-busy member;
 *  - rs_stat / rs_pattern_count / rs_pattern_evictions are summed over the
 *    members; rs_pattern_rows / rs_kernel_name / rs_device / rs_device_alloc
 *    are member 0's.
 * A single-device context is a set of one for the calls below. */
int rs_new_devices(int k, int n, const int *devices, int count, rs_ctx **out);
int rs_member_count(const rs_ctx *ctx);          /* 1 for a single-device context */
rs_ctx *rs_member(rs_ctx *ctx, int i);           /* NULL if i is out of range; owned by
                                                    the set (rs_free on it does nothing) */

/* Contiguous partition of `units` (stripes, messages) into `parts` ranges:
 * part p covers [*first, *first + *count) with first = units*p/parts, so the
 * ranges tile [0, units) in order and differ in size by at most one. */
int rs_partition(size_t units, int parts, int part, size_t *first, size_t *count);

/* Device-resident stripes already placed per member (stripe-local placement,
 * the headline): part i describes the stripes member i holds, in that
 * member's device memory, laid out as for rs_encode_stripes; stream is a
 * stream of member i's device or NULL.  All members' launches are issued
 * concurrently, one host thread per member; returns when every part is
 * queued (RS_OK, or the first failing status in member order). */
typedef struct rs_stripe_part {
    void *data;
    size_t data_stripe_stride;
    void *parity;
    size_t parity_stripe_stride;
    size_t stripes;
    void *stream;
} rs_stripe_part;
int rs_encode_stripes_parts(rs_ctx *ctx, const rs_stripe_part *parts, size_t shard_pitch, size_t shard_len);
/* erased: HOST flags [sum of parts' stripes][n], in part order (part i's
 * stripes follow part i-1's). */
int rs_reconstruct_stripes_parts(rs_ctx *ctx, const rs_stripe_part *parts, size_t shard_pitch, size_t shard_len,
                                 const uint8_t *erased);

/* Shard-distributed placement (the device analogue of the
 * plugin sending every shard to a different peer, main.go:207): shard i of
 * stripe s lives on ANY member's device, at the device address
 * shard_ptrs[s * n + i] (a HOST array; 16-byte aligned).  owner[s] (HOST) is
 * the member that reconstructs stripe s: its kernel reads Rebuild's survivors
 * where they lie -- over xGMI when they sit on another GPU (peer access, no
 * staging copy, no collective) -- and writes each erased shard at its address
 * (local or peer).  streams[i] (may be NULL, or hold NULLs) is member i's
 * stream; the survivors must be complete when those streams run.  Returns
 * when every member's launch is queued; RS_EDEVICE when the set spans devices
 * without peer access. */
int rs_reconstruct_spread(rs_ctx *ctx, const uint64_t *shard_ptrs, const int *owner, size_t shard_len,
                          size_t stripes, const uint8_t *erased, void *const *streams);

/* ---- bench / test utility (not on the codec path) ------------------------
 * Fill len bytes of device memory with the splitmix64 byte stream of seed
 * (byte i = byte i%8 of splitmix64(seed + (i/8 + 1) * golden)), the same
 * stream the CPU baseline generates. */
int rs_fill_splitmix(rs_ctx *ctx, void *dev, size_t len, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RSMI_H */
