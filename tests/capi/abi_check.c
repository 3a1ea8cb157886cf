/*
 * abi_check.c -- the C ABI (include/rsmi.h, include/rsmi_wire.h) driven from
 * C the way the cgo shim (go/infectious/fec.go) drives it, checked against
 * the oracle (test infrastructure: this program links oracle/build/liboracle.so
 * as the checker only).  Run by tests/test_capi_c.py on the GPU box.
 *
 * Sequence (reference call sites): NewFEC main.go:73/:248 -> rs_new;
 * Encode main.go:262 -> rs_encode (config 1 blob); Decode main.go:77 ->
 * rs_decode with shares in arrival order (sorted in place); receive-side
 * batching -> rs_decode_batch with ShardData unmarshalled into an rs_arena
 * (zero-copy); send-side batching -> rs_encode_batch; the blake2b hash policy -> rs_blake2b_batch (RFC 7693 known
 * answers); error classes; 8 pthreads decoding on one context; the same
 * host calls on a device-set context (rs_new_devices over {0, 0}: two members
 * on the box's one GPU), the way the shim's NewFECOnDevices drives it.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rsmi.h"
#include "../../include/rsmi_wire.h"
#include "../../oracle/rs_oracle.h"

static int failures = 0;
#define CHECK(cond, ...)                          \
    do {                                          \
        if (!(cond)) {                            \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);         \
            fprintf(stderr, "\n");                \
            ++failures;                           \
        }                                         \
    } while (0)

static uint8_t *splitmix(size_t n, uint64_t seed) {
    uint8_t *b = malloc(n ? n : 1);
    orc_fill_splitmix(b, n, seed);
    return b;
}

static void hex(const uint8_t *d, int n, char *out) {
    for (int i = 0; i < n; i++) sprintf(out + 2 * i, "%02x", d[i]);
}

/* Encode + Decode of one message through the host API vs the oracle. */
static void check_encode_decode(rs_ctx *ctx, int k, int n, size_t len, uint64_t seed) {
    const int m = n - k;
    const size_t S = len / k;
    uint8_t *in = splitmix(len, seed);
    uint8_t *par = malloc(m * S), *ref = malloc(m * S), *out = malloc(len);
    uint8_t enc[256 * 256];
    orc_fec_matrix(k, n, 1, enc);
    CHECK(rs_encode(ctx, in, len, par) == RS_OK, "rs_encode");
    CHECK(orc_encode(enc, k, n, in, len, ref) == 0, "orc_encode");
    CHECK(memcmp(par, ref, m * S) == 0, "parity != oracle (k=%d n=%d len=%zu)", k, n, len);
    /* the last k shares, in reverse arrival order (first m data shards lost) */
    int nums[256];
    const uint8_t *ptrs[256];
    for (int i = 0; i < k; i++) {
        const int id = n - 1 - i;
        nums[i] = id;
        ptrs[i] = id < k ? in + (size_t)id * S : par + (size_t)(id - k) * S;
    }
    CHECK(rs_decode(ctx, nums, ptrs, k, S, out) == RS_OK, "rs_decode");
    CHECK(memcmp(out, in, len) == 0, "decoded != input (k=%d n=%d)", k, n);
    for (int i = 1; i < k; i++) CHECK(nums[i - 1] < nums[i], "numbers not sorted in place");
    free(in); free(par); free(ref); free(out);
}

/* Send-side batching: B messages' parity in one rs_encode_batch call, each
 * against the oracle (the way a cgo sender would call it). */
static void check_encode_batch(rs_ctx *ctx, int k, int n, size_t len, int B) {
    const int m = n - k;
    const size_t S = len / k;
    uint8_t enc[256 * 256];
    orc_fec_matrix(k, n, 1, enc);
    const uint8_t *ins[64];
    uint8_t *outs[64];
    int st[64];
    for (int b = 0; b < B; b++) {
        ins[b] = splitmix(len, 0xBA7 + (uint64_t)b);
        outs[b] = malloc(m * S);
    }
    const int64_t batches0 = rs_stat(ctx, RS_STAT_ENCODE_BATCHES);
    CHECK(rs_encode_batch(ctx, B, ins, len, outs, st) == RS_OK, "rs_encode_batch");
    /* one batched pass per member (a device set splits the messages) */
    CHECK(rs_stat(ctx, RS_STAT_ENCODE_BATCHES) == batches0 + rs_member_count(ctx), "rs_encode_batch not batched");
    uint8_t *ref = malloc(m * S);
    for (int b = 0; b < B; b++) {
        CHECK(orc_encode(enc, k, n, ins[b], len, ref) == 0, "orc_encode");
        CHECK(st[b] == RS_OK && memcmp(outs[b], ref, m * S) == 0, "encode batch message %d (k=%d n=%d)", b, k, n);
        free((void *)ins[b]);
        free(outs[b]);
    }
    free(ref);
}

/* Receive batching: marshalled Shards unmarshalled into an arena, decoded in
 * one rs_decode_batch that reads them in place. */
static void check_arena_batch(rs_ctx *ctx, int k, int n, size_t S, int B) {
    const int m = n - k;
    rs_arena *arena = rs_arena_new((size_t)B * k * ((S + 255) / 256 * 256) + 4096);
    CHECK(arena != NULL, "rs_arena_new");
    if (!arena) return;
    uint8_t enc[256 * 256];
    orc_fec_matrix(k, n, 1, enc);
    uint8_t **inputs = calloc(B, sizeof(uint8_t *)), **dsts = calloc(B, sizeof(uint8_t *));
    int *counts = calloc(B, sizeof(int)), *nums = calloc((size_t)B * k, sizeof(int)), *st = calloc(B, sizeof(int));
    const uint8_t **ptrs = calloc((size_t)B * k, sizeof(uint8_t *));
    uint8_t sig[64];
    memset(sig, 0x42, sizeof sig);
    const int64_t in_place0 = rs_stat(ctx, RS_STAT_BATCHES_IN_PLACE);
    for (int b = 0; b < B; b++) {
        inputs[b] = splitmix((size_t)k * S, 900 + b);
        uint8_t *par = malloc((size_t)m * S);
        orc_encode(enc, k, n, inputs[b], (size_t)k * S, par);
        counts[b] = k;
        /* keep shares b%n, b%n+1, ... (k consecutive ids mod n) */
        for (int j = 0; j < k; j++) {
            const int id = (b + j) % n;
            rs_shard_view v = {sig, sizeof sig, id < k ? inputs[b] + (size_t)id * S : par + (size_t)(id - k) * S,
                               S, (uint64_t)id, (uint64_t)n, (uint64_t)k};
            uint8_t *wire = malloc(rs_shard_size(&v));
            size_t w = 0;
            CHECK(rs_shard_marshal(&v, wire, rs_shard_size(&v), &w) == 0, "marshal");
            rs_shard_view u;
            CHECK(rs_shard_unmarshal_arena(wire, w, arena, &u) == 0, "unmarshal_arena");
            CHECK(((uintptr_t)u.shard_data & 15u) == 0 && u.shard_number == (uint64_t)id, "arena view");
            nums[b * k + j] = (int)u.shard_number;
            ptrs[b * k + j] = u.shard_data;
            free(wire);
        }
        dsts[b] = malloc((size_t)k * S);
        free(par);
    }
    CHECK(rs_decode_batch(ctx, B, counts, nums, ptrs, S, dsts, st) == RS_OK, "rs_decode_batch");
    for (int b = 0; b < B; b++)
        CHECK(st[b] == RS_OK && memcmp(dsts[b], inputs[b], (size_t)k * S) == 0, "batch message %d", b);
    CHECK(rs_stat(ctx, RS_STAT_BATCHES_IN_PLACE) == in_place0 + rs_member_count(ctx), "batch not read in place");
    for (int b = 0; b < B; b++) { free(inputs[b]); free(dsts[b]); }
    free(inputs); free(dsts); free(counts); free(nums); free(st); free(ptrs);
    /* rs_arena_put: a copy in a fresh aligned slot; NULL once the arena is full */
    rs_arena_reset(arena);
    const char msg[] = "arena put";
    void *slot = rs_arena_put(arena, msg, sizeof msg);
    CHECK(slot != NULL && ((uintptr_t)slot & 15u) == 0 && memcmp(slot, msg, sizeof msg) == 0, "rs_arena_put");
    CHECK(rs_arena_put(arena, msg, (size_t)1 << 40) == NULL, "rs_arena_put past the end");
    rs_arena_free(arena);
}

static void check_blake2b(rs_ctx *ctx) {
    const uint8_t abc[3] = {'a', 'b', 'c'};
    uint8_t kb[1024];
    for (int i = 0; i < 1024; i++) kb[i] = (uint8_t)i;
    const uint8_t *msgs[3] = {abc, kb, NULL};
    size_t lens[3] = {3, 1024, 0};
    uint8_t out[3 * 32];
    char h[65];
    CHECK(rs_blake2b_batch(ctx, 3, msgs, lens, 32, out) == RS_OK, "rs_blake2b_batch");
    hex(out, 32, h);
    CHECK(strcmp(h, "bddd813c634239723171ef3fee98579b94964e3bb1cb3e427262c8c068d52319") == 0, "blake2b-256(abc) %s", h);
    hex(out + 32, 32, h);
    CHECK(strcmp(h, "f1551feeb252c7e60bb362205bd1ac2f70b145260a91d41e8c5d0a187549a5f2") == 0, "blake2b-256(0..255 x4) %s", h);
    hex(out + 64, 32, h);
    CHECK(strcmp(h, "0e5751c026e543b2e8ab2eb06099daa1d1e5df47778f7787faab45cdf12fe3a8") == 0, "blake2b-256('') %s", h);
    uint8_t o64[64];
    CHECK(rs_blake2b_batch(ctx, 1, msgs, lens, 64, o64) == RS_OK, "rs_blake2b_batch 64");
    char h2[129];
    hex(o64, 64, h2);
    CHECK(strncmp(h2, "ba80a53f981c4d0d6a2797b69f12f6e9", 32) == 0, "blake2b-512(abc) %s", h2);
}

static void check_errors(rs_ctx *ctx) {
    rs_ctx *bad = NULL;
    CHECK(rs_new(0, 4, &bad) == RS_EINVAL_KN && bad == NULL, "rs_new(0,4)");
    CHECK(rs_new(5, 4, &bad) == RS_EINVAL_KN, "rs_new(5,4)");
    CHECK(rs_new(10, 257, &bad) == RS_EINVAL_KN, "rs_new(10,257)");
    uint8_t buf[40] = {0}, out[40];
    CHECK(rs_encode(ctx, buf, 25, out) == RS_ELEN_NOT_MULTIPLE, "len %% k");
    int nums[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 14};
    const uint8_t *ptrs[10];
    for (int i = 0; i < 10; i++) ptrs[i] = buf;
    CHECK(rs_decode(ctx, nums, ptrs, 10, 4, out) == RS_EBAD_SHARE_ID, "bad share id");
    int nums2[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 14};
    CHECK(rs_decode(ctx, nums2, ptrs, 10, 0, NULL) == RS_EBAD_SHARE_ID, "bad id, zero-length shares");
    int nums3[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 8};
    CHECK(rs_decode(ctx, nums3, ptrs, 10, 4, out) == RS_ESINGULAR, "duplicate ids");
    CHECK(rs_decode(ctx, nums3, ptrs, 9, 4, out) == RS_ENOT_ENOUGH, "not enough");
}

struct job {
    rs_ctx *ctx;
    int seed;
    int ok;
};

static void *decode_worker(void *arg) {
    struct job *j = arg;
    const int k = 10, n = 14, m = 4;
    const size_t S = 104858, len = k * S;
    uint8_t *in = splitmix(len, 5000 + j->seed), *par = malloc(m * S), *out = malloc(len);
    j->ok = rs_encode(j->ctx, in, len, par) == RS_OK;
    for (int rep = 0; rep < 4 && j->ok; rep++) {
        int nums[10];
        const uint8_t *ptrs[10];
        for (int i = 0; i < k; i++) {
            const int id = (j->seed + rep + i) % n;
            nums[i] = id;
            ptrs[i] = id < k ? in + (size_t)id * S : par + (size_t)(id - k) * S;
        }
        j->ok = rs_decode(j->ctx, nums, ptrs, k, S, out) == RS_OK && memcmp(out, in, len) == 0;
    }
    free(in); free(par); free(out);
    return NULL;
}

int main(void) {
    rs_ctx *c10 = NULL, *c64 = NULL, *c4 = NULL;
    if (rs_new(10, 14, &c10) != RS_OK || rs_new(64, 80, &c64) != RS_OK || rs_new(4, 6, &c4) != RS_OK) {
        fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    check_encode_decode(c10, 10, 14, 1048580, 0x5EED); /* BASELINE config 1 */
    /* a config-1 message's encode and decode go through the mailbox grid
     * (unless RSMI_MAILBOX=0), and no chunk was left to the caller */
    if (!getenv("RSMI_MAILBOX"))
        CHECK(rs_stat(c10, RS_STAT_MAILBOX_CALLS) >= 2 && rs_stat(c10, RS_STAT_MAILBOX_RECOVERED) == 0, "mailbox grid");
    check_encode_decode(c10, 10, 14, 10 * 17, 3);
    check_encode_decode(c64, 64, 80, 64 * 4099, 4);
    check_encode_decode(c4, 4, 6, 64, 5);              /* plugin default RS(4,2) */
    check_encode_batch(c10, 10, 14, 1048580, 24);     /* config-1 messages, chunked staging */
    check_encode_batch(c64, 64, 80, 64 * 4099, 5);
    check_arena_batch(c10, 10, 14, 6554, 64);
    check_arena_batch(c64, 64, 80, 4099, 8);
    check_blake2b(c10);
    check_errors(c10);
    pthread_t th[8];
    struct job jobs[8];
    for (int t = 0; t < 8; t++) {
        jobs[t] = (struct job){c10, t, 0};
        pthread_create(&th[t], NULL, decode_worker, &jobs[t]);
    }
    for (int t = 0; t < 8; t++) {
        pthread_join(th[t], NULL);
        CHECK(jobs[t].ok, "concurrent decode thread %d", t);
    }
    printf("abi_check: %lld leases on the RS(10,4) context after 8 concurrent decoders\n",
           (long long)rs_stat(c10, RS_STAT_LEASES));
    /* Device set {0, 0}: the plugin process's multi-GPU context (north_star's
     * stripe partition behind the C ABI), two members on one GPU here. */
    {
        const int devs[2] = {0, 0};
        rs_ctx *set = NULL;
        CHECK(rs_new_devices(10, 14, devs, 2, &set) == RS_OK && set, "rs_new_devices");
        if (set) {
            CHECK(rs_member_count(set) == 2 && rs_member(set, 1) && !rs_member(set, 2), "members");
            size_t f0 = 0, n0 = 0, f1 = 0, n1 = 0;
            CHECK(rs_partition(24, 2, 0, &f0, &n0) == RS_OK && rs_partition(24, 2, 1, &f1, &n1) == RS_OK &&
                      f0 == 0 && n0 == 12 && f1 == 12 && n1 == 12, "rs_partition");
            check_encode_decode(set, 10, 14, 1048580, 0x5E7);
            check_encode_batch(set, 10, 14, 1048580, 24); /* 12 + 12 messages, one pass per member */
            check_arena_batch(set, 10, 14, 6554, 64);
            check_blake2b(set);
            for (int t = 0; t < 8; t++) {
                jobs[t] = (struct job){set, 100 + t, 0};
                pthread_create(&th[t], NULL, decode_worker, &jobs[t]);
            }
            for (int t = 0; t < 8; t++) {
                pthread_join(th[t], NULL);
                CHECK(jobs[t].ok, "device-set concurrent decode thread %d", t);
            }
            CHECK(rs_stat(rs_member(set, 0), RS_STAT_LEASES) >= 1 && rs_stat(rs_member(set, 1), RS_STAT_LEASES) >= 1,
                  "both members served calls");
            rs_free(set);
        }
    }
    rs_free(c10);
    rs_free(c64);
    rs_free(c4);
    printf("abi_check: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
