/*
 * rsmi_wire.h -- C ABI codec of the plugin's wire message erasurecode.Shard
 * (protobuf/shard.proto:21-27), byte-compatible with the gogo-generated
 * code it would sit beside:
 *   Size       protobuf/shard.pb.go:355-375
 *   MarshalTo  protobuf/shard.pb.go:219-252 (field order 1..5, zero values
 *              and empty bytes omitted, varint lengths)
 *   Unmarshal  protobuf/shard.pb.go:413-581 (last occurrence wins, unknown
 *              fields skipped like skipShard :582-686, same error classes)
 *
 * Views are zero-copy: an unmarshalled rs_shard_view points into the input
 * buffer, so a reconstruct can read ShardData straight from a pinned receive
 * buffer.  Status codes extend rs_status (rsmi.h).
 */
#ifndef RSMI_WIRE_H
#define RSMI_WIRE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    RS_EWIRE_EOF = -11,        /* io.ErrUnexpectedEOF                         */
    RS_EWIRE_OVERFLOW = -12,   /* ErrIntOverflowShard (varint > 64 bits)      */
    RS_EWIRE_LENGTH = -13,     /* ErrInvalidLengthShard (negative length)     */
    RS_EWIRE_TYPE = -14,       /* wrong wireType / illegal tag / end group    */
    RS_EWIRE_SHORT = -15,      /* output buffer smaller than rs_shard_size()  */
};

typedef struct {
    const uint8_t *file_signature; /* field 1, bytes  */
    size_t file_signature_len;
    const uint8_t *shard_data;     /* field 2, bytes  */
    size_t shard_data_len;
    uint64_t shard_number;         /* field 3, uint64 */
    uint64_t total_shards;         /* field 4, uint64 */
    uint64_t minimum_needed_shards;/* field 5, uint64 */
} rs_shard_view;

/* (*Shard).Size() */
size_t rs_shard_size(const rs_shard_view *m);

/* (*Shard).MarshalTo(): writes rs_shard_size(m) bytes to out (cap bytes
 * available); *written receives the count. */
int rs_shard_marshal(const rs_shard_view *m, uint8_t *out, size_t cap, size_t *written);

/* (*Shard).Unmarshal(): parses buf[len]; on success the byte fields of *out
 * alias buf.  Absent fields are zero / empty. */
int rs_shard_unmarshal(const uint8_t *buf, size_t len, rs_shard_view *out);

struct rs_arena; /* rsmi.h */
/* Unmarshal that places ShardData in a 16-byte aligned slot of `arena`
 * (engine-pinned): the one copy gogo's Unmarshal makes anyway
 * (shard.pb.go:468-503, `append(m.ShardData[:0], ...)`) lands where
 * rs_decode_batch's kernel reads it in place.  FileSignature still aliases
 * buf.  RS_ENOMEM (rsmi.h) when the arena is full. */
int rs_shard_unmarshal_arena(const uint8_t *buf, size_t len, struct rs_arena *arena, rs_shard_view *out);

#ifdef __cplusplus
}
#endif
#endif /* RSMI_WIRE_H */
