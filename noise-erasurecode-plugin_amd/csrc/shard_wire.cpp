// shard_wire.cpp -- erasurecode.Shard codec (include/rsmi_wire.h).
//
// Wire layout of protobuf/shard.proto:21-27 as gogo emits it
// (protobuf/shard.pb.go:219-252): tag 0x0a len FileSignature, 0x12 len
// ShardData, 0x18 varint ShardNumber, 0x20 varint TotalShards, 0x28 varint
// MinimumNeededShards; empty bytes and zero integers are omitted.
#include "../../include/rsmi_wire.h"

#include "../../include/rsmi.h"

#include <cstring>

namespace {

size_t varint_len(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++n;
    }
    return n;
}

uint8_t* put_varint(uint8_t* p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = static_cast<uint8_t>(v | 0x80);
        v >>= 7;
    }
    *p++ = static_cast<uint8_t>(v);
    return p;
}

// Reads a varint at buf[*pos]; Go's loop errors on a 10th+ byte whose shift
// reaches 64, and on running out of input.
int get_varint(const uint8_t* buf, size_t len, size_t* pos, uint64_t* out) {
    uint64_t v = 0;
    for (unsigned shift = 0;; shift += 7) {
        if (shift >= 64) return RS_EWIRE_OVERFLOW;
        if (*pos >= len) return RS_EWIRE_EOF;
        const uint8_t b = buf[(*pos)++];
        v |= static_cast<uint64_t>(b & 0x7F) << shift;
        if (b < 0x80) break;
    }
    *out = v;
    return 0;
}

// skipShard: size of the field starting at buf[start] (tag included).
int skip_field(const uint8_t* buf, size_t len, size_t start, size_t* out) {
    size_t pos = start;
    uint64_t wire;
    int rc = get_varint(buf, len, &pos, &wire);
    if (rc) return rc;
    switch (wire & 7) {
        case 0: {
            uint64_t tmp;
            rc = get_varint(buf, len, &pos, &tmp);
            if (rc) return rc;
            break;
        }
        case 1:
            pos += 8;
            break;
        case 2: {
            uint64_t l;
            rc = get_varint(buf, len, &pos, &l);
            if (rc) return rc;
            if (static_cast<int64_t>(l) < 0) return RS_EWIRE_LENGTH;  // Go int wraps negative
            pos += l;
            break;
        }
        case 3:  // start group: skip nested fields until the matching end group
            for (;;) {
                size_t inner = pos;
                uint64_t iw;
                rc = get_varint(buf, len, &inner, &iw);
                if (rc) return rc;
                if ((iw & 7) == 4) {
                    pos = inner;
                    break;
                }
                size_t n;
                rc = skip_field(buf, len, pos, &n);
                if (rc) return rc;
                pos += n;
            }
            break;
        case 4:
            break;
        case 5:
            pos += 4;
            break;
        default:
            return RS_EWIRE_TYPE;  // "proto: illegal wireType"
    }
    *out = pos - start;
    return 0;
}

}  // namespace

extern "C" {

size_t rs_shard_size(const rs_shard_view* m) {
    if (!m) return 0;
    size_t n = 0;
    if (m->file_signature_len) n += 1 + m->file_signature_len + varint_len(m->file_signature_len);
    if (m->shard_data_len) n += 1 + m->shard_data_len + varint_len(m->shard_data_len);
    if (m->shard_number) n += 1 + varint_len(m->shard_number);
    if (m->total_shards) n += 1 + varint_len(m->total_shards);
    if (m->minimum_needed_shards) n += 1 + varint_len(m->minimum_needed_shards);
    return n;
}

int rs_shard_marshal(const rs_shard_view* m, uint8_t* out, size_t cap, size_t* written) {
    if (!m || (!out && cap)) return -8;  // RS_EINVAL
    const size_t need = rs_shard_size(m);
    if (cap < need) return RS_EWIRE_SHORT;
    uint8_t* p = out;
    if (m->file_signature_len) {
        *p++ = 0x0a;
        p = put_varint(p, m->file_signature_len);
        std::memcpy(p, m->file_signature, m->file_signature_len);
        p += m->file_signature_len;
    }
    if (m->shard_data_len) {
        *p++ = 0x12;
        p = put_varint(p, m->shard_data_len);
        std::memcpy(p, m->shard_data, m->shard_data_len);
        p += m->shard_data_len;
    }
    if (m->shard_number) {
        *p++ = 0x18;
        p = put_varint(p, m->shard_number);
    }
    if (m->total_shards) {
        *p++ = 0x20;
        p = put_varint(p, m->total_shards);
    }
    if (m->minimum_needed_shards) {
        *p++ = 0x28;
        p = put_varint(p, m->minimum_needed_shards);
    }
    if (written) *written = static_cast<size_t>(p - out);
    return 0;
}

int rs_shard_unmarshal(const uint8_t* buf, size_t len, rs_shard_view* out) {
    if (!out || (!buf && len)) return -8;  // RS_EINVAL
    std::memset(out, 0, sizeof(*out));
    size_t pos = 0;
    while (pos < len) {
        const size_t pre = pos;
        uint64_t wire;
        int rc = get_varint(buf, len, &pos, &wire);
        if (rc) return rc;
        const int64_t field = static_cast<int32_t>(wire >> 3);
        const int wt = static_cast<int>(wire & 7);
        if (wt == 4) return RS_EWIRE_TYPE;      // end group for non-group
        if (field <= 0) return RS_EWIRE_TYPE;   // illegal tag
        if (field == 1 || field == 2) {
            if (wt != 2) return RS_EWIRE_TYPE;  // wrong wireType
            uint64_t l;
            rc = get_varint(buf, len, &pos, &l);
            if (rc) return rc;
            if (static_cast<int64_t>(l) < 0) return RS_EWIRE_LENGTH;
            if (l > len - pos) return RS_EWIRE_EOF;
            if (field == 1) {
                out->file_signature = buf + pos;
                out->file_signature_len = l;
            } else {
                out->shard_data = buf + pos;
                out->shard_data_len = l;
            }
            pos += l;
        } else if (field >= 3 && field <= 5) {
            if (wt != 0) return RS_EWIRE_TYPE;
            uint64_t v;
            rc = get_varint(buf, len, &pos, &v);
            if (rc) return rc;
            (field == 3 ? out->shard_number : field == 4 ? out->total_shards
                                                         : out->minimum_needed_shards) = v;
        } else {
            size_t n;
            rc = skip_field(buf, len, pre, &n);
            if (rc) return rc;
            if (n > len - pre) return RS_EWIRE_EOF;
            pos = pre + n;
        }
    }
    return 0;
}

int rs_shard_unmarshal_arena(const uint8_t* buf, size_t len, rs_arena* arena, rs_shard_view* out) {
    if (!arena) return RS_EINVAL;
    const int rc = rs_shard_unmarshal(buf, len, out);
    if (rc != 0 || out->shard_data_len == 0) return rc;
    void* slot = rs_arena_put(arena, out->shard_data, out->shard_data_len);  // streaming stores
    if (!slot) return RS_ENOMEM;
    out->shard_data = static_cast<const uint8_t*>(slot);
    return 0;
}

}  // extern "C"
