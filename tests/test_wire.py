"""CPU: erasurecode.Shard wire codec (include/rsmi_wire.h via the C++ host
layer) against Python-protobuf golden vectors, plus the reference's own
gogo testgen checks restated (protobuf/shardpb_test.go): marshal/unmarshal
round trips of NewPopulatedShard-style messages (TestShardProto :22,
TestShardMarshalTo :56), Size (TestShardSize :167), and 100 random byte
mutations that must not crash the decoder (TestShardProto :45-53)."""
import hashlib
import json
import os
import random

import pytest

from rsmi import host as h
from oracle import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "shard_wire.json")


def cases():
    with open(GOLD) as f:
        return json.load(f)["cases"]


def build(c):
    if "data" in c:
        data = bytes.fromhex(c["data"])
    else:
        n, seed = c["data_splitmix"]
        data = oracle.splitmix_bytes(n, seed).tobytes()
    return h.Shard(bytes.fromhex(c["sig"]), data, c["num"], c["total"], c["need"])


@pytest.mark.parametrize("c", cases(), ids=lambda c: c["name"])
def test_marshal_matches_protobuf(c):
    s = build(c)
    wire = s.Marshal()
    assert s.Size() == c["size"] == len(wire)
    assert hashlib.sha256(wire).hexdigest() == c["wire_sha256"]
    if "wire" in c:
        assert wire.hex() == c["wire"]
    else:
        assert wire.hex().startswith(c["wire_prefix"])
    t = h.Shard()
    t.Unmarshal(wire)
    assert t == s


def populated(rng):
    return h.Shard(bytes(rng.randrange(256) for _ in range(rng.randrange(100))),
                   bytes(rng.randrange(256) for _ in range(rng.randrange(100))),
                   rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(32))


def test_shard_proto_roundtrip_and_mutation_fuzz():
    rng = random.Random(1234)
    for _ in range(200):
        p = populated(rng)
        d = bytearray(p.Marshal())
        msg = h.Shard()
        msg.Unmarshal(bytes(d))
        assert msg == p
        for _ in range(100):  # shardpb_test.go:45-53: must not panic
            if not d:
                break
            d[rng.randrange(len(d))] = rng.randrange(256)
        try:
            h.Shard().Unmarshal(bytes(d))
        except h.HostError:
            pass


def test_unknown_fields_skipped_and_last_wins():
    base = h.Shard(b"sig", b"data", 5, 14, 10).Marshal()
    extra = (bytes([0x30, 0x96, 0x01])                 # field 6 varint
             + bytes([0x3a, 0x03]) + b"xyz"            # field 7 bytes
             + bytes([0x45]) + b"\x01\x02\x03\x04"     # field 8 fixed32
             + bytes([0x49]) + b"\x00" * 8             # field 9 fixed64
             + bytes([0x53, 0x08, 0x01, 0x54]))        # field 10 group {field 1 varint}
    t = h.Shard()
    t.Unmarshal(base + extra + bytes([0x18, 0x07]))    # second shard_number wins
    assert (t.FileSignature, t.ShardData, t.ShardNumber, t.TotalShards,
            t.MinimumNeededShards) == (b"sig", b"data", 7, 14, 10)


@pytest.mark.parametrize("bad,code", [
    (b"\x0a\x05ab", -11),                    # truncated bytes -> io.ErrUnexpectedEOF
    (b"\x18" + b"\xff" * 10 + b"\x01", -12),  # varint over 64 bits -> ErrIntOverflowShard
    (b"\x0a" + b"\xff" * 9 + b"\x01", -13),   # negative length -> ErrInvalidLengthShard
    (b"\x08\x01", -14),                       # field 1 with wire type 0 -> wrong wireType
    (b"\x00\x01", -14),                       # field 0 -> illegal tag
    (b"\x0c", -14),                           # end group -> wiretype end group for non-group
    (b"\x1a\x01", -14),                       # field 3 as bytes -> wrong wireType
    (b"\x18", -11),                           # varint missing
    (b"\x45\x01", -11),                       # unknown fixed32 truncated
])
def test_unmarshal_errors(bad, code):
    with pytest.raises(h.HostError) as ei:
        h.Shard().Unmarshal(bad)
    assert ei.value.args[1] == code


def test_c_abi_views_alias_input():
    import ctypes
    import rsmi

    class View(ctypes.Structure):
        _fields_ = [("file_signature", ctypes.c_void_p), ("file_signature_len", ctypes.c_size_t),
                    ("shard_data", ctypes.c_void_p), ("shard_data_len", ctypes.c_size_t),
                    ("shard_number", ctypes.c_uint64), ("total_shards", ctypes.c_uint64),
                    ("minimum_needed_shards", ctypes.c_uint64)]

    lib = ctypes.CDLL(rsmi.LIB_PATH)
    wire = h.Shard(b"S" * 64, b"D" * 300, 9, 14, 10).Marshal()
    buf = ctypes.create_string_buffer(wire, len(wire))
    v = View()
    assert lib.rs_shard_unmarshal(buf, len(wire), ctypes.byref(v)) == 0
    base = ctypes.addressof(buf)
    assert v.file_signature == base + 2 and v.shard_data == base + 2 + 64 + 3
    assert (v.shard_data_len, v.shard_number, v.total_shards, v.minimum_needed_shards) == (300, 9, 14, 10)
    out = ctypes.create_string_buffer(len(wire))
    w = ctypes.c_size_t()
    assert lib.rs_shard_marshal(ctypes.byref(v), out, len(wire) - 1, ctypes.byref(w)) == -15
    assert lib.rs_shard_marshal(ctypes.byref(v), out, len(wire), ctypes.byref(w)) == 0
    assert out.raw[:w.value] == wire


def test_helpers():
    # main.go:276-302 framing
    pid = h.PeerID("tcp://localhost:3000", b"\x01\x02")
    s = h.serializeMessage(pid, b"msg")
    assert s == (len("tcp://localhost:3000")).to_bytes(4, "little") + b"tcp://localhost:3000" \
        + (2).to_bytes(4, "little") + b"\x01\x02" + b"msg"
    # main.go:303-335
    assert [h.largestPrimeFactors(v) for v in (1, 2, 12, 97, 1 << 20, 15, 49, 1048580)] == \
        [-1, 2, 3, 97, 2, 5, 7, 109]
