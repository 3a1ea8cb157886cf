"""Generates tests/golden/shard_wire.json: erasurecode.Shard wire vectors
serialised by Python protobuf (7.x, installed in the build container) from a
descriptor restating protobuf/shard.proto:21-27 (proto3, package
erasurecode, fields 1 bytes file_signature, 2 bytes shard_data, 3 uint64
shard_number, 4 uint64 total_shards, 5 uint64 minimum_needed_shards).
Python protobuf emits fields in number order and omits proto3 defaults, the
same bytes gogo's MarshalTo produces (protobuf/shard.pb.go:219-252).
Random messages follow NewPopulatedShard (shard.pb.go:263-281): 0-99 random
bytes per bytes field, random uint32 per integer field.
    python tests/golden/make_wire_golden.py
"""
import hashlib
import json
import os
import random

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory


def shard_class():
    fd = descriptor_pb2.FileDescriptorProto(name="shard.proto", package="erasurecode",
                                            syntax="proto3")
    msg = fd.message_type.add(name="Shard")
    T = descriptor_pb2.FieldDescriptorProto
    for num, name, typ in [(1, "file_signature", T.TYPE_BYTES), (2, "shard_data", T.TYPE_BYTES),
                           (3, "shard_number", T.TYPE_UINT64), (4, "total_shards", T.TYPE_UINT64),
                           (5, "minimum_needed_shards", T.TYPE_UINT64)]:
        msg.field.add(name=name, number=num, type=typ, label=T.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("erasurecode.Shard"))


def main():
    Shard = shard_class()
    rng = random.Random(0x5EED)
    cases = []

    def add(name, sig, data, num, total, need):
        m = Shard(file_signature=sig, shard_data=data, shard_number=num, total_shards=total,
                  minimum_needed_shards=need)
        wire = m.SerializeToString()
        rec = {"name": name, "sig": sig.hex(), "num": num, "total": total, "need": need,
               "wire_sha256": hashlib.sha256(wire).hexdigest(), "size": len(wire)}
        if len(data) <= 4096:
            rec["data"] = data.hex()
            rec["wire"] = wire.hex()
        else:
            rec["data_splitmix"] = [len(data), 77]
            rec["wire_prefix"] = wire[:80].hex()
        cases.append(rec)

    add("empty", b"", b"", 0, 0, 0)
    add("plugin_default", bytes(range(64)), b"hello, world! __"[:4], 2, 6, 4)
    add("number_zero_omitted", b"\x00" * 64, b"ab", 0, 14, 10)
    add("max_u64", b"s", b"d", 2**64 - 1, 2**63, 2**32 + 5)
    add("varint_edges", b"x" * 127, b"y" * 128, 127, 128, 16383)
    for i in range(40):
        sig = bytes(rng.randrange(256) for _ in range(rng.randrange(100)))
        data = bytes(rng.randrange(256) for _ in range(rng.randrange(100)))
        add(f"populated_{i}", sig, data, rng.getrandbits(32), rng.getrandbits(32),
            rng.getrandbits(32))
    # 1 MiB-class shard (BASELINE config 1: S = 104,858 bytes of RS(10,4) on 1 MiB + 4)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from oracle import oracle
    data = oracle.splitmix_bytes(104858, 77).tobytes()
    add("config1_shard", b"\x00" * 64, data, 13, 14, 10)
    data = oracle.splitmix_bytes(1 << 20, 77).tobytes()
    add("one_mib_shard", b"\x00" * 64, data, 3, 14, 10)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "shard_wire.json")
    with open(out, "w") as f:
        json.dump({"note": "serialised by python protobuf from a descriptor restating "
                           "protobuf/shard.proto:21-27", "cases": cases}, f, indent=0)
    print("wrote", out, len(cases))


if __name__ == "__main__":
    main()
