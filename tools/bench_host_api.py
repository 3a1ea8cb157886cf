#!/usr/bin/env python3
"""Host-buffer (PCIe-inclusive) rates of the engine: the cgo path the plugin
uses (rs_encode / rs_decode: pageable host buffers, H2D, kernel, D2H) and
BASELINE config 1 end to end through the C++ ShardPlugin mirror, next to
the CPU oracle on the same inputs.  Not the bench.py headline (which is
device-resident); DESIGN.md quotes these as the PCIe-inclusive numbers.

    python tools/bench_host_api.py [--reps 20]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import rsmi
    from rsmi import host as h
    from oracle import oracle

    out = {}
    k, n = 10, 14
    f = rsmi.NewFEC(k, n)
    E = oracle.fec_matrix(k, n)
    for name, size in (("config1_blob_1MiB+4", (1 << 20) + 4), ("msg_64KiB", 65540),
                       ("msg_64MiB", 64 << 20), ("msg_640MiB", 640 << 20)):
        size -= size % k
        blob = oracle.splitmix_bytes(size, 1).tobytes()
        S = size // k
        t_enc = timeit(lambda: f.encode_parity(blob), a.reps if size < (100 << 20) else 3)
        shares = []
        f.Encode(blob, lambda s: shares.append(s.DeepCopy()))
        keep = [shares[i] for i in (13, 1, 9, 2, 12, 3, 11, 7, 5, 8)]  # 4 lost (0, 4, 6, 10)
        t_dec = timeit(lambda: f.Decode(None, list(keep)), a.reps if size < (100 << 20) else 3)
        assert f.Decode(None, list(keep)) == blob
        rec = {"bytes": size,
               "encode_ms": round(t_enc * 1e3, 3),
               "encode_GBps_pcie_inclusive": round(size * (n / k) / t_enc / 1e9, 2),
               "decode4_ms": round(t_dec * 1e3, 3),
               "decode4_GBps_pcie_inclusive": round(size * (n / k) / t_dec / 1e9, 2)}
        if size <= (64 << 20):
            t_cpu = timeit(lambda: oracle.encode(E, k, n, blob), 3)
            rec["cpu_oracle_scalar_encode_ms"] = round(t_cpu * 1e3, 3)
        out[name] = rec

    # config 1 through the plugin mirror: prepareShards -> Marshal -> drop 4 ->
    # Unmarshal -> Receive x10 -> Decode of the pooled shares.
    blob = oracle.splitmix_bytes(1 << 20, 0x5EED).tobytes() + b"\0" * 4
    me = h.PeerID("tcp://localhost:3000", b"\x11" * 32)
    sign = lambda m: hashlib.sha512(m).digest()  # ed25519 stand-in (out of scope)
    verify = lambda m, s: hashlib.sha512(m).digest() == s

    def config1():
        p = h.NewShardPlugin(sign, verify, k, n)
        wires = [s.Marshal() for s in p.prepareShards(me, blob)]
        recv = h.NewShardPlugin(sign, verify, k, n)
        got = []
        for i in (1, 2, 3, 5, 7, 8, 9, 11, 12, 13):
            s = h.Shard()
            s.Unmarshal(wires[i])
            recv.Receive(me, s)
            got.append(h.Share(int(s.ShardNumber), s.ShardData))
        msg, _ = h.NewFEC(k, n).Decode(None, got)
        assert msg == blob
    out["config1_plugin_end_to_end_ms"] = round(timeit(config1, a.reps) * 1e3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
