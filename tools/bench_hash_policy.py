#!/usr/bin/env python3
"""Host/GPU crossover of the BLAKE2b hash policy (rs_blake2b).

For each batch shape (messages x bytes): median wall time of the host path
(rs_blake2b_host, 1 thread and every usable CPU), the GPU path
(rs_blake2b_batch, pinned staging + kernel, PCIe-inclusive), and the policy
(rs_blake2b) with the side it took.  Then the plugin's prepareShards of the
config-1 blob: without a hash, hash alone (host), and with the hash policy
(hash on the host overlapping the GPU encode).  One JSON line.

    python tools/bench_hash_policy.py [--reps 7]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402

SHAPES = [(1, 1048620), (1, 65536), (2, 1048620), (4, 1048620), (16, 1048620), (64, 1048620), (256, 1048620),
          (4, 65536), (64, 65536), (512, 65536), (2048, 65536), (16, 4096), (256, 4096), (16384, 4096),
          (65536, 1024)]


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import bench
    import rsmi
    from rsmi import host as h

    info = bench.host_cpu_info()
    f = rsmi.FEC(10, 14)
    rng = np.random.default_rng(1)
    rows = []
    for B, L in SHAPES:
        msgs = [rng.integers(0, 256, size=L, dtype=np.uint8).tobytes() for _ in range(B)]
        ref = rsmi.blake2b_host(msgs, 32)
        assert f.blake2b_batch(msgs, 32) == ref
        got, where = f.blake2b(msgs, 32)
        assert got == ref
        reps = a.reps if B * L < (64 << 20) else 3
        t1 = med(lambda: rsmi.blake2b_host(msgs, 32, 1), reps)
        ta = med(lambda: rsmi.blake2b_host(msgs, 32, 0), reps)
        tg = med(lambda: f.blake2b_batch(msgs, 32), reps)
        tp = med(lambda: f.blake2b(msgs, 32), reps)
        best = min(ta, tg)
        rows.append({"messages": B, "bytes": L, "host_1t_ms": round(t1 * 1e3, 3), "host_all_ms": round(ta * 1e3, 3),
                     "gpu_ms": round(tg * 1e3, 3), "policy_ms": round(tp * 1e3, 3),
                     "policy_side": "gpu" if where else "host",
                     "policy_vs_best": round(tp / best, 3),
                     "host_1t_GBps": round(B * L / t1 / 1e9, 3)})
        print(json.dumps(rows[-1]), file=sys.stderr)
    # prepareShards of the config-1 blob (main.go:211-241)
    k, n = 10, 14
    blob = rng.integers(0, 256, size=1048580, dtype=np.uint8).tobytes()
    me = h.PeerID("tcp://localhost:3000", b"\x11" * 32)
    ser = h.serializeMessage(me, blob)
    p0 = h.NewShardPlugin(None, None, k, n)
    p1 = h.NewShardPlugin(lambda d: b"s" * 64, None, k, n, hash_len=32)
    prep = {
        "prepareShards_no_hash_ms": round(med(lambda: p0.prepareShards(me, blob), a.reps) * 1e3, 3),
        "host_hash_1t_ms": round(med(lambda: rsmi.blake2b_host([ser], 32, 1), a.reps) * 1e3, 3),
        "gpu_hash_ms": round(med(lambda: f.blake2b_batch([ser], 32), a.reps) * 1e3, 3),
        "prepareShards_hash_policy_ms": round(med(lambda: p1.prepareShards(me, blob), a.reps) * 1e3, 3),
    }
    print(json.dumps({"cpu_model": info["model"], "usable_cpus": info["usable_cpus"], "shapes": rows,
                      "config1_prepareShards": prep}))


if __name__ == "__main__":
    main()
