#!/usr/bin/env python3
"""Per-message latency of the host API on the config-1 message (SURVEY §8d:
a 1,048,580-byte blob, RS(10,4), 4 data shards lost), the plugin's Receive
path (main.go:72-79): rs_encode and rs_decode with pageable buffers and with
engine-pinned ones (rs_pinned_alloc: in place over PCIe).  Median of --reps
calls; every decode is checked against the input.  Run under
`rocprofv3 --kernel-trace --hip-trace --stats` to split a call into its HIP
operations.

    python tools/bench_decode_latency.py [--reps 200] [--size 1048580]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--size", type=int, default=1048580)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=14)
    a = ap.parse_args()
    import rsmi
    from oracle import oracle

    lib = rsmi.load()
    k, n = a.k, a.n
    m = n - k
    size = a.size - a.size % k
    S = size // k
    f = rsmi.FEC(k, n)
    P = ctypes.c_void_p
    blob = oracle.splitmix_bytes(size, 1)
    out = {"k": k, "n": n, "message_bytes": size, "reps": a.reps}

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(ts), 4)

    # pageable
    par = np.zeros(m * S, dtype=np.uint8)
    dst = np.zeros(size, dtype=np.uint8)
    keep = list(range(m, n))  # first m data shards lost
    bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]) for i in keep]

    def enc():
        assert lib.rs_encode(f.handle, P(blob.ctypes.data), size, P(par.ctypes.data)) == 0

    enc()
    bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]) for i in keep]

    def dec():
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(dst.ctypes.data)) == 0

    out["encode_pageable_ms"] = timed(enc)
    out["decode4_pageable_ms"] = timed(dec)
    assert np.array_equal(dst, blob)
    # engine-pinned: input, parity and destination from rs_pinned_alloc
    pin_in, pin_par, pin_dst = lib.rs_pinned_alloc(size), lib.rs_pinned_alloc(m * S), lib.rs_pinned_alloc(size)
    try:
        ctypes.memmove(pin_in, blob.ctypes.data, size)

        def penc():
            assert lib.rs_encode(f.handle, P(pin_in), size, P(pin_par)) == 0

        def pdec():
            nums = (ctypes.c_int * k)(*keep)
            ptrs = (ctypes.c_void_p * k)(*[pin_in + i * S if i < k else pin_par + (i - k) * S for i in keep])
            assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(pin_dst)) == 0

        out["encode_pinned_ms"] = timed(penc)
        out["decode4_pinned_ms"] = timed(pdec)
        assert ctypes.string_at(pin_dst, size) == blob.tobytes()
    finally:
        for p in (pin_in, pin_par, pin_dst):
            lib.rs_pinned_free(p)
    out["stats"] = {"batches_in_place": f.stat(f.STAT_BATCHES_IN_PLACE), "encodes_in_place": f.stat(f.STAT_ENCODES_IN_PLACE)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
