#!/usr/bin/env python3
"""Aggregate host-API throughput of one rs_ctx under concurrent callers.

The reference's Receive runs once per peer connection, concurrently
(main.go:49-52), and the Go shim shares one context per (k, n).  T threads
each decode (rs_decode, 4 of 14 shards lost) or encode (rs_encode) their own
config-1-sized messages (1,048,580 B, RS(10,4)) on ONE context through
ctypes (the GIL is released inside each call).  Reported: messages/s and
GB/s ((k+m)*S bytes per message, PCIe-inclusive) for T = 1, 2, 4, 8, and
the speedup over T = 1.  Every output is checked against the input.

    python tools/bench_concurrency.py [--seconds 2] [--size 1048580]
Select another build with RSMI_LIB (same-box A/B); RSMI_MAX_LEASES=1
serialises the calls like the round-1 single-mutex context.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--size", type=int, default=(1 << 20) + 4)
    ap.add_argument("--threads", default="1,2,4,8")
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
    out = {"lib": rsmi.LIB_PATH, "max_leases": os.environ.get("RSMI_MAX_LEASES", "16"),
           "message_bytes": size, "k": k, "n": n}
    tmax = max(int(t) for t in a.threads.split(","))
    # per-thread message, parity, survivors and destination
    work = []
    for t in range(tmax):
        blob = oracle.splitmix_bytes(size, 77 + t)
        par = np.zeros(m * S, dtype=np.uint8)
        assert lib.rs_encode(f.handle, P(blob.ctypes.data), size, P(par.ctypes.data)) == 0
        lost = {(t + j * 3) % n for j in range(m)}
        keep = [i for i in range(n) if i not in lost][:k]
        bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S])
                for i in keep]
        work.append((blob, par, keep, bufs, np.zeros(size, dtype=np.uint8), np.zeros(m * S, dtype=np.uint8)))

    def run(op, T):
        stop = time.perf_counter() + a.seconds
        counts = [0] * T
        bad = []

        def body(t):
            blob, par, keep, bufs, dst, pout = work[t]
            while time.perf_counter() < stop:
                if op == "decode":
                    nums = (ctypes.c_int * k)(*keep)
                    ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
                    rc = lib.rs_decode(f.handle, nums, ptrs, k, S, P(dst.ctypes.data))
                else:
                    rc = lib.rs_encode(f.handle, P(blob.ctypes.data), size, P(pout.ctypes.data))
                if rc != 0:
                    bad.append(rc)
                    return
                counts[t] += 1
            if op == "decode" and not np.array_equal(dst, blob):
                bad.append("decode mismatch")
            if op == "encode" and not np.array_equal(pout, par):
                bad.append("encode mismatch")

        ths = [threading.Thread(target=body, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        assert not bad, bad[:3]
        msgs = sum(counts)
        return {"threads": T, "messages": msgs, "msgs_per_s": round(msgs / dt, 1),
                "GBps_pcie_inclusive": round(msgs * n * S / dt / 1e9, 2)}

    for op in ("decode", "encode"):
        run(op, 1)  # warm the leases
        rows = [run(op, int(T)) for T in a.threads.split(",")]
        base = rows[0]["msgs_per_s"]
        for r in rows:
            r["speedup_vs_1"] = round(r["msgs_per_s"] / base, 2)
        out[op] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
