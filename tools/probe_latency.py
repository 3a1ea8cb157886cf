#!/usr/bin/env python3
"""Where a config-1 message's host-API time goes (one MI355X; diagnostics,
not a bench line).  Medians over --reps calls of:

  encode_pageable   rs_encode on caller-owned pageable buffers (the cgo path)
  decode_pageable   rs_decode of 10 survivors (4 seeded drops)
  encode_pinned     rs_encode with input and parity in engine-pinned memory
                    (16-byte shards: the kernel reads / writes them in place,
                    no staging copies) -- the GPU part alone
  decode_pinned     rs_decode of 10 engine-pinned survivors into a pinned dst
                    (read and written in place)
  launch_sync       an empty torch kernel + synchronize (launch + completion
                    latency floor)
  copy_1mib_1t      numpy copy of 1 MiB pageable -> pinned on one thread
  cpu_avx2_encode   the oracle's AVX2 encode on one thread (the reference
                    point of the config1 leg)

    python tools/probe_latency.py [--reps 300]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    import torch

    import rsmi
    from oracle import oracle
    k, n = 10, 14
    m = n - k
    lib = rsmi.load()
    f = rsmi.FEC(k, n, device=0)
    P = ctypes.c_void_p
    blob = np.concatenate([oracle.splitmix_bytes(1 << 20, 0x5EED), np.zeros(4, dtype=np.uint8)])
    L = blob.size
    S = L // k
    par = np.zeros(m * S, dtype=np.uint8)
    out = {"message_bytes": L, "env": {k_: v for k_, v in os.environ.items() if k_.startswith("RSMI_")}}
    out["encode_pageable"] = med(lambda: lib.rs_encode(f.handle, P(blob.ctypes.data), L, P(par.ctypes.data)), a.reps)
    keep = [1, 2, 3, 5, 7, 8, 9, 11, 12, 13]
    bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S])
            for i in keep]
    dst = np.zeros(L, dtype=np.uint8)

    def dec():
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(dst.ctypes.data)) == 0
    out["decode_pageable"] = med(dec, a.reps)
    assert np.array_equal(dst, blob)
    Sp = S // 16 * 16
    pin_in, pin_par = lib.rs_pinned_alloc(Sp * k), lib.rs_pinned_alloc(Sp * m)
    ctypes.memmove(pin_in, blob.ctypes.data, Sp * k)
    out["encode_pinned"] = med(lambda: lib.rs_encode(f.handle, pin_in, Sp * k, pin_par), a.reps)
    pin_dst = lib.rs_pinned_alloc(Sp * k)

    def pdec():
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[pin_in + i * Sp if i < k else pin_par + (i - k) * Sp for i in keep])
        assert lib.rs_decode(f.handle, nums, ptrs, k, Sp, pin_dst) == 0
    out["decode_pinned"] = med(pdec, a.reps)
    assert ctypes.string_at(pin_dst, Sp * k) == ctypes.string_at(pin_in, Sp * k)
    lib.rs_pinned_free(pin_dst)
    x = torch.zeros(1, device="cuda")

    def ls():
        x.add_(1)
        torch.cuda.synchronize()
    out["launch_sync"] = med(ls, a.reps)
    pinned = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True).numpy()
    src = blob[:1 << 20]
    out["copy_1mib_1t"] = med(lambda: np.copyto(pinned, src), a.reps)
    E = oracle.fec_matrix(k, n)
    out["cpu_avx2_encode"] = med(lambda: oracle.encode_batch(E, k, n, blob, S, 1, simd=True, threads=1, out=par),
                                 max(20, a.reps // 5))
    lib.rs_pinned_free(pin_in)
    lib.rs_pinned_free(pin_par)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
