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
  decode_pinned_src rs_decode of 10 engine-pinned survivors (read in place)
                    into a pageable dst (outputs through staging)
  encode_tiny, decode_tiny   the same calls on 16-byte shards: the fixed cost
                    of a call (launch, completion, host bookkeeping)
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
    bp, pp = P(blob.ctypes.data), P(par.ctypes.data)
    out["encode_pageable"] = med(lambda: lib.rs_encode(f.handle, bp, L, pp), a.reps)
    keep = [1, 2, 3, 5, 7, 8, 9, 11, 12, 13]
    bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S])
            for i in keep]
    dst = np.zeros(L, dtype=np.uint8)

    # Share arrays built once per case (keep is sorted, so rs_decode's
    # in-place sort leaves them unchanged): no numpy .ctypes accesses inside
    # the timed calls.
    nums = (ctypes.c_int * k)(*keep)
    ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
    dptr = P(dst.ctypes.data)

    def dec():
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, dptr) == 0
    out["decode_pageable"] = med(dec, a.reps)
    assert np.array_equal(dst, blob)
    Sp = S // 16 * 16
    pin_in, pin_par = lib.rs_pinned_alloc(Sp * k), lib.rs_pinned_alloc(Sp * m)
    ctypes.memmove(pin_in, blob.ctypes.data, Sp * k)
    out["encode_pinned"] = med(lambda: lib.rs_encode(f.handle, pin_in, Sp * k, pin_par), a.reps)
    pin_dst = lib.rs_pinned_alloc(Sp * k)

    pptrs = (ctypes.c_void_p * k)(*[pin_in + i * Sp if i < k else pin_par + (i - k) * Sp for i in keep])

    def pdec():
        assert lib.rs_decode(f.handle, nums, pptrs, k, Sp, pin_dst) == 0
    out["decode_pinned"] = med(pdec, a.reps)
    assert ctypes.string_at(pin_dst, Sp * k) == ctypes.string_at(pin_in, Sp * k)
    lib.rs_pinned_free(pin_dst)
    pdst = np.zeros(Sp * k, dtype=np.uint8)

    pdptr = P(pdst.ctypes.data)

    def psdec():
        assert lib.rs_decode(f.handle, nums, pptrs, k, Sp, pdptr) == 0
    out["decode_pinned_src"] = med(psdec, a.reps)
    assert pdst.tobytes() == ctypes.string_at(pin_in, Sp * k)
    tb = blob[:16 * k].copy()
    tpar = np.zeros(16 * m, dtype=np.uint8)
    tbp, tpp = P(tb.ctypes.data), P(tpar.ctypes.data)
    out["encode_tiny"] = med(lambda: lib.rs_encode(f.handle, tbp, 16 * k, tpp), a.reps)
    tbufs = [np.ascontiguousarray(tb[i * 16:(i + 1) * 16] if i < k else tpar[(i - k) * 16:(i - k + 1) * 16]) for i in keep]
    tdst = np.zeros(16 * k, dtype=np.uint8)

    tptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in tbufs])
    tdptr = P(tdst.ctypes.data)

    def tdec():
        assert lib.rs_decode(f.handle, nums, tptrs, k, 16, tdptr) == 0
    out["decode_tiny"] = med(tdec, a.reps)
    assert np.array_equal(tdst, tb)
    x = torch.zeros(1, device="cuda")

    def ls():
        x.add_(1)
        torch.cuda.synchronize()
    out["launch_sync"] = med(ls, a.reps)
    pinned = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True).numpy()
    src = blob[:1 << 20]
    out["copy_1mib_1t"] = med(lambda: np.copyto(pinned, src), a.reps)
    E = oracle.fec_matrix(k, n)
    olib = oracle.lib()
    Ec = np.ascontiguousarray(E)
    ep = P(Ec.ctypes.data)
    out["cpu_avx2_encode"] = med(lambda: olib.orc_encode_batch(ep, k, n, bp, pp, S, 1, 1, 1), max(20, a.reps // 5))
    lib.rs_pinned_free(pin_in)
    lib.rs_pinned_free(pin_par)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
