#!/usr/bin/env python3
"""Per-message cost of the batched host-API calls against batch size (one
MI355X; diagnostics, not a bench line): config-1 messages (RS(10,4),
1,048,580 bytes, pageable) through rs_encode_batch and rs_decode_batch (4
seeded drops per message, survivors in the caller's pageable buffers), B =
1, 2, 4, 8, 16, 32, 64, 128 messages per call, medians of --reps calls, every
output checked once against the oracle; the oracle's AVX2 encode / decode on
one thread as the yardstick (decode: the mean over 16 messages' own drop
sets).  Prints one JSON line.

    python tools/bench_batch_sweep.py [--reps 15]
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


def median_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    import rsmi
    from oracle import oracle

    k, n = 10, 14
    m = n - k
    L = 1048580
    S = L // k
    lib = rsmi.load()
    f = rsmi.FEC(k, n)
    E = oracle.fec_matrix(k, n)
    bmax = 128
    msgs = [np.ascontiguousarray(oracle.splitmix_bytes(L, 100 + b)) for b in range(bmax)]
    pars = [np.frombuffer(oracle.encode(E, k, n, x.tobytes()), dtype=np.uint8) for x in msgs]
    rng = np.random.default_rng(0xBA7C)
    keeps = [sorted(set(range(n)) - set(int(v) for v in rng.choice(n, size=4, replace=False))) for _ in range(bmax)]

    def shard_ptr(b, i):
        return msgs[b].ctypes.data + i * S if i < k else pars[b].ctypes.data + (i - k) * S

    out = {"message_bytes": L, "reps": a.reps, "encode_ms_per_message": {}, "decode_ms_per_message": {}}
    for B in (1, 2, 4, 8, 16, 32, 64, 128):
        epar = [np.zeros(m * S, dtype=np.uint8) for _ in range(B)]
        ins = (ctypes.c_void_p * B)(*[msgs[b].ctypes.data for b in range(B)])
        outs = (ctypes.c_void_p * B)(*[p.ctypes.data for p in epar])
        st = (ctypes.c_int * B)()

        def enc():
            assert lib.rs_encode_batch(f.handle, B, ins, L, outs, st) == 0

        out["encode_ms_per_message"][B] = round(median_ms(enc, a.reps) / B, 4)
        assert all(np.array_equal(epar[b], pars[b]) for b in range(B))
        dsts = [np.zeros(L, dtype=np.uint8) for _ in range(B)]
        cnts = (ctypes.c_int * B)(*[k] * B)
        nums = (ctypes.c_int * (B * k))(*[i for b in range(B) for i in keeps[b]])
        ptrs = (ctypes.c_void_p * (B * k))(*[shard_ptr(b, i) for b in range(B) for i in keeps[b]])
        dd = (ctypes.c_void_p * B)(*[d.ctypes.data for d in dsts])

        def dec():
            assert lib.rs_decode_batch(f.handle, B, cnts, nums, ptrs, S, dd, st) == 0

        out["decode_ms_per_message"][B] = round(median_ms(dec, a.reps) / B, 4)
        assert all(np.array_equal(dsts[b], msgs[b]) for b in range(B))
        print(f"B={B}: encode {out['encode_ms_per_message'][B]} ms, decode {out['decode_ms_per_message'][B]} ms "
              "per message", file=sys.stderr, flush=True)
    # one AVX2 core: encode of one message, decode = present shares copied + Rebuild
    olib = oracle.lib()
    P = ctypes.c_void_p
    Ec = np.ascontiguousarray(E)
    par = np.zeros(m * S, dtype=np.uint8)
    blob = msgs[0]
    out["cpu_avx2_1t_encode_ms"] = round(median_ms(
        lambda: olib.orc_encode_batch(P(Ec.ctypes.data), k, n, P(blob.ctypes.data), P(par.ctypes.data), S, 1, 1, 1),
        a.reps), 4)
    # decode: the mean over the first 16 messages' own drop sets (the number of
    # lost data shards, hence the CPU's work, varies with the set)
    dec_ms = []
    for b in range(16):
        lost = [i for i in range(k) if i not in keeps[b]]
        er = np.zeros((1, n), dtype=np.uint8)
        er[0, lost] = 1
        dst = np.zeros(L, dtype=np.uint8)
        src = msgs[b]
        pb = pars[b].copy()
        present = [i for i in range(k) if i not in lost]

        def cpu_dec():
            for i in present:
                ctypes.memmove(dst.ctypes.data + i * S, src.ctypes.data + i * S, S)
            return olib.orc_reconstruct_batch(P(Ec.ctypes.data), k, n, P(dst.ctypes.data), P(pb.ctypes.data), S, 1,
                                              P(er.ctypes.data), 1, 1)

        dec_ms.append(median_ms(cpu_dec, max(3, a.reps // 3)))
        assert np.array_equal(dst, src)
    out["cpu_avx2_1t_decode_ms"] = round(float(np.mean(dec_ms)), 4)
    out["encode_vs_1core"] = {B: round(out["cpu_avx2_1t_encode_ms"] / v, 3) for B, v in out["encode_ms_per_message"].items()}
    out["decode_vs_1core"] = {B: round(out["cpu_avx2_1t_decode_ms"] / v, 3) for B, v in out["decode_ms_per_message"].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
