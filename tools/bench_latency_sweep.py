#!/usr/bin/env python3
"""Latency per stripe batch of the device-resident batched API (SURVEY §8d
config 5: "report latency per stripe batch and GB/s"; BASELINE configs[4]'s
small-shard latency).

For RS(k, n) stripes of S-byte shards already in HBM, and batch sizes from
one stripe up, times with HIP events on the launch stream (median of --reps
after one warm-up):
  * encode:            rs_encode_stripes of the batch;
  * reconstruct (cached patterns): rs_reconstruct_stripes with random 1..m
    erasures per stripe whose patterns are already built (the same erasure
    set as a warm-up call) -- host lookup, descriptor upload and kernel;
  * reconstruct (new patterns): a fresh random erasure set every call, so
    the call also builds (GPU Gauss-Jordan) every pattern it meets.
GB/s counts algorithmic bytes ((k+m)*S encode, (k+e)*S reconstruct).  One
JSON line per code.

    python tools/bench_latency_sweep.py [--k 64 --n 80 --shard 65536]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--n", type=int, default=80)
    ap.add_argument("--shard", type=int, default=65536)
    ap.add_argument("--batches", default="1,2,4,8,16,32,64,128,256,512,1024,2048,4096,8192,16384")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import rsmi

    k, n, S = a.k, a.n, a.shard
    m = n - k
    batches = [int(b) for b in a.batches.split(",")]
    top = max(batches)
    dev = torch.device("cuda", 0)
    f = rsmi.FEC(k, n)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    data = torch.empty(top * k * S, dtype=torch.uint8, device=dev)
    parity = torch.empty(top * m * S, dtype=torch.uint8, device=dev)
    f.fill_splitmix(data.data_ptr(), data.numel(), 7, sh)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, top, sh)
    if bench.pattern_total(n, m) <= (1 << 20):
        f.prepare_patterns(m, sh)  # every pattern exists: "new" equals "cached" for such codes
    torch.cuda.synchronize(dev)
    rng = np.random.default_rng(0xE4A5)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1)

    rows = []
    for b in batches:
        enc = lambda: f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, b, sh)  # noqa: E731
        timed(enc)
        enc_ms = statistics.median(timed(enc) for _ in range(a.reps))
        fixed = bench.erasure_sets(rng, 1, b, n, 1, m)[0]
        fixed_b = fixed.tobytes()
        rec = lambda er: f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, b, er, sh)  # noqa: E731
        timed(lambda: rec(fixed_b))  # builds its patterns
        cached_ms = statistics.median(timed(lambda: rec(fixed_b)) for _ in range(a.reps))
        fresh_sets = [s.tobytes() for s in bench.erasure_sets(rng, a.reps, b, n, 1, m)]
        fresh_ms = statistics.median(timed(lambda s=s: rec(s)) for s in fresh_sets)
        rec_bytes = float(((k + fixed.sum(axis=1)) * S).sum())
        rows.append({"stripes": b, "encode_ms": round(enc_ms, 4),
                     "encode_GBps": round(b * (k + m) * S / (enc_ms / 1e3) / 1e9, 1),
                     "reconstruct_cached_ms": round(cached_ms, 4),
                     "reconstruct_cached_GBps": round(rec_bytes / (cached_ms / 1e3) / 1e9, 1),
                     "reconstruct_new_patterns_ms": round(fresh_ms, 4)})
        print(f"{b} stripes: encode {enc_ms:.4f} ms, reconstruct {cached_ms:.4f} ms cached / "
              f"{fresh_ms:.4f} ms new patterns", file=sys.stderr, flush=True)
    print(json.dumps({"code": f"RS({k},{n})", "shard_bytes": S, "reps": a.reps,
                      "encode_kernel": f.kernel_name(0), "reconstruct_kernel": f.kernel_name(1),
                      "timing": "HIP events on the launch stream around one call, median", "rows": rows}))


if __name__ == "__main__":
    main()
