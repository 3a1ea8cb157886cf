#!/usr/bin/env python3
"""Host cost of the pattern cache on fresh-pattern reconstructs.

A batched reconstruct looks up every stripe's erasure pattern; patterns not
cached are created on the host (Rebuild's survivor choice, descriptor rows)
and built on the GPU (invert_patterns_kernel) inside the call.  With a fresh
random pattern per stripe -- SURVEY §8d config 5 -- that host work is on the
critical path of a reconstruct-only step.  This tool times, for RS(k, n)
stripes with small shards (so the coding kernel is short):
  * call_ms:  wall time of rs_reconstruct_stripes returning (host work +
              enqueue; the GPU runs asynchronously),
  * step_ms:  the same plus the stream draining,
for (a) a fresh erasure set every call and (b) the same set again (every
pattern cached: lookups only).  Median of --reps calls after one warm-up.

    python tools/bench_patterns.py [--k 64 --n 80 --stripes 16384 --shard 4096]
Select another build with RSMI_LIB (same-box A/B).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--n", type=int, default=80)
    ap.add_argument("--stripes", type=int, default=16384)
    ap.add_argument("--shard", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    import rsmi

    k, n, S, st = a.k, a.n, a.shard, a.stripes
    m = n - k
    dev = torch.device("cuda", 0)
    f = rsmi.FEC(k, n)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    data = torch.empty(st * k * S, dtype=torch.uint8, device=dev)
    parity = torch.empty(st * m * S, dtype=torch.uint8, device=dev)
    f.fill_splitmix(data.data_ptr(), data.numel(), 5, sh)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, st, sh)
    rng = np.random.default_rng(0xE4A5)
    sets = [s.tobytes() for s in bench.erasure_sets(rng, a.reps + 1, st, n, 1, m)]

    def run(erased):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, st, erased, sh)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t0) * 1e3

    run(sets[0])
    fresh = [run(s) for s in sets[1:]]
    cached = [run(sets[-1]) for _ in range(a.reps)]
    med = lambda xs, i: round(statistics.median(x[i] for x in xs), 3)
    out = {"lib": rsmi.LIB_PATH, "k": k, "n": n, "stripes": st, "shard_bytes": S,
           "fresh": {"call_ms": med(fresh, 0), "step_ms": med(fresh, 1),
                     "host_ns_per_stripe": round(med(fresh, 0) * 1e6 / st, 1)},
           "cached": {"call_ms": med(cached, 0), "step_ms": med(cached, 1),
                      "host_ns_per_stripe": round(med(cached, 0) * 1e6 / st, 1)},
           "patterns": f.pattern_count(), "evictions": f.pattern_evictions()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
