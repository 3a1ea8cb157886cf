#!/usr/bin/env python3
"""Diagnostics: one-stripe rs_reconstruct_stripes calls (RS(10,4), 1 MiB
shards, cached patterns) back to back, timed on the host and with HIP events,
for a rocprofv3 --hip-trace run that places the call's API calls and kernel
on one timeline.

    python tools/probe_rec_small.py [--reps 200]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    import rsmi
    k, n, S = 10, 14, 1 << 20
    m = n - k
    f = rsmi.FEC(k, n)
    st = torch.cuda.Stream()
    data = torch.empty(k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 5, st.cuda_stream)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, 1, st.cuda_stream)
    er = np.zeros((1, n), dtype=np.uint8)
    er[0, [1, 6, 11, 13]] = 1
    erb = er.tobytes()
    out = {}
    for name, fn in (("encode", lambda: f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, 1,
                                                          st.cuda_stream)),
                     ("reconstruct", lambda: f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S,
                                                                    S, S, 1, erb, st.cuda_stream))):
        fn()
        st.synchronize()
        host, ev = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            fn()
            t1 = time.perf_counter()
            e1.record(st)
            st.synchronize()
            host.append((t1 - t0) * 1e3)
            ev.append(e0.elapsed_time(e1))
        out[name] = {"host_call_ms": round(statistics.median(host), 4), "event_ms": round(statistics.median(ev), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
