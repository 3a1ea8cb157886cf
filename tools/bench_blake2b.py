#!/usr/bin/env python3
"""Batched BLAKE2b throughput (the plugin's sign /
verify hash of serializeMessage, main.go:219-223 / :82-89) on the GPU next to
Python hashlib (OpenSSL / libb2 BLAKE2b) on the host's cores.

Per batch shape (messages x bytes):
  * device: messages resident in HBM at 16-byte aligned offsets,
    rs_blake2b_device timed with HIP events on the launch stream (median of
    --reps), GB/s of message bytes;
  * host API: rs_blake2b_batch on pageable host messages (pinned staging,
    PCIe-inclusive), median wall time;
  * CPU: hashlib.blake2b over the same messages, 1 thread and every usable
    CPU (a thread pool; hashlib releases the GIL for messages > 2 KiB).
Digests are checked against hashlib for every shape.

    python tools/bench_blake2b.py [--reps 5] [--digest 32]
"""
import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

SHAPES = [(256, 1048620), (2048, 65536), (16384, 4096), (65536, 1024), (4, 1048620)]


def median_time(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--digest", type=int, default=32)
    a = ap.parse_args()
    import bench
    import rsmi

    info = bench.host_cpu_info()
    cpus = info["usable_cpus"]
    f = rsmi.FEC(10, 14)
    dl = a.digest
    out = {"digest_len": dl, "cpu_model": info["model"], "usable_cpus": cpus, "host_cpus": info["host_cpus"],
           "shapes": []}
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(5)
    for B, L in SHAPES:
        pitch = (L + 15) // 16 * 16
        host = rng.integers(0, 256, size=B * pitch, dtype=np.uint8)
        msgs = [host[i * pitch:i * pitch + L].tobytes() for i in range(B)]
        dev = torch.from_numpy(host).cuda()
        base = dev.data_ptr()
        ptrs = torch.tensor([base + i * pitch for i in range(B)], dtype=torch.int64, device="cuda")
        lens = torch.full((B,), L, dtype=torch.int64, device="cuda")
        dout = torch.zeros(B * dl, dtype=torch.uint8, device="cuda")
        run = lambda: f.blake2b_device(B, ptrs.data_ptr(), lens.data_ptr(), 0, dl, dout.data_ptr(),
                                       stream.cuda_stream)
        run()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run()
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        dev_ms = float(np.median(ms))
        got = dout.cpu().numpy().tobytes()
        want = [hashlib.blake2b(m, digest_size=dl).digest() for m in msgs]
        assert all(got[i * dl:(i + 1) * dl] == want[i] for i in range(B)), (B, L)
        host_s = median_time(lambda: f.blake2b_batch(msgs, dl), max(1, a.reps // 2))
        assert f.blake2b_batch(msgs, dl) == want
        cpu1 = median_time(lambda: [hashlib.blake2b(m, digest_size=dl).digest() for m in msgs], 1)
        with ThreadPoolExecutor(cpus) as ex:
            cpun = median_time(lambda: list(ex.map(lambda m: hashlib.blake2b(m, digest_size=dl).digest(), msgs,
                                                   chunksize=max(1, B // (4 * cpus)))), 2)
        tot = B * L
        out["shapes"].append({
            "messages": B, "bytes_each": L,
            "gpu_device_ms": round(dev_ms, 3), "gpu_device_GBps": round(tot / dev_ms / 1e6, 2),
            "gpu_host_api_ms": round(host_s * 1e3, 3), "gpu_host_api_GBps_pcie_inclusive": round(tot / host_s / 1e9, 2),
            "cpu_hashlib_1t_GBps": round(tot / cpu1 / 1e9, 2),
            f"cpu_hashlib_{cpus}t_GBps": round(tot / cpun / 1e9, 2),
        })
        print(json.dumps(out["shapes"][-1]), file=sys.stderr, flush=True)
        del dev, ptrs, lens, dout
    print(json.dumps(out))


if __name__ == "__main__":
    main()
