"""Lease-buffer growth under a HIP API trace.

8 threads on one RS(10,4) context call DecodeBatch and Decode with message
sizes that grow every call, so each call outgrows its lease's device
workspaces, pinned staging and pipeline slots.  Run under
`rocprofv3 --hip-trace --stats`: the HIP API summary shows how many
hipDeviceSynchronize / hipFree / hipHostFree calls the growth made (the
context's rs_free at exit accounts for one device sync and the final frees).
Prints one JSON line with the call counts and wall time."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402

import rsmi  # noqa: E402


def main():
    k, n = 10, 14
    f = rsmi.FEC(k, n)
    sizes = [4096 * (2 ** (i / 2)) for i in range(14)]  # 4 KiB .. ~360 KiB per shard
    calls = [0]
    lock = threading.Lock()

    def worker(t):
        rng = np.random.default_rng(t)
        for i, sz in enumerate(sizes):
            S = int(sz) // 16 * 16 + 16 * t
            raw = rng.integers(0, 256, size=k * S, dtype=np.uint8).tobytes()
            shares = [None] * n
            f.Encode(raw, lambda s: shares.__setitem__(s.Number, s.DeepCopy()))
            keep = rng.choice(n, size=k, replace=False).tolist()
            outs, st = f.DecodeBatch([[shares[x] for x in keep]] * (1 + i % 3))
            assert st == [0] * len(outs) and all(o == raw for o in outs)
            assert f.Decode(None, [shares[x] for x in keep]) == raw
            with lock:
                calls[0] += 3

    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    wall = time.perf_counter() - t0
    f.close()
    print(json.dumps({"threads": 8, "engine_calls": calls[0], "wall_s": round(wall, 3),
                      "max_shard_bytes": int(sizes[-1]) + 16 * 7}))


if __name__ == "__main__":
    main()
