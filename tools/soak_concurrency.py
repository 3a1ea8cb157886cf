#!/usr/bin/env python3
"""Concurrency soak of one context (RS(64,16) by default; --code 10:14
--shard 104858 gives config-1-sized messages, whose host-API calls take the
two-chunk staged path) (SURVEY §8b threading): for
--seconds, T threads mix every C-ABI entry point that shares the context's
pattern cache -- rs_decode (host API), rs_decode_batch, rs_encode,
rs_encode_batch and rs_reconstruct_stripes on their own device stripes with fresh erasure
patterns -- with a small pattern cap (RSMI_PATTERN_CAP) so the cache is
evicted over and over while other threads read it.  Every result is checked
(host API against the input, device stripes against a clone).  Prints one
JSON line with call counts, evictions and failures.

    RSMI_PATTERN_CAP=2000 python tools/soak_concurrency.py [--seconds 60 --threads 8 --code K:N --shard S]
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
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--code", default="64:80")
    ap.add_argument("--shard", type=int, default=4096, help="shard bytes of thread 0 (thread t: + 16 t)")
    a = ap.parse_args()
    import rsmi
    from oracle import oracle

    lib = rsmi.load()
    k, n = (int(v) for v in a.code.split(":"))
    m = n - k
    f = rsmi.FEC(k, n)
    P = ctypes.c_void_p
    stop = time.time() + a.seconds
    counts = {"decode": 0, "decode_batch": 0, "encode": 0, "reconstruct_stripes": 0, "encode_batch": 0}
    failures = []
    lock = threading.Lock()

    def worker(tid):
        try:
            body(tid)
        except Exception as e:  # a thread that dies outside the checked loop is a failure too
            with lock:
                failures.append(f"thread {tid}: {e!r}")

    def body(tid):
        rng = np.random.default_rng(1000 + tid)
        S = a.shard + 16 * tid
        blob = oracle.splitmix_bytes(k * S, tid)
        par = np.zeros(m * S, dtype=np.uint8)
        assert lib.rs_encode(f.handle, P(blob.ctypes.data), k * S, P(par.ctypes.data)) == 0
        shard = lambda i: blob[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]
        stripes = 64
        Sd = (S + 15) // 16 * 16  # device stripes: 16-byte pitch (rs_encode_stripes)
        stream = torch.cuda.Stream()
        data = torch.empty(stripes * k * Sd, dtype=torch.uint8, device="cuda")
        parity = torch.empty(stripes * m * Sd, dtype=torch.uint8, device="cuda")
        f.fill_splitmix(data.data_ptr(), data.numel(), 77 + tid, stream.cuda_stream)
        f.encode_stripes(data.data_ptr(), k * Sd, parity.data_ptr(), m * Sd, Sd, Sd, stripes, stream.cuda_stream)
        stream.synchronize()
        d0, p0 = data.clone(), parity.clone()
        local = dict.fromkeys(counts, 0)
        it = 0
        while time.time() < stop:
            op = it % 5
            it += 1
            try:
                if op == 0:
                    lost = set(rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False).tolist())
                    keep = [i for i in range(n) if i not in lost][:k]
                    bufs = [np.ascontiguousarray(shard(i)) for i in keep]
                    out = np.zeros(k * S, dtype=np.uint8)
                    nums = (ctypes.c_int * k)(*keep)
                    ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
                    assert lib.rs_decode(f.handle, nums, ptrs, k, S, P(out.ctypes.data)) == 0
                    assert np.array_equal(out, blob)
                elif op == 1:
                    B = 6
                    keeps = []
                    for _ in range(B):
                        lost = set(rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False).tolist())
                        keeps.append([i for i in range(n) if i not in lost][:k])
                    bufs = [[np.ascontiguousarray(shard(i)) for i in kp] for kp in keeps]
                    outs = [np.zeros(k * S, dtype=np.uint8) for _ in range(B)]
                    cnts = (ctypes.c_int * B)(*[k] * B)
                    nums = (ctypes.c_int * (B * k))(*[i for kp in keeps for i in kp])
                    ptrs = (ctypes.c_void_p * (B * k))(*[b.ctypes.data for bl in bufs for b in bl])
                    dsts = (ctypes.c_void_p * B)(*[o.ctypes.data for o in outs])
                    st = (ctypes.c_int * B)()
                    assert lib.rs_decode_batch(f.handle, B, cnts, nums, ptrs, S, dsts, st) == 0
                    assert list(st) == [0] * B and all(np.array_equal(o, blob) for o in outs)
                elif op == 4:
                    B = 6
                    pars = [np.zeros(m * S, dtype=np.uint8) for _ in range(B)]
                    ins = (ctypes.c_void_p * B)(*[blob.ctypes.data] * B)
                    outs = (ctypes.c_void_p * B)(*[x.ctypes.data for x in pars])
                    st = (ctypes.c_int * B)()
                    assert lib.rs_encode_batch(f.handle, B, ins, k * S, outs, st) == 0
                    assert list(st) == [0] * B and all(np.array_equal(x, par) for x in pars)
                elif op == 2:
                    p2 = np.zeros(m * S, dtype=np.uint8)
                    assert lib.rs_encode(f.handle, P(blob.ctypes.data), k * S, P(p2.ctypes.data)) == 0
                    assert np.array_equal(p2, par)
                elif op == 3:
                    er = np.zeros((stripes, n), dtype=np.uint8)
                    for s in range(stripes):
                        er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
                    with torch.cuda.stream(stream):
                        mask = torch.from_numpy(er).to("cuda", non_blocking=False).bool()
                        data.view(stripes, k, Sd)[mask[:, :k]] = 0
                        parity.view(stripes, m, Sd)[mask[:, k:]] = 0
                    f.reconstruct_stripes(data.data_ptr(), k * Sd, parity.data_ptr(), m * Sd, Sd, Sd, stripes,
                                          er.tobytes(), stream.cuda_stream)
                    stream.synchronize()
                    assert torch.equal(data, d0) and torch.equal(parity, p0)
                local[list(counts)[op]] += 1
            except AssertionError as e:  # record and go on: one line at the end
                with lock:
                    failures.append(f"thread {tid} op {op} iteration {it}: {e!r}")
                if len(failures) > 20:
                    break
        with lock:
            for key, v in local.items():
                counts[key] += v

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
    # Process CPU time (every thread, user + system) over the soak: with the
    # engine's polled waits (rsmi::wait_event, RSMI_SYNC_SPIN_US /
    # RSMI_SYNC_SPINNERS / RSMI_SYNC_ADAPTIVE) against runs without polling,
    # the difference is what the polling costs.
    cpu0, wall0 = time.process_time(), time.time()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    cpu, wall = time.process_time() - cpu0, time.time() - wall0
    ncalls = sum(counts.values())
    print(json.dumps({"code": a.code, "shard": a.shard, "seconds": a.seconds, "threads": a.threads, "calls": counts,
                      "cpu_seconds": round(cpu, 2), "cpu_cores_busy": round(cpu / wall, 2),
                      "cpu_ms_per_call": round(1e3 * cpu / max(1, ncalls), 4),
                      "spin_env": {v: os.environ.get(v) for v in ("RSMI_SYNC_SPIN_US", "RSMI_SYNC_SPINNERS",
                                                                  "RSMI_SYNC_ADAPTIVE")},
                      "pattern_cap": os.environ.get("RSMI_PATTERN_CAP"), "evictions": f.pattern_evictions(),
                      "patterns": f.pattern_count(), "leases": f.stat(f.STAT_LEASES),
                      "failures": len(failures), "first_failures": failures[:5]}))
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
