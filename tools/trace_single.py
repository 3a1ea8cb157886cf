#!/usr/bin/env python3
"""Phase trace of one config-1 message's rs_encode / rs_decode (the bench's
configs[0] calls, pageable buffers, 4 seeded drops): run with RSMI_TRACE=1,
the engine prints mean microseconds per phase at exit (host_pipeline.cpp
trace_*).  Usage: RSMI_TRACE=1 python3 tools/trace_single.py {encode|decode} [reps]"""
import ctypes
import os
import sys
import time

if os.environ.get("RSMI_PIN_CPU"):  # before any HIP call: the calling thread's CPU (NUMA A/B runs)
    os.sched_setaffinity(0, {int(os.environ["RSMI_PIN_CPU"])})
elif os.environ.get("RSMI_PIN_GPU_NUMA"):  # the CPUs of the GPU's NUMA node, as bench.py runs
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
    import bench  # noqa: E402
    bench.torch.cuda.set_device(0)
    print("affinity", bench.pin_to_gpu_numa(0))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]
import numpy as np  # noqa: E402

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

what = sys.argv[1]  # encode | decode | decode_arena | encode_batch | decode_batch (64 messages per call)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
k, n = 10, 14
m = n - k
blob = np.concatenate([oracle.splitmix_bytes(1 << 20, 0x5EED), np.zeros(4, dtype=np.uint8)])
L = blob.size
S = L // k
lib = rsmi.load()
f = rsmi.FEC(k, n, device=0)
parity = np.zeros(m * S, dtype=np.uint8)
P = ctypes.c_void_p
lib.rs_encode(f.handle, P(blob.ctypes.data), L, P(parity.ctypes.data))
lost = sorted(int(v) for v in np.random.default_rng(0xC0F1).choice(n, size=4, replace=False))
keep = [i for i in range(n) if i not in lost]
bufs = [np.ascontiguousarray(blob[i * S:(i + 1) * S] if i < k else parity[(i - k) * S:(i - k + 1) * S]) for i in keep]
nums = (ctypes.c_int * k)(*keep)
ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
dst = np.zeros(L, dtype=np.uint8)
bp, pp, dp = P(blob.ctypes.data), P(parity.ctypes.data), P(dst.ctypes.data)
B = 64
if what == "decode_arena":  # the survivors in an engine-pinned rs_arena (read in place)
    arena = rsmi.Arena(k * (S + 256) + 4096)
    ptrs = (ctypes.c_void_p * k)(*[arena.put(b.tobytes()) for b in bufs])
if what.endswith("batch"):
    reps = max(5, reps // 20)
    rng = np.random.default_rng(0xBA7C)
    bkeeps = [sorted(set(range(n)) - set(int(v) for v in rng.choice(n, size=4, replace=False))) for _ in range(B)]
    base = {i: (blob.ctypes.data + i * S if i < k else parity.ctypes.data + (i - k) * S) for i in range(n)}
    bdst = [np.zeros(L, dtype=np.uint8) for _ in range(B)]
    bcounts = (ctypes.c_int * B)(*[k] * B)
    bnums = (ctypes.c_int * (B * k))(*[i for kp in bkeeps for i in kp])
    bptrs = (ctypes.c_void_p * (B * k))(*[base[i] for kp in bkeeps for i in kp])
    bout = (ctypes.c_void_p * B)(*[d.ctypes.data for d in bdst])
    emsgs = [np.ascontiguousarray(np.roll(blob, 4099 * b)) for b in range(B)]
    epar = [np.zeros(m * S, dtype=np.uint8) for _ in range(B)]
    eins = (ctypes.c_void_p * B)(*[x.ctypes.data for x in emsgs])
    eout = (ctypes.c_void_p * B)(*[x.ctypes.data for x in epar])
    bst = (ctypes.c_int * B)()
ts = []
for _ in range(reps):
    t0 = time.perf_counter()
    if what == "encode":
        lib.rs_encode(f.handle, bp, L, pp)
    elif what in ("decode", "decode_arena"):
        lib.rs_decode(f.handle, nums, ptrs, k, S, dp)
    elif what == "encode_batch":
        lib.rs_encode_batch(f.handle, B, eins, L, eout, bst)
    else:
        lib.rs_decode_batch(f.handle, B, bcounts, bnums, bptrs, S, bout, bst)
    ts.append(time.perf_counter() - t0)
if what in ("decode", "decode_arena"):
    assert np.array_equal(dst, blob)
if what == "decode_batch":
    assert all(np.array_equal(d, blob) for d in bdst)
per = B if what.endswith("batch") else 1
print(f"{what}: median {np.median(ts) * 1e6:.1f} us over {reps} calls ({np.median(ts) * 1e6 / per:.1f} us per message; "
      f"single-message drops {lost})")
try:  # where the calling thread ran (NUMA A/B runs)
    cpu = ctypes.CDLL(None).sched_getcpu()
    node = [d for d in os.listdir(f"/sys/devices/system/cpu/cpu{cpu}") if d.startswith("node")]
    print(f"cpu {cpu} {node[0] if node else 'node?'}")
except OSError:
    pass
