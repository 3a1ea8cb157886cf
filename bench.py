#!/usr/bin/env python3
"""RS(10,4) encode + reconstruct throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over the whole per-GPU batch, device
resident (inputs already in HBM when the timed region starts):
  1. rs_encode_stripes: parity of every stripe (configs[1]: 6,553 stripes x
     10 x 1 MiB shards = 64 GiB of data per GPU), and
  2. rs_reconstruct_stripes: every stripe loses 1-4 random shards (uniform
     count, uniform positions; a fresh erasure set per step, seed 0xE4A5),
     which are regenerated in place (configs[2]), including the host-side
     per-stripe pattern lookup and the stripe->pattern upload.
value = algorithmic bytes of all steps on all ranks / max-over-ranks time,
where encode moves (k+m)*S per stripe and reconstruct (k+e)*S.

Multi-GPU (configs[3], stripe-local placement): each rank owns its own
stripes (stripe s of the global job -> rank s mod N), no collective on the
data path -> weak scaling.  The driver launches N>1 with torch.distributed.run.

Also reported: the roofline of the dominant kernel (encode, HIP events on the
launch stream) against the 8 TB/s HBM3E peak, and the CPU baseline (the
oracle's ports of infectious's scalar and split-nibble addmul, 1 thread and
all usable CPUs, on a bounded sample of the same workload, on rank 0 after
the timed region at every N).  At N = 1 two more legs follow, never part of
value: "config1" (configs[0], the reference's one-call-per-message pattern on
the 1,048,580-byte blob, median latencies next to the oracle on one core) and
"config5" (configs[4], RS(64,16) with 64 KiB shards, fresh 1-16 erasures).

`--gpus N` with N > 1 and no launcher starts N ranks itself
(torch.distributed.run as a child process, the JSON line relayed); under a
launcher, WORLD_SIZE must equal --gpus.  At N > 1 the same ranks then run a
short shard-distributed leg (configs[3]: the RCCL survivor gather and the
pointer-mode reconstruct, the last two steps checked on a sample) reported
as "gather" -- never part of value.  A per-rank watchdog abandons a leg stuck
in a collective: the headline line is still printed, then the ranks exit
with EXIT_GATHER_ABANDONED (75), so a hung gather never reads as success.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
# Exit status of a rank whose N > 1 gather leg was abandoned by its watchdog
# (a collective that never completed): the headline line is printed first,
# but the run must not read as a success.
EXIT_GATHER_ABANDONED = 75


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--shard", type=int, default=1 << 20, help="shard bytes S")
    ap.add_argument("--stripes", type=int, default=6553, help="stripes per GPU")
    ap.add_argument("--emin", type=int, default=1)
    ap.add_argument("--emax", type=int, default=None)
    ap.add_argument("--mode", choices=["both", "encode", "reconstruct"], default="both")
    ap.add_argument("--placement", choices=["local", "sharded"], default="local",
                    help="local: stripe s on rank s mod N (headline). sharded: shard i of "
                         "every stripe on rank i mod N; a step gathers each stripe's k "
                         "survivors to its owner over RCCL, then reconstructs (configs[3])")
    ap.add_argument("--pattern-pool", type=int, default=0,
                    help="draw per-stripe erasures from this many distinct patterns "
                         "(0: every stripe independent; new patterns are inverted on the "
                         "GPU inside the timed step)")
    ap.add_argument("--erase", default=None,
                    help="fixed erased shard ids for every stripe, e.g. 0,1,2,3 (default random)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the CPU baseline sample, timed on rank 0 at N = 1 only (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this job may use (affinity and cgroup quota)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--stream", action="store_true",
                    help="configs[1] second mode: the stripes stream from pinned host memory "
                         "(H2D data, encode, D2H parity per chunk, two HIP streams); "
                         "PCIe-inclusive, never the headline")
    ap.add_argument("--stream-chunk", type=int, default=32, help="stripes per streamed chunk")
    ap.add_argument("--chunks", type=int, default=8,
                    help="sharded placement: exchange chunks per step (two chunks' buffers live)")
    ap.add_argument("--gather-stripes", type=int, default=512,
                    help="N > 1, local placement: after the timed region (and the CPU baseline), "
                         "a short shard-distributed leg with this many owned stripes per rank "
                         "runs the RCCL survivor gather + pointer reconstruct and checks it "
                         "(configs[3]); reported as 'gather', never 'value'. 0 disables")
    ap.add_argument("--gather-timeout", type=float, default=180.0,
                    help="seconds after which a stuck gather leg is abandoned (the line is still printed, "
                         f"then the ranks exit {EXIT_GATHER_ABANDONED})")
    ap.add_argument("--device-set-stripes", type=int, default=512,
                    help="N = 1: stripes per member of the device-set leg (a child process: one rs_new_devices "
                         "context over every visible GPU, [0, 0] on a one-GPU box; never value); 0 skips")
    ap.add_argument("--device-set-timeout", type=float, default=240.0)
    ap.add_argument("--device-set-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-extra-legs", dest="extra_legs", action="store_false",
                    help="N = 1: skip the configs[0] (per-message latency), configs[4] (RS(64,16)) and "
                         "configs[2] worst-case legs reported beside the headline")
    ap.add_argument("--config1-reps", type=int, default=200)
    ap.add_argument("--config5-stripes", type=int, default=16384)
    ap.add_argument("--config5-steps", type=int, default=5)
    ap.add_argument("--config5-warmup", type=int, default=2)
    ap.add_argument("--config3-steps", type=int, default=3,
                    help="N = 1: steps of the configs[2] worst-case leg (4 data erasures in every stripe; 0 skips)")
    return ap.parse_args()


def erasure_sets(rng, count, stripes, n, emin, emax, pool=0):
    """`count` arrays of per-stripe erasure flags: e uniform in [emin, emax],
    positions uniform without replacement; with pool > 0 every stripe takes
    one of `pool` such patterns (drawn once)."""
    def draw(rows):
        er = np.zeros((rows, n), dtype=np.uint8)
        es = rng.integers(emin, emax + 1, size=rows)
        for s in range(rows):
            er[s, rng.choice(n, size=int(es[s]), replace=False)] = 1
        return er
    if pool > 0:
        pats = draw(pool)
        return [pats[rng.integers(0, pool, size=stripes)] for _ in range(count)]
    return [draw(stripes) for _ in range(count)]


def pattern_total(n, emax):
    from math import comb
    return sum(comb(n, e) for e in range(1, emax + 1))


def job_totals(per_rank):
    """(job seconds, job bytes) from the all-gathered per-rank rows
    [seconds, ..., bytes]: the slowest rank's time and every rank's own
    algorithmic bytes summed (value = bytes / seconds)."""
    return max(r[0] for r in per_rank), sum(r[-1] for r in per_rank)


def host_cpu_info():
    """CPU model, the machine's logical CPUs, and the CPUs this process may
    use (affinity mask, then the cgroup quota: the GPU box gives a job a
    share of a large host)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    if quota:
        usable = min(usable, quota)
    return {"model": model, "host_cpus": total, "usable_cpus": usable, "cgroup_quota_cpus": quota}


def _cpu_leg(oracle, E, k, n, S, seconds, threads, simd, rng):
    """Encode + 1..m-erasure reconstruct batches of `threads` stripes for
    `seconds`; returns (GB/s over algorithmic bytes, stripes, busy s)."""
    m = n - k
    batch = max(threads, 1)
    data = oracle.splitmix_bytes(batch * k * S, 0xC0FFEE)
    parity = np.ones(batch * m * S, dtype=np.uint8)  # touched: no page faults in the loop
    done_bytes = 0
    stripes_done = 0
    busy = 0.0
    while busy < seconds:
        er = erasure_sets(rng, 1, batch, n, 1, m)[0]
        a = time.perf_counter()
        oracle.encode_batch(E, k, n, data, S, batch, simd=simd, threads=threads, out=parity)
        rc = oracle.reconstruct_batch(E, k, n, data, parity, S, batch, er, simd=simd, threads=threads)
        busy += time.perf_counter() - a
        assert rc == 0
        done_bytes += batch * (k + m) * S + int(((k + er.sum(axis=1)) * S).sum())
        stripes_done += batch
    return done_bytes / busy / 1e9, stripes_done, busy


def cpu_baseline(k, n, S, seconds, threads):
    """The oracle (oracle/rs_oracle.c, a C restatement of infectious) on a
    bounded sample of the same workload: batches of RS(k, n) stripes with
    S-byte shards, each batch encoded and then reconstructed from 1..m random
    erasures (Rebuild per stripe), pthreads over stripes, the GPU line's
    algorithmic byte accounting.  Four legs share `seconds`: infectious's
    generic scalar mul_table addmul and its amd64 split-nibble (PSHUFB, here
    AVX2) addmul, each on 1 thread and on every CPU this job may use.
    value = the all-CPU AVX2 leg."""
    from oracle import oracle

    info = host_cpu_info()
    allc = threads or info["usable_cpus"]
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(0xE4A5)
    legs = {}
    samples = []
    for name, simd, thr in (("scalar_1t", False, 1), ("scalar_all", False, allc),
                            ("avx2_1t", True, 1), ("avx2_all", True, allc)):
        gbps, st, busy = _cpu_leg(oracle, E, k, n, S, seconds / 4, thr, simd, rng)
        legs[name] = {"GBps": round(gbps, 3), "threads": thr, "stripes": st, "seconds": round(busy, 2)}
        samples.append(f"{name}: {st} stripes")
    return {
        "value": legs["avx2_all"]["GBps"],
        "unit": "GB/s",
        "cores": allc,
        "kind": "port",
        "cpu_model": info["model"],
        "host_cpus": info["host_cpus"],
        "usable_cpus": info["usable_cpus"],
        "cgroup_quota_cpus": info["cgroup_quota_cpus"],
        "legs": legs,
        "sample": f"RS({k},{n}) stripes of {S} B shards, encode + 1-{n - k}-erasure reconstruct "
                  f"(oracle/rs_oracle.c: scalar mul_table and AVX2 split-nibble addmul), "
                  f"1 thread and {allc} threads (all CPUs this job may use; the host has "
                  f"{info['host_cpus']}): " + ", ".join(samples),
    }


def stats_device(dev):
    """Where the per-rank statistics are all-gathered: the GPU under RCCL,
    host memory under the gloo rehearsal backend."""
    return dev if os.environ.get("RSMI_BENCH_BACKEND", "nccl") == "nccl" else torch.device("cpu")


# The one JSON line goes to the real stdout; everything else written to fd 1
# (RCCL's init banner, library prints) is sent to stderr so a driver reading
# stdout sees only that line.
_RESULT_OUT = None


def emit(obj):
    out = _RESULT_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(gpus: int, argv, port: int):
    """The torch.distributed.run command that runs this script as `gpus`
    ranks on this node (one per GPU), with every flag passed through."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__)] + list(argv)


def check_world(gpus: int, env=None):
    """How this process should run for `--gpus gpus`:
      "single": one process, no launcher (N = 1);
      "launch": no launcher set RANK and N > 1 -> start N ranks as a child;
      "rank":   started by a launcher whose WORLD_SIZE matches --gpus.
    A launcher world that disagrees with --gpus is an error (SystemExit 2),
    so a record can never claim N GPUs while running another count."""
    env = os.environ if env is None else env
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" in env or "RANK" in env:
        world = int(env.get("WORLD_SIZE", "1"))
        if world != gpus:
            sys.stderr.write(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {gpus}\n")
            raise SystemExit(2)
        return "rank"
    return "launch" if gpus > 1 else "single"


def self_launch(gpus: int, argv) -> int:
    """Runs N ranks under torch.distributed.run as a child process (never an
    exec: this process has not touched the GPU, and must not replace itself
    after any process has) and relays the one JSON line rank 0 prints.
    Returns the child's exit code."""
    import subprocess
    cmd = launch_command(gpus, argv, _free_port())
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.stderr.write("bench.py: launching " + " ".join(cmd) + "\n")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = 0
    for line in proc.stdout:
        if line.lstrip().startswith("{"):
            sys.stdout.write(line)
            sys.stdout.flush()
            lines += 1
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and lines != 1:
        sys.stderr.write(f"bench.py: expected one JSON line from rank 0, got {lines}\n")
        return 1
    return rc


def device_run(f, k, n, S, stripes, steps, warmup, ersets, do_enc, do_rec, dev, seed=0x5EED,
               prepare_emax=None, distributed=False):
    """The device-resident hot path: `stripes` stripes of RS(k, n) with
    S-byte shards allocated and filled in HBM (splitmix64, untimed), then
    `warmup` untimed and `steps` timed steps, each = rs_encode_stripes of
    every stripe and/or rs_reconstruct_stripes with that step's erasure
    flags (ersets[i], host -> pattern lookup and upload inside the step).
    Timed region bracketed by synchronize (+ barrier when distributed); HIP
    events on the launch stream time each kernel.  The buffers are freed
    before returning.  When every pattern of <= prepare_emax erasures fits
    the ctx cache they are built before timing (prep_ms)."""
    m = n - k
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device=dev)
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device=dev)
    f.fill_splitmix(data.data_ptr(), data.numel(), seed, sh)
    f.fill_splitmix(parity.data_ptr(), parity.numel(), 1, sh)
    prep_ms = None
    if prepare_emax is not None and pattern_total(n, prepare_emax) <= (1 << 20):
        # Every pattern inverted on the GPU + uploaded once, before timing (a
        # context keeps them cached for its lifetime); its one-off cost is
        # reported as breakdown.pattern_prepare_ms.
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        f.prepare_patterns(prepare_emax, sh)
        torch.cuda.synchronize(dev)
        prep_ms = (time.perf_counter() - tp) * 1e3
    if not do_enc:  # reconstruct needs valid parity once
        f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, sh)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(steps)]

    def step(i, timed):
        e = ev[i - warmup] if timed else None
        if e:
            e[0].record(stream)
        if do_enc:
            f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, sh)
        if e:
            e[1].record(stream)
        if do_rec:
            f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                                  ersets[i].tobytes(), sh)
        if e:
            e[2].record(stream)

    for i in range(warmup):
        step(i, False)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(i, True)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    res = {"elapsed": elapsed, "encode_ms": [a.elapsed_time(b) for a, b, _ in ev],
           "reconstruct_ms": [b.elapsed_time(c) for _, b, c in ev], "prep_ms": prep_ms}
    del data, parity
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return res


def guarded_leg(fn):
    """Runs an extra (non-headline) leg; a failure is reported in the line
    instead of costing the headline measurement."""
    try:
        return fn()
    except Exception as e:  # reported, never silent
        return {"status": f"error: {type(e).__name__}: {e}"}


def _median_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e3, 4)


def config1_leg(local, reps=50):
    """configs[0]: the reference's own per-message call pattern.  The
    1,048,580-B blob (1 MiB of splitmix64 bytes zero-padded to a multiple
    of k = 10) is encoded once per call the way
    shardInput does (main.go:243-267) and decoded from 10 of its 14 shares
    after 4 seeded drops the way Receive does (main.go:72-79).  Timed as the
    median of `reps` calls:
      * codec: rs_encode / rs_decode at the C ABI on caller-owned pageable
        buffers (what the cgo shim hands over; PCIe-inclusive);
      * plugin: the C++ ShardPlugin mirror timed in C++
        (host/plugin_latency.cpp, no binding in the timed region):
        prepareShards into 14 Shards, those Shards marshalled the way
        net.Broadcast sends them, ShardAndBroadcastWire (marshalled straight
        from the encode output), and the 10 surviving Shards received
        (pooled) plus an 11th arrival that decodes the pool (with m = 4 lost
        the reference never gets a k+1-th shard, main.go:65-72: a resent
        survivor plays it);
      * cpu: the oracle on 1 thread for the same blob (scalar mul_table and
        AVX2 split-nibble addmul: encode, and Rebuild of the dropped data
        shards).
    Outputs are checked against the oracle / the blob."""
    import ctypes

    import rsmi
    from oracle import oracle
    from rsmi import host as h

    k, n = 10, 14
    m = n - k
    blob_np = np.concatenate([oracle.splitmix_bytes(1 << 20, 0x5EED), np.zeros(4, dtype=np.uint8)])
    L = blob_np.size
    S = L // k
    lib = rsmi.load()
    f = rsmi.FEC(k, n, device=local)
    P = ctypes.c_void_p
    parity = np.zeros(m * S, dtype=np.uint8)
    bptr, pptr = P(blob_np.ctypes.data), P(parity.ctypes.data)
    enc_ms = _median_ms(lambda: lib.rs_encode(f.handle, bptr, L, pptr), reps)
    E = oracle.fec_matrix(k, n)
    ref_par = np.frombuffer(oracle.encode(E, k, n, blob_np.tobytes()), dtype=np.uint8)
    if not np.array_equal(parity, ref_par):
        raise RuntimeError("config1: rs_encode parity differs from the oracle")
    rng = np.random.default_rng(0xC0F1)
    lost = sorted(int(v) for v in rng.choice(n, size=4, replace=False))
    keep = [i for i in range(n) if i not in lost]
    shard = lambda i: blob_np[i * S:(i + 1) * S] if i < k else parity[(i - k) * S:(i - k + 1) * S]
    bufs = [np.ascontiguousarray(shard(i)) for i in keep]
    dst = np.zeros(L, dtype=np.uint8)

    # The share arrays are built once, as a cgo caller holds them: keep is in
    # ascending order, so rs_decode's in-place sort (sort.Sort(byNumber))
    # leaves them as they are, and no call pays for the binding's array
    # construction (~1 us per numpy .ctypes access).
    nums = (ctypes.c_int * k)(*keep)
    ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data for b in bufs])
    dptr = P(dst.ctypes.data)

    def dec():
        rc = lib.rs_decode(f.handle, nums, ptrs, k, S, dptr)
        if rc:
            raise RuntimeError(f"config1: rs_decode returned {rc}")
    dec_ms = _median_ms(dec, reps)
    if not np.array_equal(dst, blob_np):
        raise RuntimeError("config1: rs_decode did not return the blob")
    # The zero-copy receive path: the 10 surviving shares in an engine-pinned
    # arena (each in its own slot, where rs_shard_unmarshal_arena puts a
    # Shard's data), read in place by the kernel; dst pageable.
    arena = rsmi.Arena(k * (S + 256) + 4096)
    aptrs = [arena.put(b.tobytes()) for b in bufs]
    dst_a = np.zeros(L, dtype=np.uint8)
    in0 = f.stat(f.STAT_DECODES_IN_PLACE)

    anums = (ctypes.c_int * k)(*keep)
    aptrs_c = (ctypes.c_void_p * k)(*aptrs)
    daptr = P(dst_a.ctypes.data)

    def dec_arena():
        rc = lib.rs_decode(f.handle, anums, aptrs_c, k, S, daptr)
        if rc:
            raise RuntimeError(f"config1: rs_decode (arena) returned {rc}")
    dec_arena_ms = _median_ms(dec_arena, reps)
    if not np.array_equal(dst_a, blob_np) or f.stat(f.STAT_DECODES_IN_PLACE) <= in0:
        raise RuntimeError("config1: the arena decode did not run in place or did not return the blob")
    arena.free()
    # Receive batching (rs_decode_batch, one GPU pass for many messages --
    # the engine's answer to one call per message): 64 config-1 messages,
    # each with its own 4 seeded drops, survivors read from the caller's
    # pageable shards, per-message time.
    B = 64
    brng = np.random.default_rng(0xBA7C)
    bkeeps = [sorted(set(range(n)) - set(int(v) for v in brng.choice(n, size=4, replace=False))) for _ in range(B)]
    base = {i: (blob_np.ctypes.data + i * S if i < k else parity.ctypes.data + (i - k) * S) for i in range(n)}
    bdst = [np.zeros(L, dtype=np.uint8) for _ in range(B)]
    bcounts = (ctypes.c_int * B)(*[k] * B)
    bnums = (ctypes.c_int * (B * k))(*[i for kp in bkeeps for i in kp])
    bptrs = (ctypes.c_void_p * (B * k))(*[base[i] for kp in bkeeps for i in kp])
    bout = (ctypes.c_void_p * B)(*[d.ctypes.data for d in bdst])
    bst = (ctypes.c_int * B)()

    def dec_batch():
        rc = lib.rs_decode_batch(f.handle, B, bcounts, bnums, bptrs, S, bout, bst)
        if rc or any(bst):
            raise RuntimeError(f"config1: rs_decode_batch returned {rc} / {list(bst)[:4]}")
    batch_ms = _median_ms(dec_batch, max(5, reps // 5)) / B
    if not all(np.array_equal(d, blob_np) for d in bdst):
        raise RuntimeError("config1: rs_decode_batch did not return the blob")
    del bdst
    # Send-side batching (rs_encode_batch): 64 config-1 messages' parity in
    # one GPU pass, per-message time, every message checked.
    emsgs = [np.ascontiguousarray(np.roll(blob_np, 4099 * b)) for b in range(B)]
    epar = [np.zeros(m * S, dtype=np.uint8) for _ in range(B)]
    eins = (ctypes.c_void_p * B)(*[x.ctypes.data for x in emsgs])
    eout = (ctypes.c_void_p * B)(*[x.ctypes.data for x in epar])
    est = (ctypes.c_int * B)()

    def enc_batch():
        rc = lib.rs_encode_batch(f.handle, B, eins, L, eout, est)
        if rc or any(est):
            raise RuntimeError(f"config1: rs_encode_batch returned {rc} / {list(est)[:4]}")
    ebatch_ms = _median_ms(enc_batch, max(5, reps // 5)) / B
    for b in (0, 1, B - 1):
        if not np.array_equal(epar[b], np.frombuffer(oracle.encode(E, k, n, emsgs[b].tobytes()), dtype=np.uint8)):
            raise RuntimeError("config1: rs_encode_batch parity differs from the oracle")
    del emsgs, epar
    # plugin mirror, timed in C++ (host/plugin_latency.cpp)
    blob = blob_np.tobytes()
    plug = h.plugin_latency(blob, k, n, lost, reps)
    r4 = lambda v: round(v, 4)
    # The oracle on one thread, same blob.  Encode: parity only (infectious
    # emits the data shares as views).  Decode: what Decode does for dst --
    # the present data shares copied in, the dropped ones regenerated into
    # their slots (Rebuild) -- like rs_decode.
    cpu = {}
    er = np.zeros((1, n), dtype=np.uint8)
    er[0, [i for i in lost if i < k]] = 1  # Rebuild regenerates the dropped data shares only
    par = np.zeros(m * S, dtype=np.uint8)
    dst_cpu = np.zeros(L, dtype=np.uint8)
    present = [i for i in range(k) if i not in lost]
    # The oracle's C entry points with their pointers bound once, like the
    # GPU calls above (no per-call numpy .ctypes accesses on either side).
    olib = oracle.lib()
    Ec = np.ascontiguousarray(E)
    e_p, b_p, par_p, dst_p, er_p = (P(a_.ctypes.data) for a_ in (Ec, blob_np, par, dst_cpu, er))
    src0, dst0 = blob_np.ctypes.data, dst_cpu.ctypes.data
    for name, simd in (("scalar_1t", False), ("avx2_1t", True)):
        e_ms = _median_ms(lambda: olib.orc_encode_batch(e_p, k, n, b_p, par_p, S, 1, int(simd), 1), max(5, reps // 5))
        if not np.array_equal(par, ref_par):
            raise RuntimeError("config1: the oracle's encode differs")

        def cpu_dec():
            for i in present:
                ctypes.memmove(dst0 + i * S, src0 + i * S, S)
            return olib.orc_reconstruct_batch(e_p, k, n, dst_p, par_p, S, 1, er_p, int(simd), 1)
        d_ms = _median_ms(cpu_dec, max(5, reps // 5))
        if not np.array_equal(dst_cpu, blob_np):
            raise RuntimeError("config1: the oracle's decode did not return the blob")
        cpu[name] = {"encode_ms": e_ms, "decode4_ms": d_ms}
    best = min(cpu.values(), key=lambda v: v["encode_ms"])
    return {
        "status": "ok",
        "what": "configs[0]: 1,048,580-B blob, RS(10,4), one call per message (main.go:243-267 encode, "
                "main.go:72-79 decode after 4 seeded drops); median latency; PCIe-inclusive",
        "message_bytes": L, "shard_bytes": S, "dropped": lost, "reps": reps,
        "codec": {"encode_ms": enc_ms, "decode4_ms": dec_ms,
                  "encode_GBps": round(L * n / k / enc_ms / 1e6, 2),
                  "decode4_arena_ms": dec_arena_ms,
                  "decode4_batch64_ms_per_message": round(batch_ms, 4),
                  "encode_batch64_ms_per_message": round(ebatch_ms, 4),
                  "note": "caller-owned pageable buffers (what cgo passes), staged through pinned memory; "
                          "decode4_arena: the survivors in an engine-pinned rs_arena, read in place; "
                          "decode4_batch64: 64 messages (own drops each) in one rs_decode_batch call; "
                          "encode_batch64: 64 messages' parity in one rs_encode_batch call"},
        "plugin": {"prepareShards_ms": r4(plug["prepareShards"]),
                   "prepareShards_marshal_ms": r4(plug["prepareShards_marshal"]),
                   "broadcast_wire_ms": r4(plug["broadcast_wire"]),
                   "receive10_then_decode_ms": r4(plug["receive_then_decode"]),
                   "receive10_copy_then_decode_ms": r4(plug["receive_copy_then_decode"]),
                   "receive10_pool_ms": r4(plug["receive_pool10"]), "receive_trigger_ms": r4(plug["receive_trigger"]),
                   "codec_encode_ms": r4(plug["codec_encode"]), "codec_decode4_ms": r4(plug["codec_decode"]),
                   "memcpy_wire_ms": r4(plug["memcpy_wire"]), "wire_bytes": int(plug["wire_bytes"]),
                   "note": "C++ ShardPlugin mirror timed in C++ (host/plugin_latency.cpp), medians; no signer / "
                           "verifier. prepareShards_marshal = the reference's copies (DeepCopy main.go:255-258, then "
                           "Marshal per Shard); broadcast_wire = ShardAndBroadcastWire, each share byte copied once "
                           "into the wire; receive10_then_decode = 10 Receive(Shard&&) pooling + the decoding "
                           "arrival; memcpy_wire = one copy of the 14 marshalled Shards"},
        "cpu_1t": cpu,
        "gpu_vs_1core": {"encode": round(best["encode_ms"] / enc_ms, 3),
                         "decode4": round(min(v["decode4_ms"] for v in cpu.values()) / dec_ms, 3),
                         "decode4_arena": round(min(v["decode4_ms"] for v in cpu.values()) / dec_arena_ms, 3),
                         "decode4_batch64": round(min(v["decode4_ms"] for v in cpu.values()) / batch_ms, 3),
                         "encode_batch64": round(best["encode_ms"] / ebatch_ms, 3)},
    }


def traffic_of(key, path=os.path.join(ROOT, "profiles", "traffic.json")):
    """{traffic_GB, traffic_ratio, trace_frac, source} of one role in
    profiles/traffic.json (rocprofv3 passes of the default line,
    tools/prof_line.py), or None."""
    try:
        with open(path) as fh:
            e = json.load(fh).get("entries", {}).get(key)
    except (OSError, ValueError, AttributeError):
        return None
    if not e:
        return None
    return {"traffic_GB": e.get("traffic_GB"), "traffic_ratio": e.get("traffic_ratio"),
            "trace_frac": e.get("trace_frac"), "source": e.get("profile")}


def config3_worst_leg(local, dev, stripes, S, steps=3, warmup=1):
    """configs[2]'s worst case: RS(10,4) with the same
    four data shards (0-3) erased in every stripe, so every stripe
    regenerates 4 data shards from 6 data + 4 parity survivors -- the most
    arithmetic a reconstruct does and the encode's byte count (k + 4 shards
    per stripe).  Reconstruct only (parity encoded once, untimed), HIP
    events, GB/s on the algorithmic bytes."""
    import rsmi
    k, n = 10, 14
    f = rsmi.FEC(k, n, device=local)
    fixed = np.zeros((stripes, n), dtype=np.uint8)
    fixed[:, [0, 1, 2, 3]] = 1
    run = device_run(f, k, n, S, stripes, steps, warmup, [fixed] * (warmup + steps), False, True, dev,
                     prepare_emax=4)
    rec_bytes = stripes * (k + 4) * S
    rec_ms = sum(run["reconstruct_ms"]) / steps
    gbps = rec_bytes / (rec_ms / 1e3) / 1e9
    return {
        "status": "ok",
        "what": f"configs[2] worst case: RS(10,4), {stripes} stripes x 10 x {S} B, data shards 0-3 erased in "
                "every stripe (4 regenerated from 6 data + 4 parity)",
        "steps": steps, "warmup": warmup, "stripes": stripes, "shard_bytes": S,
        "reconstruct": {"kernel": f.kernel_name(1), "ms": round(rec_ms, 3), "GBps": round(gbps, 1),
                        "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes": rec_bytes,
                        "pmc": traffic_of(f"config3_worst_reconstruct_k{k}_n{n}_S{S}_stripes{stripes}")},
    }


def config5_leg(local, dev, stripes=16384, steps=5, warmup=2):
    """configs[4]: the wide code RS(64,16) with 64 KiB shards, `stripes`
    stripes (64 x 64 KiB = 4 MiB of data each) device-resident, a fresh
    1-16-erasure set per step (patterns inverted on the GPU inside the step,
    the pattern space is too large to prepare).  Encode and reconstruct
    times from HIP events, GB/s on the algorithmic bytes and the fraction of
    the HBM roofline."""
    import rsmi
    k, n, S = 64, 80, 65536
    m = n - k
    f = rsmi.FEC(k, n, device=local)
    rng = np.random.default_rng(0xE4A5)
    ersets = erasure_sets(rng, warmup + steps, stripes, n, 1, m)
    run = device_run(f, k, n, S, stripes, steps, warmup, ersets, True, True, dev)
    enc_bytes = stripes * n * S
    rec_bytes = sum(int(((k + er.sum(axis=1)) * S).sum()) for er in ersets[warmup:]) / steps
    enc_ms = sum(run["encode_ms"]) / steps
    rec_ms = sum(run["reconstruct_ms"]) / steps
    enc_gbps = enc_bytes / (enc_ms / 1e3) / 1e9
    rec_gbps = rec_bytes / (rec_ms / 1e3) / 1e9
    return {
        "status": "ok",
        "what": f"configs[4]: RS(64,16), {stripes} stripes x 64 x 64 KiB shards, fresh 1-16 erasures per "
                "stripe per step (patterns built on the GPU inside the step)",
        "steps": steps, "warmup": warmup, "stripes": stripes, "shard_bytes": S,
        "ms_per_step": round(run["elapsed"] / steps * 1e3, 3),
        "value_GBps": round((enc_bytes + rec_bytes) / (run["elapsed"] / steps) / 1e9, 1),
        "encode": {"kernel": f.kernel_name(0), "ms": round(enc_ms, 3), "GBps": round(enc_gbps, 1),
                   "frac": round(enc_gbps / HBM_PEAK_GBS, 4), "bytes": enc_bytes,
                   "pmc": traffic_of(f"config5_encode_k{k}_n{n}_S{S}_stripes{stripes}")},
        "reconstruct": {"kernel": f.kernel_name(1), "ms": round(rec_ms, 3), "GBps": round(rec_gbps, 1),
                        "frac": round(rec_gbps / HBM_PEAK_GBS, 4), "bytes": int(rec_bytes),
                        "pmc": traffic_of(f"config5_reconstruct_k{k}_n{n}_S{S}_stripes{stripes}")},
        "note": "frac: algorithmic bytes / HIP-event time (incl. the step's fresh-pattern builds for the "
                "reconstruct); pmc: the rocprofv3 passes of the default line (traffic, trace-based frac, source)",
    }


def device_set_leg(k, n, S, stripes, steps=3, warmup=1, spread_stripes=256, seed=0xD5E7):
    """north_star's node-level partition through the product boundary (VERDICT
    r05 next #1): ONE process, one device-set context (rs_new_devices, the
    Go shim's NewFECOnDevices) over every GPU this process sees -- [0, 0], two
    members on one GPU, on a one-GPU box.  Member i holds its own `stripes`
    stripes in its own HBM; a step is rs_encode_stripes_parts then
    rs_reconstruct_stripes_parts with fresh 1..m erasures per stripe, every
    member at once from its own host thread, timed by the wall clock around
    every device's synchronize.  Then the shard-distributed placement
    (configs[3]): shard i of each of `spread_stripes` stripes
    on GPU i mod G, stripe s reconstructed by member s mod G with
    rs_reconstruct_spread -- survivors on other GPUs read in place over xGMI
    (peer access).  Both checked: erased shards zeroed, reconstructed, and
    every member's buffers equal their checksums from before.  Never `value`."""
    import rsmi
    m = n - k
    G = torch.cuda.device_count()
    devices = list(range(G)) if G > 1 else [0, 0]
    f = rsmi.FEC(k, n, devices=devices)
    M = f.member_count()
    data = [torch.empty(stripes * k * S, dtype=torch.uint8, device=f"cuda:{d}") for d in devices]
    par = [torch.empty(stripes * m * S, dtype=torch.uint8, device=f"cuda:{d}") for d in devices]

    def sync():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    for i in range(M):
        f.member(i).fill_splitmix(data[i].data_ptr(), data[i].numel(), seed + i)
    parts = [(data[i].data_ptr(), k * S, par[i].data_ptr(), m * S, stripes, 0) for i in range(M)]
    if pattern_total(n, m) <= (1 << 20):
        f.prepare_patterns(m)  # every member's cache, before timing (like the headline)
    f.encode_stripes_parts(parts, S, S)
    sync()

    def checksum(ts):
        return [int(t.view(torch.int64).sum().item()) for t in ts]

    ck = (checksum(data), checksum(par))
    rng = np.random.default_rng(seed)
    ersets = erasure_sets(rng, warmup + steps + 1, stripes * M, n, 1, m)
    enc_s, rec_s = [], []
    for i in range(warmup + steps):
        t0 = time.perf_counter()
        f.encode_stripes_parts(parts, S, S)
        sync()
        t1 = time.perf_counter()
        f.reconstruct_stripes_parts(parts, S, S, ersets[i].tobytes())  # intact shards: the same bytes rewritten
        sync()
        t2 = time.perf_counter()
        if i >= warmup:
            enc_s.append(t1 - t0)
            rec_s.append(t2 - t1)

    def zero_erased(er, views):
        for i, (dv, pv) in enumerate(views):
            e = torch.from_numpy(er[i * stripes:(i + 1) * stripes].astype(bool)).to(dv.device)
            dv[e[:, :k]] = 0
            pv[e[:, k:]] = 0

    er = ersets[-1]
    zero_erased(er, [(data[i].view(stripes, k, S), par[i].view(stripes, m, S)) for i in range(M)])
    f.reconstruct_stripes_parts(parts, S, S, er.tobytes())
    sync()
    ok = (checksum(data), checksum(par)) == ck
    enc_bytes = M * stripes * n * S
    rec_bytes = sum(int(((k + x.sum(axis=1)) * S).sum()) for x in ersets[warmup:warmup + steps]) / steps
    enc_ms, rec_ms = np.median(enc_s) * 1e3, np.median(rec_s) * 1e3
    out = {
        "status": "ok" if ok else "error: reconstructed shards differ from the encoded stripes",
        "what": f"one process, one rs_new_devices context over devices {devices}: RS({k},{n}), "
                f"{stripes} stripes x {k} x {S} B per member; step = rs_encode_stripes_parts + "
                f"rs_reconstruct_stripes_parts (fresh 1-{m} erasures), wall clock around every device's "
                "synchronize; never value",
        "members": M, "devices": devices, "stripes_per_member": stripes, "steps": steps,
        "encode": {"ms": round(enc_ms, 3), "GBps": round(enc_bytes / enc_ms / 1e6, 1)},
        "reconstruct": {"ms": round(rec_ms, 3), "GBps": round(rec_bytes / rec_ms / 1e6, 1)},
        "value_GBps": round((enc_bytes + rec_bytes) / (enc_ms + rec_ms) / 1e6, 1),
        "per_gpu_GBps": round((enc_bytes + rec_bytes) / (enc_ms + rec_ms) / 1e6 / len(set(devices)), 1),
        "checked": ok,
    }
    del data, par
    torch.cuda.empty_cache()
    # Shard-distributed placement: holders on GPU h = i mod H (H = G, or two
    # allocations on one GPU), owner of stripe s = member s mod M.
    try:
        H = G if G > 1 else 2
        hdev = list(range(G)) if G > 1 else [0, 0]
        T = spread_stripes
        per = [len(range(h, n, H)) for h in range(H)]
        src_d = torch.empty(T * k * S, dtype=torch.uint8, device=f"cuda:{devices[0]}")
        src_p = torch.empty(T * m * S, dtype=torch.uint8, device=f"cuda:{devices[0]}")
        f.member(0).fill_splitmix(src_d.data_ptr(), src_d.numel(), seed ^ 0x5D)
        f.member(0).encode_stripes(src_d.data_ptr(), k * S, src_p.data_ptr(), m * S, S, S, T)
        sync()
        full = torch.cat([src_d.view(T, k, S), src_p.view(T, m, S)], dim=1)
        holders = [torch.empty(T * per[h] * S, dtype=torch.uint8, device=f"cuda:{hdev[h]}") for h in range(H)]
        for h in range(H):
            holders[h].view(T, per[h], S).copy_(full[:, h::H, :])
        del full, src_d, src_p
        sync()
        ptrs = np.zeros((T, n), dtype=np.uint64)
        for s_ in range(T):
            for i in range(n):
                h = i % H
                ptrs[s_, i] = holders[h].data_ptr() + (s_ * per[h] + i // H) * S
        owner = [s_ % M for s_ in range(T)]
        hck = checksum(holders)
        sets = erasure_sets(np.random.default_rng(seed + 1), warmup + steps + 1, T, n, 1, m)
        tab = ptrs.reshape(-1).tolist()
        sp_s = []
        for i in range(warmup + steps):
            t0 = time.perf_counter()
            f.reconstruct_spread(tab, owner, S, T, sets[i].tobytes())
            sync()
            if i >= warmup:
                sp_s.append(time.perf_counter() - t0)
        er = sets[-1]
        for s_ in range(T):
            for i in np.flatnonzero(er[s_]):
                h = int(i) % H
                holders[h].view(T, per[h], S)[s_, int(i) // H].zero_()
        f.reconstruct_spread(tab, owner, S, T, er.tobytes())
        sync()
        sok = checksum(holders) == hck
        # survivor / output bytes that live on another GPU than the owner's
        remote = 0
        for s_ in range(T):
            od = devices[owner[s_]]
            for i in range(n):
                remote += (hdev[i % H] != od) and G > 1
        sp_ms = np.median(sp_s) * 1e3
        sp_bytes = sum(int(((k + x.sum(axis=1)) * S).sum()) for x in sets[warmup:warmup + steps]) / steps
        out["spread"] = {
            "status": "ok" if sok else "error: spread reconstruct differs",
            "stripes": T, "holders": hdev, "ms": round(sp_ms, 3), "GBps": round(sp_bytes / sp_ms / 1e6, 1),
            "remote_shard_fraction": round(remote / (T * n), 3),
            "what": "shard i of every stripe on GPU i mod G, stripe s reconstructed by member s mod G reading "
                    "its survivors in place (peer HBM over xGMI when G > 1)"}
        del holders
        torch.cuda.empty_cache()
    except Exception as e:  # reported in the leg, never silent
        out["spread"] = {"status": f"error: {type(e).__name__}: {e}"}
    f.close()
    return out


def device_set_child(args, k, n, S):
    """device_set_leg in a child process (bench.py --device-set-child), its
    JSON relayed; a failure, crash or timeout becomes the leg's status."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--device-set-child", "--k", str(k), "--n", str(n),
           "--shard", str(S), "--device-set-stripes", str(args.device_set_stripes)]
    try:
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=args.device_set_timeout)
    except subprocess.TimeoutExpired:
        return {"status": f"error: device-set child timed out after {args.device_set_timeout} s"}
    lines = [ln for ln in p.stdout.splitlines() if ln.lstrip().startswith("{")]
    if p.returncode != 0 or not lines:
        return {"status": f"error: device-set child exited {p.returncode}: {p.stderr[-400:]}"}
    return json.loads(lines[-1])


def _cpulist(text: str) -> set:
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def pin_to_gpu_numa(local: int):
    """Runs the calling thread -- and the threads it starts later -- on the
    CPUs of the NUMA node GPU `local` hangs off (sysfs numa_node of its PCI
    function), as a deployment pins a GPU process.  The single-message legs
    depend on it: a config-1 decode / encode from a thread on the GPU's node
    took 47.6-48.2 / 50.9-52.1 us, from the other socket 59.8-60.1 / 64.2-64.5
    us (profiles/r06q/).  The headline (device resident) does not.  Returns
    what was done, for the JSON line; RSMI_BENCH_NO_PIN=1 leaves the
    affinity alone."""
    if os.environ.get("RSMI_BENCH_NO_PIN"):
        return {"pinned": False, "why": "RSMI_BENCH_NO_PIN"}
    try:
        p = torch.cuda.get_device_properties(local)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as fh:
            node = int(fh.read())
        if node < 0:
            return {"pinned": False, "gpu_pci": bdf, "why": "no NUMA node"}
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            cpus = _cpulist(fh.read()) & os.sched_getaffinity(0)
        if not cpus:
            return {"pinned": False, "gpu_pci": bdf, "gpu_numa_node": node, "why": "no allowed CPU on the node"}
        os.sched_setaffinity(0, cpus)
        return {"pinned": True, "gpu_pci": bdf, "gpu_numa_node": node, "cpus": len(cpus)}
    except (OSError, ValueError, RuntimeError, AttributeError) as e:
        return {"pinned": False, "why": repr(e)[:120]}


def main():
    global _RESULT_OUT
    args = parse()
    if args.device_set_child:  # bench.py's own child (device_set_child): one JSON line, nothing else
        print(json.dumps(guarded_leg(lambda: device_set_leg(args.k, args.n, args.shard, args.device_set_stripes))))
        return
    how = check_world(args.gpus)
    if how == "launch":
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RSMI_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a
    # device round-robin; the driver's runs use RCCL, one rank per GPU).
    backend = os.environ.get("RSMI_BENCH_BACKEND", "nccl")
    if backend == "nccl" and world > torch.cuda.device_count():
        sys.stderr.write(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPUs visible "
                         "(RSMI_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs)\n")
        raise SystemExit(2)
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    affinity = pin_to_gpu_numa(local)
    distributed = "RANK" in os.environ  # launched by torch.distributed.run (any N)
    if distributed:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    if args.placement == "sharded":
        return sharded_main(args, world, rank, local, dev, distributed)
    if args.stream:
        return stream_main(args, world, rank, local, dev, distributed)

    import rsmi

    k, n, S = args.k, args.n, args.shard
    m = n - k
    emax = args.emax if args.emax is not None else m
    stripes = args.stripes
    f = rsmi.FEC(k, n, device=local)
    pool = args.pattern_pool
    rng = np.random.default_rng(0xE4A5 + rank)
    if args.erase:
        fixed = np.zeros((stripes, n), dtype=np.uint8)
        fixed[:, [int(v) for v in args.erase.split(",")]] = 1
        ersets = [fixed] * (args.warmup + args.steps)
    else:
        ersets = erasure_sets(rng, args.warmup + args.steps, stripes, n, args.emin, emax, pool)
    rec_bytes = [int(((k + er.sum(axis=1)) * S).sum()) for er in ersets]
    enc_bytes = stripes * (k + m) * S
    do_enc = args.mode in ("both", "encode")
    do_rec = args.mode in ("both", "reconstruct")
    run = device_run(f, k, n, S, stripes, args.steps, args.warmup, ersets, do_enc, do_rec, dev,
                     seed=0x5EED ^ (rank << 32), prepare_emax=emax, distributed=distributed)
    elapsed, enc_ms, rec_ms, prep_ms = run["elapsed"], run["encode_ms"], run["reconstruct_ms"], run["prep_ms"]
    # Per-rank wall time, kernel times and algorithmic bytes (each rank draws
    # its own erasure sets, so its reconstruct bytes are its own); the job's
    # time is the max over ranks, its bytes the sum.
    step_bytes_local = sum((enc_bytes if do_enc else 0) + (rec_bytes[i] if do_rec else 0)
                           for i in range(args.warmup, args.warmup + args.steps))
    mine = torch.tensor([elapsed, sum(enc_ms) / len(enc_ms), sum(rec_ms) / len(rec_ms), step_bytes_local],
                        dtype=torch.float64, device=stats_device(dev))
    if distributed:
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(gathered, mine)
        per_rank = [g.tolist() for g in gathered]
    else:
        per_rank = [mine.tolist()]
    elapsed, total_bytes = job_totals(per_rank)
    value = total_bytes / elapsed / 1e9

    enc_avg_ms = sum(enc_ms) / len(enc_ms)
    rec_avg_ms = sum(rec_ms) / len(rec_ms)
    rec_avg_bytes = sum(rec_bytes[args.warmup:]) / args.steps
    dominant = "encode" if do_enc else "reconstruct"
    dom_bytes = enc_bytes if do_enc else rec_avg_bytes
    dom_ms = enc_avg_ms if do_enc else rec_avg_ms
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    # HBM traffic of the dominant kernel: measured by rocprofv3 PMC passes of
    # this same default line (tools/prof_line.py -> profiles/traffic.json,
    # keyed by role and workload, naming the profile it came from); the run
    # itself cannot read counters.
    traffic = traffic_entry = None
    try:
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        traffic_entry = tj.get("entries", {}).get(f"{dominant}_k{k}_n{n}_S{S}_stripes{stripes}")
        if traffic_entry:
            traffic = traffic_entry.get("traffic_GB")
    except (OSError, ValueError, AttributeError):
        pass

    out = None
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0 and world == 1:  # after the timed region, rank 0 at N = 1 only
            cpu = cpu_baseline(k, n, S, args.cpu_seconds, args.cpu_threads)
        out = {
            "metric": "RS(10,4) encode+reconstruct GB/s at 1/8 GPUs; % HBM roofline",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes, device-generated; " +
                    (f"erasures {args.erase} in every stripe)" if args.erase else
                     f"random {args.emin}-{emax} erasures/stripe)"),
            "config": {
                "workload": f"RS({k},{n}) encode + " +
                            (f"erasures-{args.erase.replace(',', '+')} " if args.erase else f"{args.emin}-{emax}-erasure ") +
                            f"reconstruct of "
                            f"{stripes} stripes x {k} x {S} B shards per GPU (configs[1]+[2])",
                "k": k, "n": n, "shard_bytes": S, "stripes_per_gpu": stripes,
                "data_bytes_per_gpu": stripes * k * S,
                "parallelism": f"stripe-partitioned x{world}, no collective",
                "host_affinity": affinity,
                "erasure_patterns": "all" if pool == 0 else f"pool of {pool}",
                "mode": args.mode,
            },
            "breakdown": {
                "encode_ms": round(enc_avg_ms, 3),
                "encode_GBps": round(enc_bytes / (enc_avg_ms / 1e3) / 1e9, 1) if do_enc else None,
                "encode_data_GBps": round(stripes * k * S / (enc_avg_ms / 1e3) / 1e9, 1) if do_enc else None,
                "reconstruct_ms": round(rec_avg_ms, 3),
                "reconstruct_GBps": round(rec_avg_bytes / (rec_avg_ms / 1e3) / 1e9, 1) if do_rec else None,
                "reconstruct_frac": round(rec_avg_bytes / (rec_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if do_rec else None,
                "encode_kernel": f.kernel_name(0),
                "reconstruct_kernel": f.kernel_name(1),
                "patterns_prepared": pattern_total(n, emax) if prep_ms is not None else 0,
                "pattern_prepare_ms": round(prep_ms, 2) if prep_ms is not None else None,
            },
            "roofline": {
                "kernel": f"{f.kernel_name(0 if do_enc else 1)} ({dominant})",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": int(dom_bytes),
                "traffic_source": traffic_entry.get("profile") if traffic_entry else None,
                "traffic_ratio": traffic_entry.get("traffic_ratio") if traffic_entry else None,
                "trace_frac": traffic_entry.get("trace_frac") if traffic_entry else None,
                "note": "achieved/frac: algorithmic bytes / HIP-event time of this run; traffic, traffic_ratio and "
                        "trace_frac: the rocprofv3 passes of the same default line named by traffic_source",
            },
            "cpu_baseline": cpu,
            "per_rank": [{"rank": r, "ms_per_step": round(v[0] / args.steps * 1e3, 3),
                          "value": round(v[3] / v[0] / 1e9, 2), "bytes": int(v[3]),
                          "encode_ms": round(v[1], 3), "reconstruct_ms": round(v[2], 3)}
                         for r, v in enumerate(per_rank)],
        }
    if args.device_set_stripes > 0 and world == 1 and args.extra_legs:
        # The device-set context over every GPU a process sees (N = 1 only:
        # all of a node's GPUs are visible to it), in a child process, so a
        # fault or hang there (its peer reads have never run on an 8-GPU
        # node here) cannot cost the headline line.
        del f
        torch.cuda.empty_cache()
        out["device_set"] = device_set_child(args, k, n, S)
        f = rsmi.FEC(k, n, device=local)
    if distributed and world > 1 and args.gather_stripes > 0:
        # configs[3]'s survivor gather on the same ranks, after the headline
        # is measured (device_run freed its buffers).
        gather_leg(args, f, k, n, S, emax, world, rank, dev, out)  # emits the line and tears down
        return
    if rank == 0 and world == 1 and args.extra_legs:
        # The reference's own per-message path (configs[0]) and the wide code
        # (configs[4]) at N = 1: reported beside the headline, never in value.
        del f
        torch.cuda.empty_cache()
        out["config1"] = guarded_leg(lambda: config1_leg(local, args.config1_reps))
        out["config5"] = guarded_leg(lambda: config5_leg(local, dev, args.config5_stripes, args.config5_steps,
                                                         args.config5_warmup))
        if args.config3_steps > 0:
            out["config3_worst"] = guarded_leg(lambda: config3_worst_leg(local, dev, stripes, S, args.config3_steps))
    if rank == 0:
        emit(out)
    if distributed:
        torch.distributed.destroy_process_group()


def gather_what(backend: str) -> str:
    """What the N > 1 gather leg does, naming the backend that moved the
    survivors (RCCL on the driver's runs, gloo in a rehearsal)."""
    how = ("RCCL (batch_isend_irecv = ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd over xGMI)"
           if backend == "nccl" else
           f"{backend} (rehearsal: device rows staged through host memory, ranks sharing GPUs)")
    return ("shard i of every stripe on rank i mod N; each owner gathers exactly Rebuild's survivors over "
            + how + " and reconstructs from the receive buffers (rs_reconstruct_ptrs); not part of value")


class OnceLine:
    """Rank 0's JSON line, printed exactly once: by the gather leg when it
    finishes, or by its watchdog when it does not.  finish() returns True to
    the one caller that printed it."""

    def __init__(self, rank, out):
        import threading
        self.lock = threading.Lock()
        self.emitted = False
        self.rank, self.out = rank, out

    def finish(self, gather) -> bool:
        with self.lock:
            if self.emitted:
                return False
            self.emitted = True
        if self.rank == 0 and self.out is not None:
            self.out["gather"] = gather
            emit(self.out)
        return True


def make_abandon(line: OnceLine, timeout: float, exit_fn=None):
    """The watchdog's action: print the headline line with the gather leg
    marked abandoned, then end the process with EXIT_GATHER_ABANDONED (a
    collective that never completed is a failed run even though the
    headline was measured).  os._exit: the stuck collective's threads
    cannot be joined."""
    exit_fn = exit_fn or os._exit

    def abandon():
        if line.finish({"status": f"abandoned after {timeout:.0f} s (collective did not complete)"}):
            sys.stderr.write("bench.py: gather leg abandoned\n")
            sys.stderr.flush()
            exit_fn(EXIT_GATHER_ABANDONED)
    return abandon


def gather_leg(args, f, k, n, S, emax, world, rank, dev, out):
    """N > 1: a short shard-distributed leg (sharded_run with
    --gather-stripes owned stripes per rank, 1 warm-up + 2 timed steps,
    each timed step's output checked on a sample) reported as
    out["gather"].  A watchdog per rank abandons a leg stuck in a collective
    after --gather-timeout seconds: rank 0 still prints the headline line
    (gather.status says what happened) and every rank exits with
    EXIT_GATHER_ABANDONED, so the headline measurement is kept but the run
    is not reported as a success.  Wrong shards exit non-zero after the
    line is printed."""
    import threading

    line = OnceLine(rank, out)
    torch.distributed.barrier()  # rank 0's CPU baseline is done: start every clock together
    timer = threading.Timer(args.gather_timeout, make_abandon(line, args.gather_timeout))
    timer.daemon = True
    timer.start()
    steps, warmup = 2, 1
    backend = os.environ.get("RSMI_BENCH_BACKEND", "nccl")
    gather = {"status": "ok", "backend": backend, "owned_stripes_per_rank": args.gather_stripes,
              "shard_bytes": S, "steps": steps, "warmup": warmup, "what": gather_what(backend)}
    bad = 0
    try:
        res = sharded_run(f, k, n, S, args.gather_stripes, steps, warmup, args.emin, emax, 0, args.chunks,
                          world, rank, dev, True, budget_exit=False)
        if res is None:
            gather["status"] = "skipped: HBM budget"
        else:
            gather.update(gather_summary(res, steps, world))
            bad = res["verified"]["mismatched_shards"]
            if bad:
                gather["status"] = "wrong shards"
        torch.distributed.destroy_process_group()
    except Exception as e:  # reported; the headline line is still printed
        gather["status"] = f"error: {type(e).__name__}: {e}"
    timer.cancel()
    line.finish(gather)
    if bad:
        raise SystemExit("bench.py: the gather leg reconstructed wrong shards")
    if gather["status"].startswith("error"):
        raise SystemExit("bench.py: the gather leg failed: " + gather["status"])


def stream_main(args, world, rank, local, dev, distributed):
    """configs[1], second mode: the same 6,553 stripes, but the
    data starts in pinned host memory and the parity ends there.  Chunks of
    --stream-chunk stripes alternate between two HIP streams: H2D copy of the
    chunk's data, rs_encode_stripes, D2H copy of its parity, so one chunk's
    copies overlap the other's.  The host side is a two-slot pinned ring
    (reused for every chunk: the bytes repeat, the PCIe and HBM work does
    not).  value = (k+m) bytes per stripe over the wall time; the PCIe rates
    are reported beside it."""
    import rsmi

    k, n, S = args.k, args.n, args.shard
    m = n - k
    stripes, C = args.stripes, max(1, min(args.stream_chunk, args.stripes))
    f = rsmi.FEC(k, n, device=local)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    h_data = [torch.empty(C * k * S, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    h_par = [torch.empty(C * m * S, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    d_data = [torch.empty(C * k * S, dtype=torch.uint8, device=dev) for _ in range(2)]
    d_par = [torch.empty(C * m * S, dtype=torch.uint8, device=dev) for _ in range(2)]
    for slot in range(2):
        f.fill_splitmix(d_data[slot].data_ptr(), d_data[slot].numel(), 0x5EED + slot, streams[slot].cuda_stream)
        streams[slot].synchronize()
        h_data[slot].copy_(d_data[slot].cpu())
    chunks = [(s0, min(C, stripes - s0)) for s0 in range(0, stripes, C)]

    def one_pass():
        for i, (s0, nb) in enumerate(chunks):
            slot = i & 1
            st = streams[slot]
            with torch.cuda.stream(st):
                d_data[slot][:nb * k * S].copy_(h_data[slot][:nb * k * S], non_blocking=True)
                f.encode_stripes(d_data[slot].data_ptr(), k * S, d_par[slot].data_ptr(), m * S, S, S, nb,
                                 st.cuda_stream)
                h_par[slot][:nb * m * S].copy_(d_par[slot][:nb * m * S], non_blocking=True)

    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    mine = torch.tensor([elapsed], dtype=torch.float64, device=stats_device(dev))
    if distributed:
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(gathered, mine)
        per_rank = [g.item() for g in gathered]
    else:
        per_rank = [elapsed]
    elapsed = max(per_rank)
    total = args.steps * stripes * world
    if rank == 0:
        emit({
            "metric": "RS(10,4) encode GB/s streamed from pinned host memory (configs[1] second mode, PCIe-inclusive)",
            "value": round(total * (k + m) * S / elapsed / 1e9, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes in a two-slot pinned host ring)",
            "config": {"workload": f"RS({k},{n}) encode of {stripes} stripes x {k} x {S} B shards per GPU, "
                                   f"data H2D and parity D2H in chunks of {C} stripes on two HIP streams",
                       "k": k, "n": n, "shard_bytes": S, "stripes_per_gpu": stripes, "chunk_stripes": C},
            "pcie": {"h2d_GBps": round(total * k * S / elapsed / 1e9, 2),
                     "d2h_GBps": round(total * m * S / elapsed / 1e9, 2)},
            "per_rank": [{"rank": r, "ms_per_step": round(v / args.steps * 1e3, 3)} for r, v in enumerate(per_rank)],
        })
    if distributed:
        torch.distributed.destroy_process_group()


def agree_max(value: int, distributed: bool, dev) -> int:
    """max over ranks of an integer (identity without a process group)."""
    if not distributed:
        return value
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.int64, device=stats_device(dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t[0])


def sharded_run(f, k, n, S, stripes, steps, warmup, emin, emax, pool, chunks, world, rank, dev, distributed,
                budget_exit=True, outs=2):
    """configs[3], shard-distributed placement: shard i of every stripe is
    held by rank i mod N (the p2p analogue of main.go:207 broadcasting each
    shard to peers).  One step = the survivor gather (exactly the survivors
    each owner reads, rsmi/distributed.py) in `chunks` chunks, chunk c + 1's
    exchange (communication stream) overlapping chunk c's
    rs_reconstruct_ptrs (compute stream), which reads survivors where they
    landed; steps are queued back to back with no host sync.  The per-rank
    HBM budget is computed before anything is allocated; a budget over the
    free HBM raises the chunk count (agreed over ranks: the max), and past
    64 chunks every rank exits non-zero with the numbers (budget_exit) or
    returns None.  Step i writes output buffer i mod `outs`, so the last
    `outs` timed steps' outputs (the last step and the one before it, whose
    receive slots the last step reused) are checked on a sample afterwards.
    Every rank returns the all-gathered per-rank statistics and the summary."""
    from rsmi import distributed as rd

    m = n - k
    gstripes = stripes * world           # global stripes; each rank owns `stripes`
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ids = rd.local_shard_ids(rank, n, world)
    rng = np.random.default_rng(0xE4A5)  # same erasure map on every rank
    ersets = erasure_sets(rng, warmup + steps, gstripes, n, emin, emax, pool)
    # Plans first (host metadata, identical on every rank), then the budget.
    free_b, _ = torch.cuda.mem_get_info(dev)
    if os.environ.get("RSMI_BENCH_BACKEND", "nccl") != "nccl":
        free_b //= -(-world // max(torch.cuda.device_count(), 1))  # ranks share the rehearsal GPU(s)
    outs = max(1, min(outs, steps))
    headroom = 4 << 30

    def plan_all(c):
        tp = time.perf_counter()
        ps = [rd.plan_exchange(er, k, n, rank, world, S, chunks=c) for er in ersets]
        return ps, (time.perf_counter() - tp) * 1e3 / len(ersets)

    chunks = max(1, chunks)
    while True:
        plans, plan_ms = plan_all(chunks)
        budget = rd.hbm_budget(gstripes, len(ids), S, plans, n, k=k, outs=outs)
        if budget["total"] * 1e9 <= free_b - headroom or chunks >= 64:
            break
        chunks *= 2
    # Every rank must plan with the same chunk count (plan_exchange pairs
    # rank p's send segments with rank o's receive slots), and either every
    # rank runs or none does: two collectives, made by every rank.
    agreed = agree_max(chunks, distributed, dev)
    if agreed != chunks:
        chunks = agreed
        plans, plan_ms = plan_all(chunks)
        budget = rd.hbm_budget(gstripes, len(ids), S, plans, n, k=k, outs=outs)
    fits = not agree_max(int(budget["total"] * 1e9 > free_b - headroom), distributed, dev)
    if not fits:
        sys.stderr.write(f"bench.py: sharded placement needs {budget['total']:.1f} GB on rank {rank} "
                         f"({', '.join(f'{key} {v:.1f}' for key, v in budget.items() if key != 'total')}) "
                         f"with {free_b / 1e9:.1f} GB free, or another rank's budget does not fit: "
                         "lower --stripes\n")
        if budget_exit:
            raise SystemExit(3)
        return None
    held = torch.empty((gstripes, len(ids), S), dtype=torch.uint8, device=dev)
    # Setup (untimed): the global data is one splitmix stream, generated in
    # batches; a rank keeps the rows of its shard ids and encodes only when
    # it holds parity ids (ranks holding data ids alone skip the encode).
    batch = 64
    needs_parity = any(i >= k for i in ids)
    tmp_d = torch.empty(batch * k * S, dtype=torch.uint8, device=dev)
    tmp_p = torch.empty(batch * m * S, dtype=torch.uint8, device=dev) if needs_parity else None
    gamma = 0x9E3779B97F4A7C15
    for b0 in range(0, gstripes, batch):
        nb = min(batch, gstripes - b0)
        f.fill_splitmix(tmp_d.data_ptr(), nb * k * S, (0x5EED + b0 * k * S // 8 * gamma) & (2**64 - 1), sh)
        if needs_parity:
            f.encode_stripes(tmp_d.data_ptr(), k * S, tmp_p.data_ptr(), m * S, S, S, nb, sh)
        dv = tmp_d[:nb * k * S].view(nb, k, S)
        for j, i in enumerate(ids):
            held[b0:b0 + nb, j].copy_(dv[:, i] if i < k else tmp_p[:nb * m * S].view(nb, m, S)[:, i - k])
    del tmp_d, tmp_p
    if pattern_total(n, emax) <= (1 << 20):
        f.prepare_patterns(emax, sh)
    bufs = rd.make_buffers(plans, S, dev, outs=outs)
    tables = [torch.from_numpy(rd.shard_table(p, held, bufs, out=i % outs)).to(dev) for i, p in enumerate(plans)]
    er_owned = [np.ascontiguousarray(er[p.owned]) for er, p in zip(ersets, plans)]
    torch.cuda.synchronize(dev)
    rccl = distributed and os.environ.get("RSMI_BENCH_BACKEND", "nccl") == "nccl"
    # The exchange runs on its own stream under either backend (under gloo
    # the device rows are staged through host memory on that stream).
    comm = torch.cuda.Stream(dev) if distributed else None

    def step(i):
        return rd.run_step(f, held, plans[i], bufs, tables[i], er_owned[i], S, stream, comm)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    evs = [step(i) for i in range(warmup, warmup + steps)]
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    rec_ms = [a.elapsed_time(b) for a, b in evs if a is not None]
    rec_ms = sum(rec_ms) / len(rec_ms) if rec_ms else 0.0
    rec_bytes = sum(int(((k + ersets[i][plans[i].owned].sum(axis=1)) * S).sum())
                    for i in range(warmup, warmup + steps))
    xgmi_bytes = sum(plans[i].bytes_in for i in range(warmup, warmup + steps))
    # Check (untimed) the outputs of the last `outs` timed steps on a sample
    # of owned stripes: each stripe regenerated from the global stream and
    # encoded here, its erased shards compared with what the gather +
    # reconstruct wrote into that step's output buffer.
    chk_d = torch.empty(k * S, dtype=torch.uint8, device=dev)
    chk_p = torch.empty(m * S, dtype=torch.uint8, device=dev)
    bad = checked = 0
    checked_steps = list(range(warmup + steps - outs, warmup + steps))
    for si in checked_steps:
        pl = plans[si]
        out_buf = bufs.outs[si % outs]
        sample = np.unique(np.linspace(0, len(pl.owned) - 1, num=min(16, len(pl.owned))).astype(np.int64))
        for j in sample:
            gs = int(pl.owned[j])
            f.fill_splitmix(chk_d.data_ptr(), k * S, (0x5EED + gs * k * S // 8 * gamma) & (2**64 - 1), sh)
            f.encode_stripes(chk_d.data_ptr(), k * S, chk_p.data_ptr(), m * S, S, S, 1, sh)
            full = torch.cat([chk_d.view(k, S), chk_p.view(m, S)])
            for i in np.nonzero(ersets[si][gs])[0]:
                bad += int(not torch.equal(out_buf[int(pl.row[j, i])], full[i]))
            checked += 1
    torch.cuda.synchronize(dev)
    mine = torch.tensor([elapsed, rec_bytes, xgmi_bytes, budget["total"], plan_ms, checked, bad, rec_ms],
                        dtype=torch.float64, device=stats_device(dev))
    if distributed:
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(gathered, mine)
        per_rank = [g.tolist() for g in gathered]
    else:
        per_rank = [mine.tolist()]
    del held, bufs, tables
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    elapsed = max(r[0] for r in per_rank)
    return {"per_rank": per_rank, "elapsed": elapsed, "rec_total": sum(r[1] for r in per_rank),
            "xgmi_total": sum(r[2] for r in per_rank), "chunks": len(plans[0].chunks), "budget": budget,
            "free_b": free_b, "plan_ms": plan_ms, "rccl": rccl, "comm_stream": comm is not None,
            "backend": os.environ.get("RSMI_BENCH_BACKEND", "nccl") if distributed else "none",
            "verified": {"stripes": int(sum(r[5] for r in per_rank)),
                         "mismatched_shards": int(sum(r[6] for r in per_rank)),
                         "steps": [s - warmup for s in checked_steps],
                         "how": f"the last {outs} timed steps (own output buffers; the last step reused the "
                                "previous one's receive slots), up to 16 owned stripes per rank per step "
                                "regenerated and encoded locally"}}


def gather_summary(res, steps, world):
    """The survivor-gather leg's numbers (xGMI roofline: gathered bytes)."""
    xg = res["xgmi_total"] / res["elapsed"] / 1e9
    return {
        "reconstruct_GBps": round(res["rec_total"] / res["elapsed"] / 1e9, 2),
        "ms_per_step": round(res["elapsed"] / steps * 1e3, 3),
        "xgmi": {"gathered_GB": round(res["xgmi_total"] / 1e9, 3),
                 "gathered_GB_per_step": round(res["xgmi_total"] / steps / 1e9, 3),
                 "achieved_GBps_total": round(xg, 1), "per_rank_GBps": round(xg / max(world, 1), 1),
                 "link_peak_GBps": 153.0, "links_per_gpu": 7},
        "chunks": res["chunks"],
        "overlap": ("RCCL" if res["rccl"] else res.get("backend", "gloo") + " (host-staged)")
                   + " exchange of chunk c+1 on a communication stream || reconstruct of chunk c"
                   if res.get("comm_stream", res["rccl"]) else "none (chunks in sequence)",
        "hbm_budget_GB": {key: round(v, 2) for key, v in res["budget"].items()},
        "hbm_free_GB": round(res["free_b"] / 1e9, 1),
        "plan_ms_per_step": round(res["plan_ms"], 2),
        "reconstruct_stream_ms_per_step": round(max(r[7] for r in res["per_rank"]), 3)
        if len(res["per_rank"][0]) > 7 else None,
        "verified": res["verified"],
        "per_rank": [{"rank": r, "ms_per_step": round(v[0] / steps * 1e3, 3),
                      "gathered_GB_per_step": round(v[2] / steps / 1e9, 3),
                      "reconstruct_GBps": round(v[1] / v[0] / 1e9, 2),
                      "hbm_budget_GB": round(v[3], 2), "plan_ms": round(v[4], 2)}
                     for r, v in enumerate(res["per_rank"])],
    }


def sharded_main(args, world, rank, local, dev, distributed):
    """configs[3] as its own run (--placement sharded): see sharded_run."""
    import rsmi

    k, n, S = args.k, args.n, args.shard
    emax = args.emax if args.emax is not None else n - k
    f = rsmi.FEC(k, n, device=local)
    res = sharded_run(f, k, n, S, args.stripes, args.steps, args.warmup, args.emin, emax, args.pattern_pool,
                      args.chunks, world, rank, dev, distributed)
    if rank == 0:
        g = gather_summary(res, args.steps, world)
        emit({
            "metric": "RS(10,4) reconstruct GB/s with RCCL survivor gather (configs[3], sharded)",
            "value": g["reconstruct_GBps"], "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": g["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"RS({k},{n}) {args.emin}-{emax}-erasure reconstruct, shard i "
                                   f"on rank i mod N, {args.stripes} owned stripes x {S} B shards "
                                   "per rank", "placement": "sharded", "chunks": g["chunks"],
                       "overlap": g["overlap"]},
            "xgmi": g["xgmi"],
            "hbm_budget_GB": g["hbm_budget_GB"],
            "hbm_free_GB": g["hbm_free_GB"],
            "plan_ms_per_step": g["plan_ms_per_step"],
            "verified": g["verified"],
            "per_rank": g["per_rank"],
        })
    if distributed:
        torch.distributed.destroy_process_group()
    if res["verified"]["mismatched_shards"]:
        raise SystemExit("bench.py: sharded reconstruct produced wrong shards")


if __name__ == "__main__":
    main()
