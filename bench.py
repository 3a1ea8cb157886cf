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
the timed region at every N).

`--gpus N` with N > 1 and no launcher starts N ranks itself
(torch.distributed.run as a child process, the JSON line relayed); under a
launcher, WORLD_SIZE must equal --gpus.  At N > 1 the same ranks then run a
short shard-distributed leg (configs[3]: the RCCL survivor gather and the
pointer-mode reconstruct, checked on a sample) reported as "gather" -- never
part of value, and abandoned by a per-rank watchdog rather than allowed to
cost the headline line.
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
                    help="budget of the CPU baseline sample (0 disables)")
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
                    help="seconds after which a stuck gather leg is abandoned (the line is still printed)")
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


def main():
    global _RESULT_OUT
    args = parse()
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
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    data = torch.empty(stripes * k * S, dtype=torch.uint8, device=dev)
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device=dev)
    f.fill_splitmix(data.data_ptr(), data.numel(), 0x5EED ^ (rank << 32), sh)
    f.fill_splitmix(parity.data_ptr(), parity.numel(), 1, sh)
    pool = args.pattern_pool
    prep_ms = None
    if pattern_total(n, emax) <= (1 << 20):
        # Every pattern inverted on the GPU + uploaded once, before timing (a
        # context keeps them cached for its lifetime); its one-off cost is
        # reported as breakdown.pattern_prepare_ms.
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        f.prepare_patterns(emax, sh)
        torch.cuda.synchronize(dev)
        prep_ms = (time.perf_counter() - tp) * 1e3
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
    if not do_enc:  # reconstruct needs valid parity once
        f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, sh)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i, timed):
        e = ev[i - args.warmup] if timed else None
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

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        step(i, True)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    enc_ms = [a.elapsed_time(b) for a, b, _ in ev]
    rec_ms = [b.elapsed_time(c) for _, b, c in ev]
    # Per-rank wall time and kernel times; the job's time is the max.
    mine = torch.tensor([elapsed, sum(enc_ms) / len(enc_ms), sum(rec_ms) / len(rec_ms)],
                        dtype=torch.float64, device=stats_device(dev))
    if distributed:
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        torch.distributed.all_gather(gathered, mine)
        per_rank = [g.tolist() for g in gathered]
    else:
        per_rank = [mine.tolist()]
    elapsed = max(r[0] for r in per_rank)
    step_bytes_local = sum((enc_bytes if do_enc else 0) + (rec_bytes[i] if do_rec else 0)
                           for i in range(args.warmup, args.warmup + args.steps))
    total_bytes = step_bytes_local * world
    value = total_bytes / elapsed / 1e9

    enc_avg_ms = sum(enc_ms) / len(enc_ms)
    rec_avg_ms = sum(rec_ms) / len(rec_ms)
    rec_avg_bytes = sum(rec_bytes[args.warmup:]) / args.steps
    dominant = "encode" if do_enc else "reconstruct"
    dom_bytes = enc_bytes if do_enc else rec_avg_bytes
    dom_ms = enc_avg_ms if do_enc else rec_avg_ms
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    traffic = None
    try:
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        key = f"{dominant}_k{k}_n{n}_S{S}_stripes{stripes}"
        traffic = tj.get(key)
    except (OSError, ValueError):
        pass

    local_bytes = step_bytes_local
    out = None
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0:  # after the timed region, on rank 0, at every N
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
            },
            "cpu_baseline": cpu,
            "per_rank": [{"rank": r, "ms_per_step": round(v[0] / args.steps * 1e3, 3),
                          "value": round(local_bytes / v[0] / 1e9, 2),
                          "encode_ms": round(v[1], 3), "reconstruct_ms": round(v[2], 3)}
                         for r, v in enumerate(per_rank)],
        }
    if distributed and world > 1 and args.gather_stripes > 0:
        # configs[3]'s survivor gather on the same ranks, after the headline
        # is measured: its own buffers, so the local ones go first.
        del data, parity
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        gather_leg(args, f, k, n, S, emax, world, rank, dev, out)  # emits the line and tears down
        return
    if rank == 0:
        emit(out)
    if distributed:
        torch.distributed.destroy_process_group()


def gather_leg(args, f, k, n, S, emax, world, rank, dev, out):
    """N > 1: a short shard-distributed leg (sharded_run with
    --gather-stripes owned stripes per rank, 1 warm-up + 2 timed steps,
    every step checked on a sample) reported as out["gather"].  A watchdog
    per rank abandons a leg stuck in a collective after --gather-timeout
    seconds: rank 0 still prints the headline line (gather.status says
    what happened) and every rank exits, so the headline measurement is
    never lost to the extra leg.  Wrong shards exit non-zero after the
    line is printed."""
    import threading

    lock = threading.Lock()
    state = {"emitted": False}

    def finish(gather):
        with lock:
            if state["emitted"]:
                return False
            state["emitted"] = True
        if rank == 0 and out is not None:
            out["gather"] = gather
            emit(out)
        return True

    def abandon():
        if finish({"status": f"abandoned after {args.gather_timeout:.0f} s (collective did not complete)"}):
            sys.stderr.write("bench.py: gather leg abandoned\n")
            sys.stderr.flush()
            os._exit(0)

    torch.distributed.barrier()  # rank 0's CPU baseline is done: start every clock together
    timer = threading.Timer(args.gather_timeout, abandon)
    timer.daemon = True
    timer.start()
    steps, warmup = 2, 1
    gather = {"status": "ok", "owned_stripes_per_rank": args.gather_stripes, "shard_bytes": S,
              "steps": steps, "warmup": warmup,
              "what": "shard i of every stripe on rank i mod N; each owner gathers exactly Rebuild's "
                      "survivors over RCCL (batch_isend_irecv) and reconstructs from the receive buffers "
                      "(rs_reconstruct_ptrs); not part of value"}
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
    finish(gather)
    if bad:
        raise SystemExit("bench.py: the gather leg reconstructed wrong shards")


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


def sharded_run(f, k, n, S, stripes, steps, warmup, emin, emax, pool, chunks, world, rank, dev, distributed,
                budget_exit=True):
    """configs[3], shard-distributed placement: shard i of every stripe is
    held by rank i mod N (the p2p analogue of main.go:207 broadcasting each
    shard to peers).  One step = the survivor gather (exactly the survivors
    each owner reads, rsmi/distributed.py) in `chunks` chunks, chunk c + 1's
    RCCL exchange (communication stream) overlapping chunk c's
    rs_reconstruct_ptrs (compute stream), which reads survivors where they
    landed.  The per-rank HBM budget is computed before anything is
    allocated; a budget over the free HBM raises the chunk count, and past
    64 chunks exits non-zero with the numbers (budget_exit) or returns None.
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
    chunks = max(1, chunks)
    while True:
        tp = time.perf_counter()
        plans = [rd.plan_exchange(er, k, n, rank, world, S, chunks=chunks) for er in ersets]
        plan_ms = (time.perf_counter() - tp) * 1e3 / len(ersets)
        budget = rd.hbm_budget(gstripes, len(ids), S, plans, n, k=k)
        if budget["total"] * 1e9 <= free_b - (4 << 30) or chunks >= 64:
            break
        chunks *= 2
    if budget["total"] * 1e9 > free_b - (4 << 30):
        sys.stderr.write(f"bench.py: sharded placement needs {budget['total']:.1f} GB per rank "
                         f"({', '.join(f'{key} {v:.1f}' for key, v in budget.items() if key != 'total')}) "
                         f"but {free_b / 1e9:.1f} GB are free: lower --stripes\n")
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
    bufs = rd.make_buffers(plans, S, dev)
    tables = [torch.from_numpy(rd.shard_table(p, held, bufs)).to(dev) for p in plans]
    er_owned = [np.ascontiguousarray(er[p.owned]) for er, p in zip(ersets, plans)]
    torch.cuda.synchronize(dev)
    rccl = distributed and os.environ.get("RSMI_BENCH_BACKEND", "nccl") == "nccl"
    comm = torch.cuda.Stream(dev) if rccl else None

    def step(i):
        rd.run_step(f, held, plans[i], bufs, tables[i], er_owned[i], S, stream, comm)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(i)
    torch.cuda.synchronize(dev)
    if distributed:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    rec_bytes = sum(int(((k + ersets[i][plans[i].owned].sum(axis=1)) * S).sum())
                    for i in range(warmup, warmup + steps))
    xgmi_bytes = sum(plans[i].bytes_in for i in range(warmup, warmup + steps))
    # Check (untimed) the last step's outputs on a sample of owned stripes:
    # each stripe regenerated from the global stream and encoded here, its
    # erased shards compared with what the gather + reconstruct produced.
    last = plans[-1]
    sample = np.unique(np.linspace(0, len(last.owned) - 1, num=min(16, len(last.owned))).astype(np.int64))
    chk_d = torch.empty(k * S, dtype=torch.uint8, device=dev)
    chk_p = torch.empty(m * S, dtype=torch.uint8, device=dev)
    bad = 0
    for j in sample:
        gs = int(last.owned[j])
        f.fill_splitmix(chk_d.data_ptr(), k * S, (0x5EED + gs * k * S // 8 * gamma) & (2**64 - 1), sh)
        f.encode_stripes(chk_d.data_ptr(), k * S, chk_p.data_ptr(), m * S, S, S, 1, sh)
        full = torch.cat([chk_d.view(k, S), chk_p.view(m, S)])
        for i in np.nonzero(ersets[-1][gs])[0]:
            bad += int(not torch.equal(bufs.out[int(last.row[j, i])], full[i]))
    torch.cuda.synchronize(dev)
    mine = torch.tensor([elapsed, rec_bytes, xgmi_bytes, budget["total"], plan_ms, len(sample), bad],
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
            "free_b": free_b, "plan_ms": plan_ms, "rccl": rccl,
            "verified": {"stripes": int(sum(r[5] for r in per_rank)),
                         "mismatched_shards": int(sum(r[6] for r in per_rank)),
                         "how": "last step, up to 16 owned stripes per rank regenerated and encoded locally"}}


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
        "overlap": "RCCL exchange of chunk c+1 on a communication stream || reconstruct of chunk c"
                   if res["rccl"] else "none (gloo rehearsal: chunks in sequence)",
        "hbm_budget_GB": {key: round(v, 2) for key, v in res["budget"].items()},
        "hbm_free_GB": round(res["free_b"] / 1e9, 1),
        "plan_ms_per_step": round(res["plan_ms"], 2),
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
