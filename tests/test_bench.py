"""bench.py's host-side pieces on the CPU: the config-3 erasure generator,
the pattern count that decides up-front preparation, the CPU description and
the cpu_baseline leg structure (the oracle timed on a tiny sample).  The GPU
line itself is produced by the driver on an MI355X."""
import os
import sys

import numpy as np
import pytest

import bench


def test_erasure_sets_counts_and_determinism():
    n, stripes = 14, 500
    a = bench.erasure_sets(np.random.default_rng(0xE4A5), 3, stripes, n, 1, 4)
    b = bench.erasure_sets(np.random.default_rng(0xE4A5), 3, stripes, n, 1, 4)
    assert len(a) == 3
    for x, y in zip(a, b):
        assert x.shape == (stripes, n) and x.dtype == np.uint8
        assert np.array_equal(x, y)
        e = x.sum(axis=1)
        assert e.min() >= 1 and e.max() <= 4
        assert set(np.unique(e)) == {1, 2, 3, 4}  # uniform count: all occur at this size
    assert not np.array_equal(a[0], a[1])  # a fresh erasure set per step


def test_erasure_sets_pattern_pool():
    sets = bench.erasure_sets(np.random.default_rng(1), 2, 1000, 80, 1, 16, pool=7)
    for er in sets:
        assert len({row.tobytes() for row in er}) <= 7
        assert er.sum(axis=1).max() <= 16


def test_pattern_total_decides_preparation():
    assert bench.pattern_total(14, 4) == 14 + 91 + 364 + 1001 == 1470
    assert bench.pattern_total(6, 2) == 6 + 15
    assert bench.pattern_total(80, 16) > (1 << 20)  # config 5: patterns built on demand


def test_host_cpu_info():
    info = bench.host_cpu_info()
    assert set(info) == {"model", "host_cpus", "usable_cpus", "cgroup_quota_cpus"}
    assert 1 <= info["usable_cpus"] <= info["host_cpus"]


def test_cpu_baseline_legs():
    cpu = bench.cpu_baseline(4, 6, 4096, 0.2, 2)
    assert cpu["kind"] == "port" and cpu["unit"] == "GB/s" and cpu["cores"] == 2
    assert set(cpu["legs"]) == {"scalar_1t", "scalar_all", "avx2_1t", "avx2_all"}
    assert cpu["value"] == cpu["legs"]["avx2_all"]["GBps"] > 0
    assert all(leg["stripes"] > 0 for leg in cpu["legs"].values())


@pytest.mark.parametrize("backend,want", [("nccl", "meta"), ("gloo", "cpu")])
def test_stats_device(monkeypatch, backend, want):
    import torch
    monkeypatch.setenv("RSMI_BENCH_BACKEND", backend)
    assert bench.stats_device(torch.device("meta")).type == want


def test_parse_stream_mode(monkeypatch):
    """bench.py --stream (configs[1] second mode) parses with its chunk size;
    the default run stays device-resident."""
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert not a.stream and a.placement == "local"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--stream", "--stream-chunk", "16"])
    a = bench.parse()
    assert a.stream and a.stream_chunk == 16


def test_check_world_modes():
    """--gpus N decides how bench.py runs: one process at N = 1, a self-launch
    of N ranks with no launcher, and a rank under a launcher whose WORLD_SIZE
    must equal --gpus (a mismatch exits non-zero rather than recording the
    wrong GPU count)."""
    assert bench.check_world(1, {}) == "single"
    assert bench.check_world(8, {}) == "launch"
    assert bench.check_world(8, {"WORLD_SIZE": "8", "RANK": "3"}) == "rank"
    assert bench.check_world(1, {"WORLD_SIZE": "1", "RANK": "0"}) == "rank"
    for gpus, env in ((8, {"WORLD_SIZE": "1", "RANK": "0"}), (1, {"WORLD_SIZE": "2", "RANK": "1"}),
                      (2, {"RANK": "0"})):
        with pytest.raises(SystemExit) as ei:
            bench.check_world(gpus, env)
        assert ei.value.code == 2
    with pytest.raises(SystemExit):
        bench.check_world(0, {})


def test_launch_command_passes_every_flag():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5", "--placement", "sharded", "--erase", "0,1"]
    cmd = bench.launch_command(8, argv, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == argv


def test_self_launch_relays_one_json_line(monkeypatch, capsys):
    """The parent relays rank 0's JSON line to stdout (anything else the
    ranks print goes to stderr) and returns the child's exit code."""
    prog = ("import sys; print('banner'); print('{\"metric\": \"m\", \"n_gpus\": 2}'); "
            "sys.stdout.flush(); sys.exit(%d)")
    monkeypatch.setattr(bench, "launch_command", lambda g, a, p: [sys.executable, "-c", prog % 0])
    assert bench.self_launch(2, []) == 0
    out = capsys.readouterr()
    assert out.out.strip() == '{"metric": "m", "n_gpus": 2}'
    assert "banner" in out.err
    monkeypatch.setattr(bench, "launch_command", lambda g, a, p: [sys.executable, "-c", prog % 3])
    assert bench.self_launch(2, []) == 3
    monkeypatch.setattr(bench, "launch_command", lambda g, a, p: [sys.executable, "-c", "print('x')"])
    assert bench.self_launch(2, []) == 1  # exit 0 but no JSON line


def test_gather_summary_arithmetic():
    """The N > 1 gather leg's report (bench.gather_summary): totals over ranks
    against the max-over-ranks time, per-rank rows, xGMI figures."""
    per_rank = [[2.0, 40e9, 10e9, 12.5, 1.0, 16, 0], [1.6, 36e9, 8e9, 12.0, 1.2, 16, 0]]
    res = {"per_rank": per_rank, "elapsed": 2.0, "rec_total": 76e9, "xgmi_total": 18e9, "chunks": 8,
           "budget": {"held": 8.0, "total": 12.5}, "free_b": 280e9, "plan_ms": 0.5, "rccl": True,
           "verified": {"stripes": 32, "mismatched_shards": 0, "how": "x"}}
    g = bench.gather_summary(res, steps=2, world=2)
    assert g["reconstruct_GBps"] == 38.0 and g["ms_per_step"] == 1000.0
    assert g["xgmi"]["gathered_GB"] == 18.0 and g["xgmi"]["gathered_GB_per_step"] == 9.0
    assert g["xgmi"]["achieved_GBps_total"] == 9.0 and g["xgmi"]["per_rank_GBps"] == 4.5
    assert g["overlap"].startswith("RCCL")
    assert [r["rank"] for r in g["per_rank"]] == [0, 1]
    assert g["per_rank"][1]["ms_per_step"] == 800.0 and g["per_rank"][1]["reconstruct_GBps"] == 22.5
    assert g["hbm_free_GB"] == 280.0 and g["verified"]["stripes"] == 32
    res["rccl"] = False
    assert bench.gather_summary(res, 2, 2)["overlap"].startswith("none")


def test_gather_flags_pass_through_the_launcher():
    argv = ["--gpus", "8", "--gather-stripes", "256", "--gather-timeout", "60"]
    cmd = bench.launch_command(8, argv, 29500)
    assert cmd[-len(argv):] == argv and "--nproc-per-node=8" in cmd


def test_job_totals_sum_each_ranks_own_bytes():
    """value = every rank's own algorithmic bytes summed over the slowest
    rank's time (ranks draw their own erasure sets, so their reconstruct
    bytes differ: rank 0's bytes x world would be wrong)."""
    per_rank = [[2.0, 1.0, 1.0, 100.0], [2.5, 1.0, 1.0, 130.0], [1.5, 1.0, 1.0, 90.0]]
    secs, total = bench.job_totals(per_rank)
    assert secs == 2.5 and total == 320.0
    assert bench.job_totals([[1.0, 7.0]]) == (1.0, 7.0)


def test_gather_watchdog_prints_once_then_exits_nonzero(monkeypatch):
    """An abandoned gather leg prints the headline line (gather.status says
    what happened) and ends the process with EXIT_GATHER_ABANDONED, never 0;
    a leg that finished first keeps the watchdog from printing again or
    exiting."""
    lines = []
    monkeypatch.setattr(bench, "emit", lambda obj: lines.append(dict(obj)))
    codes = []
    line = bench.OnceLine(0, {"metric": "m", "value": 1.0})
    bench.make_abandon(line, 5.0, exit_fn=codes.append)()
    assert codes == [bench.EXIT_GATHER_ABANDONED] and bench.EXIT_GATHER_ABANDONED != 0
    assert len(lines) == 1 and lines[0]["gather"]["status"].startswith("abandoned after 5 s")
    bench.make_abandon(line, 5.0, exit_fn=codes.append)()  # second firing: nothing
    assert codes == [bench.EXIT_GATHER_ABANDONED] and len(lines) == 1
    done = bench.OnceLine(0, {"metric": "m"})
    assert done.finish({"status": "ok"})
    bench.make_abandon(done, 5.0, exit_fn=codes.append)()
    assert codes == [bench.EXIT_GATHER_ABANDONED] and len(lines) == 2
    other = bench.OnceLine(1, {"metric": "m"})  # rank 1 prints nothing but still exits non-zero
    bench.make_abandon(other, 5.0, exit_fn=codes.append)()
    assert codes[-1] == bench.EXIT_GATHER_ABANDONED and len(lines) == 2


def test_gather_what_names_the_backend():
    assert "RCCL" in bench.gather_what("nccl") and "gloo" not in bench.gather_what("nccl")
    g = bench.gather_what("gloo")
    assert "gloo" in g and "RCCL" not in g


def test_gather_summary_overlap_names_the_backend():
    per_rank = [[2.0, 40e9, 10e9, 12.5, 1.0, 16, 0, 3.0]]
    res = {"per_rank": per_rank, "elapsed": 2.0, "rec_total": 40e9, "xgmi_total": 10e9, "chunks": 2,
           "budget": {"total": 1.0}, "free_b": 1e9, "plan_ms": 0.5, "rccl": False, "comm_stream": True,
           "backend": "gloo", "verified": {"stripes": 16, "mismatched_shards": 0, "how": "x"}}
    g = bench.gather_summary(res, 2, 1)
    assert g["overlap"].startswith("gloo (host-staged) exchange") and g["reconstruct_stream_ms_per_step"] == 3.0
    res["rccl"], res["backend"] = True, "nccl"
    assert bench.gather_summary(res, 2, 1)["overlap"].startswith("RCCL exchange")


def test_agree_max_without_a_process_group():
    assert bench.agree_max(8, False, None) == 8


def test_extra_leg_flags(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.extra_legs and a.config5_stripes == 16384 and a.config1_reps > 0
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-extra-legs", "--config5-stripes", "64"])
    a = bench.parse()
    assert not a.extra_legs and a.config5_stripes == 64


def test_guarded_leg_reports_failures():
    assert bench.guarded_leg(lambda: {"status": "ok"}) == {"status": "ok"}
    r = bench.guarded_leg(lambda: 1 / 0)
    assert r["status"].startswith("error: ZeroDivisionError")


def _agree_worker(rank, world, port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RSMI_BENCH_BACKEND="gloo")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import torch
        got = (bench.agree_max([2, 8][rank], True, torch.device("cpu")),
               bench.agree_max([0, 1][rank], True, torch.device("cpu")))
        dist.destroy_process_group()
        q.put((rank, got))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_agree_max_gloo_world2():
    """Every rank ends with the same chunk count (the max) and the same
    fits verdict (any rank over budget -> none runs)."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: (8, 1), 1: (8, 1)}, res


def test_cpulist_and_pin_opt_out(monkeypatch):
    import bench
    assert bench._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert bench._cpulist("") == set()
    monkeypatch.setenv("RSMI_BENCH_NO_PIN", "1")
    assert bench.pin_to_gpu_numa(0) == {"pinned": False, "why": "RSMI_BENCH_NO_PIN"}
