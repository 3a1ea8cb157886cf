"""bench.py end to end on the GPU, as child processes (the way the driver
runs it), at small sizes:

* N = 2 under the gloo rehearsal backend (two ranks sharing cuda:0): the
  self-launch, the stripe-local headline with per-rank bytes (no CPU
  baseline: it is timed at N = 1 only), and the configs[3] gather leg -- survivors exchanged between the
  ranks on a communication stream, reconstructed through rs_reconstruct_ptrs
  and checked against locally re-encoded stripes over the last two timed
  steps (the step whose receive slots the next step reused, and the last);
* N = 1 with rank 0's CPU baseline and the configs[0] (per-message latency, checked against the oracle
  inside the leg) and configs[4] (RS(64,16)) legs.

The driver's 8-GPU run uses RCCL instead of gloo; everything else is this
code."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_gloo_with_gather_leg(torch_dev):
    d = _run(["--gpus", "2", "--stripes", "64", "--shard", "65536", "--steps", "2", "--warmup", "1",
              "--cpu-seconds", "0.5", "--gather-stripes", "16", "--gather-timeout", "150"],
             {"RSMI_BENCH_BACKEND": "gloo"})
    assert d["n_gpus"] == 2 and len(d["per_rank"]) == 2
    # value = the two ranks' own bytes over the slower rank's time
    secs = max(r["ms_per_step"] for r in d["per_rank"]) * d["steps"] / 1e3
    total = sum(r["bytes"] for r in d["per_rank"])
    assert abs(d["value"] - total / secs / 1e9) <= 0.01 * d["value"] + 0.02
    assert d["cpu_baseline"] is None  # timed at N = 1 only
    g = d["gather"]
    assert g["status"] == "ok", g
    assert g["backend"] == "gloo" and "gloo" in g["what"] and "RCCL (" not in g["what"]
    assert g["verified"]["mismatched_shards"] == 0 and g["verified"]["stripes"] >= 2
    assert g["verified"]["steps"] == [0, 1]
    assert g["xgmi"]["gathered_GB"] > 0
    assert "communication stream" in g["overlap"]
    assert "device_set" not in d  # N = 1 only


@pytest.mark.gpu
def test_bench_single_gpu_extra_legs(torch_dev):
    d = _run(["--stripes", "64", "--shard", "65536", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0.2",
              "--config1-reps", "3", "--config5-stripes", "64", "--config5-steps", "2", "--config5-warmup", "1",
              "--config3-steps", "2", "--device-set-stripes", "24"])
    assert d["n_gpus"] == 1 and d["roofline"]["frac"] > 0
    assert d["cpu_baseline"] and d["cpu_baseline"]["value"] > 0
    c1 = d["config1"]
    assert c1["status"] == "ok", c1
    assert c1["message_bytes"] == 1048580 and len(c1["dropped"]) == 4
    assert c1["codec"]["encode_ms"] > 0 and c1["codec"]["decode4_ms"] > 0 and c1["codec"]["decode4_arena_ms"] > 0
    assert c1["codec"]["decode4_batch64_ms_per_message"] > 0
    assert c1["codec"]["encode_batch64_ms_per_message"] > 0 and c1["gpu_vs_1core"]["encode_batch64"] > 0
    assert set(c1["cpu_1t"]) == {"scalar_1t", "avx2_1t"}
    c5 = d["config5"]
    assert c5["status"] == "ok", c5
    assert c5["encode"]["GBps"] > 0 and c5["reconstruct"]["GBps"] > 0
    assert c5["encode"]["bytes"] == 64 * 80 * 65536
    c3 = d["config3_worst"]
    assert c3["status"] == "ok", c3
    assert c3["reconstruct"]["bytes"] == 64 * 14 * 65536 and c3["reconstruct"]["GBps"] > 0
    ds = d["device_set"]
    assert ds["status"] == "ok" and ds["checked"], ds
    assert ds["members"] == max(2, ds["members"]) and ds["stripes_per_member"] == 24
    assert ds["encode"]["GBps"] > 0 and ds["reconstruct"]["GBps"] > 0
    assert ds["spread"]["status"] == "ok" and ds["spread"]["GBps"] > 0, ds["spread"]
