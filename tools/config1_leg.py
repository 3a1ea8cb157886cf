#!/usr/bin/env python3
"""bench.py's configs[0] leg alone (per-message encode / decode latency against
one host core), for A/B runs of the single-message path without the headline
legs.  Usage: python3 tools/config1_leg.py [reps]  -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
bench.torch.cuda.set_device(0)
aff = bench.pin_to_gpu_numa(0)  # as bench.py does (RSMI_BENCH_NO_PIN=1: not)
d = bench.config1_leg(0, reps)
print(json.dumps({"codec": d.get("codec"), "cpu_1t": d.get("cpu_1t"), "gpu_vs_1core": d.get("gpu_vs_1core"),
                  "host_affinity": aff}))
