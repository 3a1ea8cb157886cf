#!/usr/bin/env python3
"""Host topology seen by a GPU job: the CPUs this process may use and their
NUMA nodes, and the NUMA node of each visible AMD GPU's PCI function (from
sysfs; no HIP call).  Prints JSON; `--pick` prints one allowed CPU per NUMA
node (space-separated) for A/B runs that pin the caller (RSMI_PIN_CPU)."""
import glob
import json
import os
import sys


def node_of_cpu(c):
    for d in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
        if d.startswith("node"):
            return int(d[4:])
    return -1


allowed = sorted(os.sched_getaffinity(0))
by_node = {}
for c in allowed:
    by_node.setdefault(node_of_cpu(c), []).append(c)
gpus = []
for dev in sorted(glob.glob("/sys/bus/pci/devices/*")):
    try:
        vendor = open(f"{dev}/vendor").read().strip()
        cls = open(f"{dev}/class").read().strip()
    except OSError:
        continue
    if vendor == "0x1002" and cls.startswith("0x038"):  # AMD display / processing accelerator
        try:
            numa = int(open(f"{dev}/numa_node").read())
        except (OSError, ValueError):
            numa = -1
        gpus.append({"pci": os.path.basename(dev), "numa_node": numa})
if "--pick" in sys.argv:
    print(" ".join(str(v[len(v) // 2]) for _, v in sorted(by_node.items())))
else:
    print(json.dumps({"allowed_cpus": allowed, "cpus_by_node": {str(k): v for k, v in by_node.items()},
                      "nodes_total": len(glob.glob("/sys/devices/system/node/node*")), "amd_gpus": gpus}))
