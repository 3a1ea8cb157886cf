#!/usr/bin/env python3
"""Summarise rocprofv3 passes of ONE default bench.py line (headline +
config1 + config5 legs; tools/gpu/r04*.sh layout):

  <dir>/trace/run_kernel_trace.csv   --kernel-trace --stats
  <dir>/fetch/run_counter_collection.csv, <dir>/write/...   --pmc FETCH_SIZE / WRITE_SIZE (optional)

Launches are told apart by kernel, grid size and launch order:
  headline   the first 2 x (warmup + steps) rs_matmul_kernel launches with the
             largest grid, alternating encode / reconstruct (bench.py --mode
             both);
  config3    the later largest-grid launches (the configs[2] worst-case leg:
             one encode, then its reconstructs);
  config1    the other rs_matmul_kernel launches (the host-API calls on
             1,048,580-byte messages, the device-set leg's member launches);
  config5    rs_bitslice_k64_m16 (encode) and rs_bitslice_rec_k64_m16
             (reconstruct), invert_patterns_kernel (the fresh patterns).
HBM traffic per launch = FETCH_SIZE x 1024 x 2 + WRITE_SIZE x 1024 (the gfx950
correction of /opt/skills/guides/MI355X_MICROARCH.md), matched to the trace's
roles by launch order within each kernel.  Writes markdown to <out> and, with
--traffic-json, the headline's per-launch traffic for bench.py's
roofline.traffic.

usage: tools/prof_line.py <dir> <out.md> [--bench-json line.json] [--traffic-json profiles/traffic.json]
"""
import argparse
import csv
import json
import os
import statistics


def rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def ms(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6


def grid(r):
    return int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)


def short(name):
    for key in ("rs_bitslice_rec_k", "rs_bitslice_k", "rs_matmul_kernel", "invert_patterns_kernel"):
        if key in name:
            rest = name[name.index(key):]
            return rest.split("(")[0] if key != "rs_matmul_kernel" else rest.split(">")[0] + ">"
    return name[:40]


HEAD_LAUNCHES = 2 * (3 + 10)  # bench.py defaults: --warmup 3 --steps 10, encode + reconstruct each


def roles(trace):
    """{role: [trace rows]} in launch order."""
    mm = [r for r in trace if "rs_matmul_kernel" in r["Kernel_Name"]]
    big = max((grid(r) for r in mm), default=0)
    top = [r for r in mm if grid(r) == big]
    head, worst = top[:HEAD_LAUNCHES], top[HEAD_LAUNCHES:]
    out = {"headline encode": head[0::2], "headline reconstruct": head[1::2],
           "config3 worst-case reconstruct": worst[1:],
           "config1 + device-set launches (host-API messages, members)": [r for r in mm if grid(r) != big],
           "config5 encode": [r for r in trace if "rs_bitslice_k64_m16" in r["Kernel_Name"]],
           "config5 reconstruct": [r for r in trace if "rs_bitslice_rec_k64_m16" in r["Kernel_Name"]],
           "pattern builds": [r for r in trace if "invert_patterns_kernel" in r["Kernel_Name"]]}
    return {k: v for k, v in out.items() if v}


def pmc_by_role(d, counter):
    """Counter values per role, matching the trace's classification: the
    counter rows carry the grid size too."""
    rs = [r for r in rows(os.path.join(d, counter.lower().split("_")[0], "run_counter_collection.csv"))
          if r["Counter_Name"] == counter]
    if not rs:
        return {}
    return {k: [float(r["Counter_Value"]) for r in v] for k, v in roles(rs).items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--bench-json", default=None)
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--profile", default=None, help="profile tag / path recorded in each traffic.json entry")
    a = ap.parse_args()
    a.profile = a.profile or a.dir
    trace = rows(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))
    rl = roles(trace)
    fetch = pmc_by_role(a.dir, "FETCH_SIZE")
    write = pmc_by_role(a.dir, "WRITE_SIZE")
    b = json.load(open(a.bench_json)) if a.bench_json and os.path.exists(a.bench_json) else None
    # algorithmic bytes per launch
    alg = {"headline encode": 6553 * 14 * (1 << 20),
           "headline reconstruct": 6553 * (10 + 2.5) * (1 << 20),   # E[e] = 2.5 for 1..4 uniform
           "config3 worst-case reconstruct": 6553 * 14 * (1 << 20),
           "config1 + device-set launches (host-API messages, members)": None,
           "config5 encode": 16384 * 80 * 65536,
           "config5 reconstruct": 16384 * (64 + 8.5) * 65536}       # E[e] = 8.5 for 1..16 uniform
    if b and "config" in b:
        c = b["config"]
        alg["headline encode"] = c["stripes_per_gpu"] * c["n"] * c["shard_bytes"]
        alg["headline reconstruct"] = c["stripes_per_gpu"] * (c["k"] + (c["n"] - c["k"] + 1) / 2) * c["shard_bytes"]
    if b and isinstance(b.get("config5"), dict) and b["config5"].get("status") == "ok":
        alg["config5 encode"] = b["config5"]["encode"]["bytes"]
        alg["config5 reconstruct"] = b["config5"]["reconstruct"]["bytes"]
    if b and isinstance(b.get("config3_worst"), dict) and b["config3_worst"].get("status") == "ok":
        alg["config3 worst-case reconstruct"] = b["config3_worst"]["reconstruct"]["bytes"]
    lines = [f"# rocprofv3 summary of one bench.py line: {os.path.basename(os.path.normpath(a.dir))}", "",
             "Kernel trace (`--kernel-trace --stats`) plus, when present, separate `--pmc FETCH_SIZE` and "
             "`--pmc WRITE_SIZE` passes of the same command; traffic = FETCH_SIZE x 2 + WRITE_SIZE (gfx950 "
             "correction, MI355X_MICROARCH §HBM).  Reconstruct algorithmic bytes are the expectation over the "
             "uniform erasure counts (each profiled launch drew its own sets).", "",
             "| role | kernel | launches | avg ms | algorithmic GB / launch | achieved GB/s | frac of 8 TB/s | "
             "traffic GB / launch | traffic / algorithmic |",
             "|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for role, rs in rl.items():
        d = [ms(r) for r in rs]
        avg = statistics.mean(d)
        kern = short(rs[0]["Kernel_Name"])
        al = alg.get(role)
        f, w = fetch.get(role), write.get(role)
        tr = (statistics.mean(f) * 2 + statistics.mean(w)) * 1024 / 1e9 if f and w else None
        ach = al / (avg / 1e3) / 1e9 if al else None
        lines.append(f"| {role} | `{kern}` | {len(d)} | {avg:.3f} | "
                     f"{al / 1e9 if al else float('nan'):.2f} | {ach if ach else float('nan'):.0f} | "
                     f"{ach / 8000 if ach else float('nan'):.4f} | {tr if tr is not None else float('nan'):.3f} | "
                     f"{tr / (al / 1e9) if (tr is not None and al) else float('nan'):.3f} |")
        # profiles/traffic.json entries (bench.py roofline.traffic / traffic_source),
        # keyed by role and workload, each naming the kernel and this profile
        key = {"headline encode": "encode_k10_n14_S1048576_stripes6553",
               "headline reconstruct": "reconstruct_k10_n14_S1048576_stripes6553",
               "config3 worst-case reconstruct": "config3_worst_reconstruct_k10_n14_S1048576_stripes6553",
               "config5 encode": "config5_encode_k64_n80_S65536_stripes16384",
               "config5 reconstruct": "config5_reconstruct_k64_n80_S65536_stripes16384"}.get(role)
        if key and b:
            c = b["config"]
            if role.startswith("headline"):
                key = f"{role.split()[1]}_k{c['k']}_n{c['n']}_S{c['shard_bytes']}_stripes{c['stripes_per_gpu']}"
            traffic[key] = {"kernel": kern, "launches": len(d), "trace_ms": round(avg, 3),
                            "algorithmic_GB": round(al / 1e9, 3) if al else None,
                            "trace_frac": round(ach / 8000, 4) if ach else None,
                            "traffic_GB": round(tr, 3) if tr is not None else None,
                            "traffic_ratio": round(tr / (al / 1e9), 4) if (tr is not None and al) else None,
                            "profile": a.profile}
    lines.append("")
    stats = rows(os.path.join(a.dir, "trace", "run_kernel_stats.csv"))
    if stats:
        lines += ["## rocprofv3 --stats (all launches of the line)", "",
                  "| kernel | calls | avg ms | min ms | max ms | % time |", "|---|---|---|---|---|---|"]
        for r in stats:
            lines.append(f"| `{r['Name'][:80]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | "
                         f"{float(r['MinNs']) / 1e6:.3f} | {float(r['MaxNs']) / 1e6:.3f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    if b:
        lines.append(f"bench.py line of the profiled run: value {b['value']} GB/s, encode {b['breakdown']['encode_ms']} ms "
                     f"(HIP events, frac {b['roofline']['frac']}), reconstruct {b['breakdown']['reconstruct_ms']} ms"
                     + (f"; config5 encode {b['config5']['encode']['ms']} / reconstruct {b['config5']['reconstruct']['ms']} ms"
                        if isinstance(b.get("config5"), dict) and b["config5"].get("status") == "ok" else "")
                     + (f"; config1 encode {b['config1']['codec']['encode_ms']} / decode {b['config1']['codec']['decode4_ms']} ms"
                        if isinstance(b.get("config1"), dict) and b["config1"].get("status") == "ok" else "") + ".")
    with open(a.out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    if a.traffic_json and traffic:
        out = {"_note": "per-launch HBM traffic (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction) and "
                        "kernel-trace time of each role of one default bench.py line, keyed by role and workload; "
                        "bench.py copies the entry of its dominant kernel into roofline.traffic / traffic_source. "
                        "Written by tools/prof_line.py.",
               "entries": traffic}
        json.dump(out, open(a.traffic_json, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
