#!/usr/bin/env python3
"""Summarise a tools/pmc_valu.sh SQ pass: per coding kernel, VALU
instructions per wave, the fraction of wave cycles issuing VALU / stalled on
issue / waiting, and the 'VALU-bound clock' (SQ_INSTS_VALU x 4 cycles over
the 1,024 SIMDs, divided by the kernel's duration): ~the profiled clock means
every SIMD issued one VALU instruction per 4 cycles, the rate these
wave64 integer ops sustain (VALU-issue-bound).

usage: tools/sq_summary.py <pmc dir> [<pmc dir> ...]
"""
import collections
import csv
import os
import sys


def kernel_key(name):
    for key in ("rs_bitslice_rec_k", "rs_bitslice_k", "rs_matmul_kernel"):
        if key in name:
            return name[name.index(key):].split("(")[0]
    return None


def summarise(d):
    rows = list(csv.DictReader(open(os.path.join(d, "sq", "run_counter_collection.csv"))))
    trace = list(csv.DictReader(open(os.path.join(d, "sq", "run_kernel_trace.csv"))))
    dur = collections.defaultdict(list)
    for t in trace:
        k = kernel_key(t["Kernel_Name"])
        if k:
            dur[k].append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = kernel_key(r["Kernel_Name"])
        if not k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = []
    for k, v in agg.items():
        n = len(disp[k])
        ms = sum(dur[k]) / len(dur[k]) if dur[k] else float("nan")
        waves = v["SQ_WAVES"] / n
        valu = v["SQ_INSTS_VALU"] / n
        wc = v["SQ_WAVE_CYCLES"]
        clock = valu * 4 / 1024 / (ms / 1e3) / 1e9 if ms == ms else float("nan")
        out.append((k, n, ms, valu / max(waves, 1), v["SQ_ACTIVE_INST_VALU"] / wc, v["SQ_WAIT_INST_ANY"] / wc,
                    v["SQ_WAIT_ANY"] / wc, clock))
    return out


if __name__ == "__main__":
    print("| run | kernel | dispatches | ms | VALU per wave | VALU-issuing / wave cycles | issue-stalled | waiting | VALU-bound clock (GHz) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for d in sys.argv[1:]:
        for k, n, ms, vpw, act, stall, wait, clk in summarise(d):
            print(f"| {os.path.basename(d.rstrip('/'))} | `{k}` | {n} | {ms:.2f} | {vpw:.0f} | {act:.2f} | {stall:.2f} | {wait:.2f} | {clk:.2f} |")
