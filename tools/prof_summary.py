#!/usr/bin/env python3
"""Summarise a rocprofv3 profile of bench.py (tools/profile_*.sh layout).

Reads <dir>/trace/run_kernel_trace.csv (+ run_kernel_stats.csv) and the
separate PMC passes <dir>/fetch, <dir>/write (FETCH_SIZE / WRITE_SIZE, KiB),
splits the rs_matmul launches by role (bench.py alternates encode and
reconstruct launches in --mode both), applies the gfx950 correction from
/opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE reads exactly half the
bytes of a wide coalesced streaming read: x2; WRITE_SIZE exact for 16-B
stores) and writes a markdown summary plus profiles/traffic.json, which
bench.py reports as roofline.traffic.

usage: tools/prof_summary.py <profile dir> <out.md> [--stripes N --k K --n N --shard S]
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


def matmul_only(rs):
    return [r for r in rs if "rs_matmul_kernel" in r["Kernel_Name"]]


def coding_kernels(rs):
    """Launches of the engine's coding kernels (split-table and bit-sliced)."""
    return [r for r in rs if "rs_matmul_kernel" in r["Kernel_Name"] or "rs_bitslice" in r["Kernel_Name"]]


def short_name(name):
    for key in ("rs_bitslice_rec_k", "rs_bitslice_k"):
        if key in name:
            return name[name.index(key):].split("(")[0].split("E")[0]
    if "rs_matmul_kernel<" in name:
        return name[name.index("rs_matmul_kernel<"):].split(">")[0] + ">"
    return name[:60]


def kernel_traffic_gb(a, key):
    """Mean FETCH_SIZE x2 + WRITE_SIZE (GB) per launch of kernels whose name
    contains key (and not "_rec" unless asked), or None."""
    vals = {}
    for cnt, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        v = [float(r["Counter_Value"]) for r in rows(os.path.join(a.dir, sub, "run_counter_collection.csv"))
             if r["Counter_Name"] == cnt and key in r["Kernel_Name"]
             and ("_rec" in key or "_rec" not in r["Kernel_Name"])]
        if not v:
            return None
        vals[cnt] = statistics.mean(v)
    return (vals["FETCH_SIZE"] * 2 + vals["WRITE_SIZE"]) * 1024 / 1e9


def by_name_section(a):
    """Per coding kernel: launches, average duration, HBM bytes per launch."""
    tr = coding_kernels(rows(os.path.join(a.dir, "trace", "run_kernel_trace.csv")))
    if not tr:
        return []
    out = ["## Per coding kernel (trace + separate FETCH_SIZE / WRITE_SIZE passes)", "",
           "| kernel | launches | avg ms | read GB/launch (FETCH x2) | write GB/launch | traffic GB/launch | HBM GB/s |",
           "|---|---|---|---|---|---|---|"]
    pmc = {}
    for cnt, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        for r in coding_kernels(rows(os.path.join(a.dir, sub, "run_counter_collection.csv"))):
            if r["Counter_Name"] == cnt:
                pmc.setdefault((short_name(r["Kernel_Name"]), cnt), []).append(float(r["Counter_Value"]))
    names = []
    for r in tr:
        nm = short_name(r["Kernel_Name"])
        if nm not in names:
            names.append(nm)
    for nm in names:
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr
             if short_name(r["Kernel_Name"]) == nm]
        f = pmc.get((nm, "FETCH_SIZE"), [])
        w = pmc.get((nm, "WRITE_SIZE"), [])
        rd = statistics.mean(f) * 1024 * 2 / 1e9 if f else float("nan")
        wr = statistics.mean(w) * 1024 / 1e9 if w else float("nan")
        ms = statistics.mean(d)
        out.append(f"| `{nm}` | {len(d)} | {ms:.3f} | {rd:.2f} | {wr:.2f} | {rd + wr:.2f} | "
                   f"{(rd + wr) / (ms / 1e3):.0f} |")
    out.append("")
    return out


def split_roles(rs, mode):
    """bench --mode both: launches alternate encode, reconstruct."""
    if mode == "both":
        return {"encode": rs[0::2], "reconstruct": rs[1::2]}
    return {mode: rs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("out")
    ap.add_argument("--mode", default="both")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--shard", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=6553)
    ap.add_argument("--bench-log", default=None)
    ap.add_argument("--traffic-json", default=None)
    a = ap.parse_args()
    k, n, S, st = a.k, a.n, a.shard, a.stripes
    m = n - k
    alg_enc = st * (k + m) * S

    all_tr = rows(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))
    # With generated bit-sliced kernels in the run, encode and reconstruct are
    # told apart by kernel name (per-kernel section below), not launch order.
    has_bs = any("rs_bitslice" in r["Kernel_Name"] for r in all_tr)
    tr = matmul_only(all_tr)
    roles = {} if has_bs else split_roles(tr, a.mode)
    lines = [f"# rocprofv3 summary: {os.path.basename(os.path.normpath(a.dir))}", ""]
    lines.append(f"Workload: RS({k},{n}), {st} stripes x {k} x {S} B shards, bench.py --mode {a.mode}.")
    lines.append("")
    lines.append("## Kernel trace (rocprofv3 --kernel-trace --stats)")
    lines.append("")
    stats = rows(os.path.join(a.dir, "trace", "run_kernel_stats.csv"))
    lines.append("| kernel | calls | avg ms | min ms | max ms | % time |")
    lines.append("|---|---|---|---|---|---|")
    for r in stats:
        lines.append(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                     f"{float(r['MinNs'])/1e6:.3f} | {float(r['MaxNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")
    lines.append("")
    bs_traffic = {}
    if has_bs:
        lines += by_name_section(a)
        enc = [r for r in all_tr if "rs_bitslice_k" in r["Kernel_Name"]]
        enc_traffic = kernel_traffic_gb(a, "rs_bitslice_k")
        if enc_traffic is not None:
            bs_traffic[f"encode_k{k}_n{n}_S{S}_stripes{st}"] = round(enc_traffic, 3)
        if enc:
            ms = statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in enc)
            ach = alg_enc / (ms / 1e3) / 1e9
            lines.append(f"Encode (`{short_name(enc[0]['Kernel_Name'])}`): algorithmic {alg_enc/1e9:.2f} GB per "
                         f"launch / {ms:.3f} ms = **{ach:.0f} GB/s = {ach/8000:.1%} of 8 TB/s**.")
        rec = [r for r in all_tr if "rs_bitslice_rec" in r["Kernel_Name"]]
        if rec:
            lines.append("")
            split = any("rs_matmul_kernel" in r["Kernel_Name"] for r in all_tr)
            variants = sorted({short_name(r["Kernel_Name"]) for r in rec})
            what = ("the split-table launch (stripes with e below RSMI_BITSLICE_REC_MIN_E) plus the syndrome launches"
                    if split else (f"the syndrome launches ({', '.join(f'`{v}`' for v in variants)}: each stripe in "
                                   "the smallest row-subset kernel covering its pattern)" if len(variants) > 1 else
                                   f"the syndrome kernel `{variants[0]}`, every stripe"))
            # steps = encode launches (mode both) or, in reconstruct mode, launches of the full kernel
            steps = len(enc) if a.mode == "both" and enc else max(1, len([r for r in rec if "_t" not in short_name(r["Kernel_Name"])]))
            rms = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rec) / steps
            alg_rec = st * (k + (m + 1) / 2) * S
            rec_pmc = []
            for cnt, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
                v = [float(r["Counter_Value"]) for r in rows(os.path.join(a.dir, sub, "run_counter_collection.csv"))
                     if r["Counter_Name"] == cnt and "rs_bitslice_rec" in r["Kernel_Name"]]
                rec_pmc.append(v)
            tail = ""
            if rec_pmc[0] and rec_pmc[1]:
                # the PMC runs have their own step counts: normalise by their full-kernel launches
                psteps = max(1, len([1 for r in rows(os.path.join(a.dir, "fetch", "run_counter_collection.csv"))
                                     if r["Counter_Name"] == "FETCH_SIZE" and "rs_bitslice_rec" in r["Kernel_Name"]
                                     and "_t" not in short_name(r["Kernel_Name"])]))
                tr_gb = (sum(rec_pmc[0]) * 2 + sum(rec_pmc[1])) * 1024 / 1e9 / psteps
                tail = f" HBM traffic {tr_gb:.2f} GB per step (FETCH x2 + WRITE over its launches)."
            lines.append(f"Reconstruct per step = {what}; expected algorithmic bytes {alg_rec / 1e9:.2f} GB "
                         f"(uniform 1..m erasures)" + ("." if split else
                         f" / {rms:.3f} ms of kernel time per step = **{alg_rec / (rms / 1e3) / 1e9:.0f} GB/s**.") + tail)
    rl = ["Per role (launch order alternates encode / reconstruct):"]
    rl.append("")
    rl.append("| role | launches | avg ms | grid (threads) | workgroup |")
    rl.append("|---|---|---|---|---|")
    avg = {}
    for role, rs in roles.items():
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rs]
        if not d:
            continue
        avg[role] = statistics.mean(d)
        rl.append(f"| {role} | {len(d)} | {avg[role]:.3f} | {rs[0].get('Grid_Size_X', '?')} | "
                     f"{rs[0].get('Workgroup_Size_X', '?')} |")
    rl.append("")

    traffic = {}
    pmc = {}
    for cnt, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        rs = [r for r in matmul_only(rows(os.path.join(a.dir, sub, "run_counter_collection.csv")))
              if r["Counter_Name"] == cnt]
        pmc[cnt] = split_roles(rs, a.mode)
    rl.append("## HBM traffic (separate --pmc passes, per launch)")
    rl.append("")
    rl.append("FETCH_SIZE x 1024 x 2 (gfx950: FETCH_SIZE counts half of a wide streaming read), "
                 "WRITE_SIZE x 1024 (exact for 16-B stores).")
    rl.append("")
    rl.append("Reconstruct algorithmic bytes are the expectation k + (m+1)/2 shards per stripe "
                 "(uniform 1..m erasures); the profiled launches drew their own random sets.")
    rl.append("")
    rl.append("| role | FETCH_SIZE KiB | read GB (corrected) | WRITE_SIZE KiB | write GB | traffic GB | algorithmic GB | traffic / algorithmic |")
    rl.append("|---|---|---|---|---|---|---|---|")
    for role in roles:
        f = [float(r["Counter_Value"]) for r in pmc["FETCH_SIZE"].get(role, [])]
        w = [float(r["Counter_Value"]) for r in pmc["WRITE_SIZE"].get(role, [])]
        if not f or not w:
            continue
        rd = statistics.mean(f) * 1024 * 2
        wr = statistics.mean(w) * 1024
        if role == "encode":
            alg = alg_enc
        else:
            # bench.py draws 1..m erasures uniformly: E[e] = (m + 1) / 2
            alg = st * (k + (n - k + 1) / 2) * S
        t = rd + wr
        traffic[f"{role}_k{k}_n{n}_S{S}_stripes{st}"] = round(t / 1e9, 3)
        rl.append(f"| {role} | {statistics.mean(f):.0f} | {rd/1e9:.2f} | {statistics.mean(w):.0f} | "
                     f"{wr/1e9:.2f} | {t/1e9:.2f} | {alg/1e9 if alg else float('nan'):.2f} | "
                     f"{(t/alg) if alg else float('nan'):.3f} |")
    rl.append("")
    if not has_bs:
        lines += rl
    if "encode" in avg:
        ach = alg_enc / (avg["encode"] / 1e3) / 1e9
        lines.append(f"Encode: algorithmic {alg_enc/1e9:.2f} GB per launch / {avg['encode']:.3f} ms = "
                     f"**{ach:.0f} GB/s = {ach/8000:.1%} of 8 TB/s**.")
    if not has_bs:
        lines += by_name_section(a)
    if a.bench_log and os.path.exists(a.bench_log):
        for line in open(a.bench_log):
            if line.startswith("{"):
                b = json.loads(line)
                lines.append("")
                lines.append(f"bench.py line of the profiled run: value {b['value']} GB/s, encode "
                             f"{b['breakdown']['encode_ms']} ms (HIP events), reconstruct "
                             f"{b['breakdown']['reconstruct_ms']} ms.")
    with open(a.out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    traffic.update(bs_traffic)
    if a.traffic_json:
        old = {}
        if os.path.exists(a.traffic_json):
            old = json.load(open(a.traffic_json))
        old.update({key: v for key, v in traffic.items()})
        old["_note"] = ("HBM GB per launch from rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                        "(tools/prof_summary.py)")
        json.dump(old, open(a.traffic_json, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
