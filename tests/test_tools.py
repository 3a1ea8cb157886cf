"""CPU checks of the measurement tooling behind the committed profiles:
tools/prof_line.py's per-role classification and HBM-traffic arithmetic
(the gfx950 correction FETCH_SIZE x 2 + WRITE_SIZE, in KiB units) on a
synthetic rocprofv3 layout, and that tools/fuzz_host_api.py imports without a
GPU (its engine imports happen inside run())."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")

MM = "void rsmi::(anonymous namespace)::rs_matmul_kernel<10, 4, 256, true>(rsmi::MatArgs)"
REC = "void rsmi::(anonymous namespace)::rs_bitslice_rec_k64_m16<false>(rsmi::BitsliceRecArgs)"
ENC = "rsmi::(anonymous namespace)::rs_bitslice_k64_m16(rsmi::BitsliceArgs)"


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=header)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _layout(tmp):
    """Headline encode/reconstruct alternating at the big grid, two config-1
    launches, one config-5 encode and reconstruct; FETCH/WRITE passes (KiB)."""
    launches = [(MM, 1000, 10.0), (MM, 1000, 9.0), (MM, 1000, 10.0), (MM, 1000, 9.0),
                (MM, 50, 0.02), (MM, 50, 0.02), (ENC, 800, 14.0), (REC, 800, 15.0)]
    kt = ["Kernel_Name", "Grid_Size_X", "Start_Timestamp", "End_Timestamp"]
    rows, t = [], 0
    for name, grid, ms in launches:
        rows.append({"Kernel_Name": name, "Grid_Size_X": grid, "Start_Timestamp": t,
                     "End_Timestamp": t + int(ms * 1e6)})
        t += int(ms * 1e6) + 1000
    _write(os.path.join(tmp, "trace", "run_kernel_trace.csv"), kt, rows)
    # FETCH_SIZE / WRITE_SIZE in KiB: encode 10 + 4 units, reconstruct 10 + 2.5
    fetch = {1000: [5e6, 5e6, 5e6, 5e6], 50: [1e2, 1e2], 800: [4e7, 3.2e7]}
    write = {1000: [4e6, 2.5e6, 4e6, 2.5e6], 50: [1e2, 1e2], 800: [5e6, 6e6]}
    ct = ["Kernel_Name", "Grid_Size_X", "Counter_Name", "Counter_Value"]
    for counter, vals, sub in (("FETCH_SIZE", fetch, "fetch"), ("WRITE_SIZE", write, "write")):
        seen = {g: 0 for g in vals}
        out = []
        for name, grid, _ in launches:
            v = vals[grid][seen[grid]]
            seen[grid] += 1
            out.append({"Kernel_Name": name, "Grid_Size_X": grid, "Counter_Name": counter, "Counter_Value": v})
        _write(os.path.join(tmp, sub, "run_counter_collection.csv"), ct, out)


def test_prof_line_roles_and_traffic(tmp_path):
    _layout(str(tmp_path))
    out = tmp_path / "summary.md"
    traffic = tmp_path / "traffic.json"
    bench = tmp_path / "line.json"
    bench.write_text(json.dumps({
        "value": 1.0, "config": {"stripes_per_gpu": 1, "n": 14, "k": 10, "shard_bytes": 1 << 20},
        "breakdown": {"encode_ms": 10.0, "reconstruct_ms": 9.0}, "roofline": {"frac": 0.5}}))
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "prof_line.py"), str(tmp_path), str(out),
                        "--bench-json", str(bench), "--traffic-json", str(traffic)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    md = out.read_text()
    rows = {line.split("|")[1].strip(): line for line in md.splitlines() if line.startswith("| ")}
    assert "2 | 10.000" in rows["headline encode"] and "2 | 9.000" in rows["headline reconstruct"]
    assert "| 2 |" in rows["config1 + device-set launches (host-API messages, members)"]
    assert "config5 encode" in rows and "config5 reconstruct" in rows
    # encode traffic per launch: (5e6 x 2 + 4e6) KiB = 14.336 GB, keyed by role and
    # workload, naming the kernel and the profile it came from
    tj = json.loads(traffic.read_text())["entries"]
    enc = tj["encode_k10_n14_S1048576_stripes1"]
    assert enc["traffic_GB"] == 14.336 and enc["profile"] == str(tmp_path) and "rs_matmul_kernel" in enc["kernel"]
    assert enc["launches"] == 2 and enc["trace_ms"] == 10.0
    assert tj["reconstruct_k10_n14_S1048576_stripes1"]["traffic_GB"] == (5e6 * 2 + 2.5e6) * 1024 / 1e9
    assert set(tj) >= {"config5_encode_k64_n80_S65536_stripes16384", "config5_reconstruct_k64_n80_S65536_stripes16384"}
    assert "| 14.336 |" in rows["headline encode"]


def test_fuzz_host_api_imports_without_gpu():
    r = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import fuzz_host_api as f; "
                        "assert callable(f.run) and len(f.CODES) >= 5" % TOOLS],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
