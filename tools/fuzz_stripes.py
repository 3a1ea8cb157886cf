#!/usr/bin/env python3
"""Randomised GPU soak of the batched device API: random (k, n), shard
length, pitch, stripe count and erasure sets; encode_stripes checked against
the oracle on sampled stripes, then every stripe erased and reconstructed and
compared with the original bytes (device torch.equal).  Covers the kernel
variants (split-table K*/K0, bit-sliced RS(64,16) and RS(10,4)), the XCD
block order's tails and ragged shard lengths.  Prints one JSON line.

usage: tools/fuzz_stripes.py [--seconds 120] [--seed 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    codes = [(10, 14), (64, 80), (8, 14), (4, 6), (17, 49), (1, 3), (32, 40), (100, 120), (200, 256)]
    fecs = {}
    t0 = time.time()
    cases = fails = 0
    first = []
    last_note = t0
    while time.time() - t0 < a.seconds:
        if time.time() - last_note > 30:  # progress on stderr: a long run is seen to be alive
            last_note = time.time()
            print(f"fuzz_stripes: {cases} cases, {fails} failures, {last_note - t0:.0f} s", file=sys.stderr, flush=True)
        k, n = codes[int(rng.integers(0, len(codes)))]
        m = n - k
        # half the contexts keep small calls on the bit-sliced kernels
        # (RSMI_SMALL_SPLIT=0), half route them to the split table (default)
        small = "0" if rng.integers(0, 2) else "16"
        if (k, n, small) not in fecs:
            os.environ["RSMI_SMALL_SPLIT"] = small
            fecs[(k, n, small)] = rsmi.NewFEC(k, n)
            del os.environ["RSMI_SMALL_SPLIT"]
        f = fecs[(k, n, small)]
        S = int(rng.choice([1, 15, 16, 100, 4096, 8192 + 16, 65536, 70000, 1 << 20]))
        if k * S > (64 << 20):
            S = max(1, (64 << 20) // k)
        pitch = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
        stripes = int(rng.integers(1, 40)) if S >= 65536 else int(rng.integers(1, 130))
        data = torch.empty(stripes * k * pitch, dtype=torch.uint8, device="cuda")
        f.fill_splitmix(data.data_ptr(), data.numel(), int(rng.integers(0, 1 << 30)))
        parity = torch.zeros(stripes * m * pitch, dtype=torch.uint8, device="cuda")
        f.encode_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes)
        f.sync()
        ok = True
        E = oracle.fec_matrix(k, n)
        for s in rng.choice(stripes, size=min(2, stripes), replace=False):
            hd = data.view(stripes, k, pitch)[s, :, :S].cpu().numpy().tobytes()
            hp = parity.view(stripes, m, pitch)[s, :, :S].cpu().numpy().tobytes()
            ok &= hp == oracle.encode(E, k, n, hd)
        er = np.zeros((stripes, n), dtype=np.uint8)
        for s in range(stripes):
            er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
        d0, p0 = data.clone(), parity.clone()
        data.view(stripes, k, pitch)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xA5
        parity.view(stripes, m, pitch)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0x5A
        f.reconstruct_stripes(data.data_ptr(), k * pitch, parity.data_ptr(), m * pitch, pitch, S, stripes,
                              er.tobytes())
        f.sync()
        dv, pv = data.view(stripes, k, pitch), parity.view(stripes, m, pitch)
        ok &= torch.equal(dv[:, :, :S], d0.view(stripes, k, pitch)[:, :, :S])
        ok &= torch.equal(pv[:, :, :S], p0.view(stripes, m, pitch)[:, :, :S])
        cases += 1
        if not ok:
            fails += 1
            if len(first) < 5:
                first.append({"k": k, "n": n, "S": S, "pitch": pitch, "stripes": stripes})
        del data, parity, d0, p0
        if cases % 50 == 0:
            print(f"{cases} cases, {fails} failures, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    print(json.dumps({"seconds": round(time.time() - t0, 1), "cases": cases, "failures": fails,
                      "first_failures": first, "codes": [list(c) for c in codes]}))


if __name__ == "__main__":
    main()
