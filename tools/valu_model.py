#!/usr/bin/env python3
"""VALU per wave of the bit-sliced syndrome reconstruct (rs_bitslice_rec_k64_m16,
gen_bitslice.cpp emit_reconstruct), by component, for a bench workload.

Counts the per-lane VALU instructions the generated code executes for each
stripe's pattern -- a wave runs one stripe's 2 KiB window per shard, every
lane 32 bytes -- from the same rules the generator emits:

  transpose   48 per present data input (12 delta swaps x 4), 48 per output
              leaving the planes (Rebuild parity survivors' rows, erased
              parity q rows)
  combos      22 per present data input (the 16 XOR combinations of planes
              0-3 and 4-7, bs_combos x 2)
  network     one XOR / XOR3 per (output plane, present data input) whose
              coefficient image is not empty, for every parity row in a
              guarded group of 2 (kRowGroup) that the pattern uses
  survivor    8 XORs per Rebuild parity survivor (its bytes into the row)
  solve       per (syndrome, group of R = 4 outputs): the syndrome's bit
              fields (8 words x 5) and 4 outputs x 8 words x (3 v_perm +
              2 XOR); erased parity outputs add their q row (8 XORs)
  fixed       prologue, split-table build, address and store VALU: the
              residual against the measured SQ_INSTS_VALU / SQ_WAVES
              (--measured), else omitted

usage: tools/valu_model.py [--emin 1] [--emax 16] [--stripes 4096] [--measured V]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

K, N = 64, 80
M = N - K
ROW_GROUP = 2
R = 4


def network_ops(E):
    """ops[j][t]: XOR / XOR3 instructions of data input j into parity row t."""
    from oracle import oracle
    ops = np.zeros((K, M), dtype=np.int64)
    for j in range(K):
        for t in range(M):
            c = int(E[K + t, j])
            col = [oracle.gf_mul(c, 1 << p) for p in range(8)]
            ops[j, t] = sum(1 for q in range(8) if any((col[p] >> q) & 1 for p in range(8)))
    return ops


def stripe_model(er, ops):
    """Components (dict) of one stripe's VALU per lane for erasure flags er[n]."""
    erased = np.flatnonzero(er)
    data_er = [i for i in erased if i < K]
    d = len(data_er)
    present = [j for j in range(K) if not er[j]]
    # Rebuild's parity survivors: the d highest-numbered present parity rows
    surv = [t for t in range(M - 1, -1, -1) if not er[K + t]][:d]
    qrows = [i - K for i in erased if i >= K]
    rows = set(surv) | set(qrows)
    groups = {t // ROW_GROUP for t in rows}
    run_rows = [t for t in range(M) if t // ROW_GROUP in groups]
    e = len(erased)
    ngroups = (e + R - 1) // R
    return {
        "transpose": 48 * len(present) + 48 * (len(surv) + len(qrows)),
        "combos": 22 * len(present),
        "network": int(sum(ops[j, t] for j in present for t in run_rows)),
        "survivor": 8 * len(surv),
        "solve": ngroups * len(surv) * (8 * 5 + R * 8 * 5) + 8 * len(qrows),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--emin", type=int, default=1)
    ap.add_argument("--emax", type=int, default=16)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--measured", type=float, default=None, help="SQ_INSTS_VALU / SQ_WAVES of the same workload")
    args = ap.parse_args()
    from oracle import oracle
    from bench import erasure_sets
    E = oracle.fec_matrix(K, N)
    ops = network_ops(E)
    rng = np.random.default_rng(0xE4A5)
    er = erasure_sets(rng, 1, args.stripes, N, args.emin, args.emax)[0]
    tot = {}
    for s in range(args.stripes):
        for key, v in stripe_model(er[s], ops).items():
            tot[key] = tot.get(key, 0) + v
    per_wave = {key: v / args.stripes for key, v in tot.items()}
    model = sum(per_wave.values())
    if args.measured is not None:
        per_wave["fixed (residual)"] = args.measured - model
    total = sum(per_wave.values())
    print(f"| component | VALU per wave | share |")
    print(f"|---|---|---|")
    for key, v in per_wave.items():
        print(f"| {key} | {v:,.0f} | {v / total:.1%} |")
    print(f"| total | {total:,.0f} | |")


if __name__ == "__main__":
    main()
