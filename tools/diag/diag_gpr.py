"""Diagnose the bit-sliced reconstruct: which stripes / outputs / byte
ranges differ from the originals (k=64, n=80)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "noise-erasurecode-plugin_amd"))
os.environ["RSMI_BITSLICE"] = "1"
os.environ["RSMI_BITSLICE_REC_MIN_E"] = "1"
import rsmi  # noqa: E402


def run(k, n, S, er, seed=5):
    m = n - k
    f = rsmi.NewFEC(k, n)
    stripes = len(er)
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), seed)
    parity = torch.zeros(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    dv, pv = data.view(stripes, k, S), parity.view(stripes, m, S)
    dv[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0xA5
    pv[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0x5A
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
    f.sync()
    full = torch.cat([dv, pv], dim=1).cpu().numpy()
    ref = torch.cat([d0.view(stripes, k, S), p0.view(stripes, m, S)], dim=1).cpu().numpy()
    bad = 0
    for s in range(stripes):
        ids = np.nonzero(er[s])[0]
        wrong = [i for i in range(n) if not np.array_equal(full[s, i], ref[s, i])]
        if wrong:
            bad += 1
            if bad <= 12:
                i = wrong[0]
                diff = np.nonzero(full[s, i] != ref[s, i])[0]
                win = sorted(set((diff // 2048).tolist()))
                print(f"  stripe {s}: e={len(ids)} erased={ids.tolist()} wrong={wrong} first: {len(diff)} bytes, 2KiB windows {win[:12]}")
    print(f"k={k} n={n} S={S} stripes={stripes}: {bad} bad stripes")
    f.close()


rng = np.random.default_rng(1)
k, n = 64, 80
m = n - k


def pats(cnt, emin, emax):
    er = np.zeros((cnt, n), dtype=np.uint8)
    for s in range(cnt):
        e = int(rng.integers(emin, emax + 1))
        er[s, rng.choice(n, size=e, replace=False)] = 1
    return er


CASES = ((1, 1, 1), (1, 5, 5), (1, 16, 16), (4, 1, 16), (40, 1, 4), (40, 5, 16), (200, 1, 16))
if len(sys.argv) > 1 and sys.argv[1] == "quick":
    CASES = ((200, 1, 16), (400, 1, 4), (400, 1, 16))
for S in ((65536,) if len(sys.argv) > 1 else (8208, 65536)):
    for cnt, emin, emax in CASES:
        print(f"== S={S} stripes={cnt} e={emin}..{emax}")
        run(k, n, S, pats(cnt, emin, emax))
