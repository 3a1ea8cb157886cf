"""Generates tests/golden/rs_golden.json from the C oracle, cross-checked by
the independent numpy restatement (tests/np_rs.py).  Run from the repo root:
    python tests/golden/make_golden.py
The reference holds no RS known-answer vectors, so these are
"self-derived, not infectious-produced": they pin the oracle against drift and
the GPU path against the oracle.  Inputs are splitmix64 byte streams
(oracle.splitmix_bytes(len, seed)), so only (len, seed) is stored.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import np_rs  # noqa: E402
from oracle import oracle  # noqa: E402

CONFIGS = [(1, 1), (1, 3), (4, 6), (10, 14), (8, 14), (3, 5), (17, 49), (64, 80)]
SIZES = [1, 16, 4099]


def main():
    out = {"note": "self-derived by oracle/rs_oracle.c, cross-checked by tests/np_rs.py; "
                   "not infectious-produced (parity unpinned upstream)",
           "gf_exp": [oracle.gf_exp(i) for i in range(255)],
           "matrices": {}, "encodings": []}
    for k, n in CONFIGS:
        E = oracle.fec_matrix(k, n)
        assert (E == np_rs.fec_matrix(k, n)).all()
        out["matrices"][f"{k},{n}"] = E.tobytes().hex()
        for S in SIZES:
            seed = 1000 * k + n + S
            data = oracle.splitmix_bytes(k * S, seed).tobytes()
            par = oracle.encode(E, k, n, data)
            assert par == np_rs.encode(E, k, data).tobytes()
            rec = {"k": k, "n": n, "S": S, "seed": seed,
                   "parity_sha256": hashlib.sha256(par).hexdigest()}
            if len(par) <= 256:
                rec["parity_hex"] = par.hex()
            out["encodings"].append(rec)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rs_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
