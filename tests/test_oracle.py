"""CPU: pin the oracle (oracle/rs_oracle.c) before trusting it.

Pinned by: the standard GF(2^8)/0x11D exp sequence (known answer), the
independent numpy restatement (tests/np_rs.py), the committed golden vectors
(tests/golden/rs_golden.json), and size-independent properties of the
reference's call pattern (main.go:243-267 encode, main.go:72-79 decode):
systematic data shares, every <=m erasure pattern reconstructs the input,
infectious's error conditions.
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

import np_rs
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "rs_golden.json")

# 2^i in GF(2^8) with x^8+x^4+x^3+x^2+1: the textbook sequence.
KNOWN_EXP = [1, 2, 4, 8, 16, 32, 64, 128, 29, 58, 116, 232, 205, 135, 19, 38, 76, 152, 45,
             90, 180, 117, 234, 201, 143, 3, 6, 12, 24, 48, 96, 192, 157, 39, 78]


def test_gf_known_answers():
    assert [oracle.gf_exp(i) for i in range(len(KNOWN_EXP))] == KNOWN_EXP
    assert oracle.gf_exp(255) == 1
    assert oracle.gf_mul(2, 0x80) == 0x1D
    for a in range(1, 256):
        assert oracle.gf_mul(a, oracle.lib().orc_gf_inv(a)) == 1
    # mul table agrees with numpy tables everywhere
    A = np.arange(256)
    got = np.array([[oracle.gf_mul(a, b) for b in range(0, 256, 7)] for a in range(256)])
    assert (got == np_rs.MUL[A][:, ::7]).all()


@pytest.mark.parametrize("k,n", [(1, 1), (1, 2), (2, 3), (4, 6), (8, 14), (10, 14), (16, 20),
                                 (32, 48), (64, 80), (100, 200), (128, 256), (255, 256)])
@pytest.mark.parametrize("off", [0, 1])
def test_matrix_matches_numpy(k, n, off):
    E = oracle.fec_matrix(k, n, off)
    assert (E[:k] == np.eye(k, dtype=np.uint8)).all()
    assert (E == np_rs.fec_matrix(k, n, off)).all()


@pytest.mark.parametrize("k,n", [(4, 6), (10, 14), (8, 14), (64, 80), (200, 256)])
def test_point_offset_is_immaterial(k, n):
    # SURVEY.md §8c flagged the evaluation points {0, 2^1..} (infectious) vs
    # {0, 2^0..} (zfec) as the one recall-dependent choice.  Scaling every
    # non-zero point by 2 maps V to V.D (D = diag(2^c)), and the systematic
    # matrix V_b.D.(V_t.D)^-1 = V_b.V_t^-1 is unchanged: both give the same
    # parity bytes.
    assert (oracle.fec_matrix(k, n, 1) == oracle.fec_matrix(k, n, 0)).all()


def test_newfec_errors():
    for k, n in [(0, 1), (2, 1), (1, 257), (257, 257), (-1, 4)]:
        with pytest.raises(ValueError):
            oracle.fec_matrix(k, n)


def test_golden_vectors():
    with open(GOLDEN) as f:
        g = json.load(f)
    assert g["gf_exp"][:len(KNOWN_EXP)] == KNOWN_EXP
    for key, hexm in g["matrices"].items():
        k, n = map(int, key.split(","))
        assert oracle.fec_matrix(k, n).tobytes().hex() == hexm
    for rec in g["encodings"]:
        k, n, S = rec["k"], rec["n"], rec["S"]
        E = oracle.fec_matrix(k, n)
        data = oracle.splitmix_bytes(k * S, rec["seed"]).tobytes()
        par = oracle.encode(E, k, n, data)
        assert hashlib.sha256(par).hexdigest() == rec["parity_sha256"]
        if "parity_hex" in rec:
            assert par.hex() == rec["parity_hex"]


def test_encode_length_must_be_multiple():
    E = oracle.fec_matrix(4, 6)
    with pytest.raises(ValueError):
        oracle.encode(E, 4, 6, b"abcde")
    assert oracle.encode(E, 4, 6, b"") == b""


def test_all_erasure_patterns_rs10_4():
    k, n, S = 10, 14, 24
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, 99).tobytes()
    par = oracle.encode(E, k, n, data)
    shards = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
    count = 0
    for e in range(0, n - k + 1):
        for lost in itertools.combinations(range(n), e):
            keep = [i for i in range(n) if i not in lost]
            # the plugin hands Decode exactly k shares (main.go:65); take the
            # last k survivors in a shuffled order (Decode sorts them).
            sel = keep[-k:][::-1]
            rc, out = oracle.decode(E, k, n, [(i, shards[i]) for i in sel])
            assert rc == 0 and out == data, lost
            count += 1
    assert count == 1 + 14 + 91 + 364 + 1001


def test_decode_with_extra_shares_and_errors():
    k, n, S = 4, 6, 8
    E = oracle.fec_matrix(k, n)
    data = bytes(range(k * S))
    par = oracle.encode(E, k, n, data)
    sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
    rc, out = oracle.decode(E, k, n, [(i, sh[i]) for i in range(n)])  # > k shares
    assert rc == 0 and out == data
    assert oracle.decode(E, k, n, [(i, sh[i]) for i in range(3)])[0] == -3   # NotEnoughShares
    assert oracle.decode(E, k, n, [(0, sh[0]), (1, sh[1]), (2, sh[2]), (9, sh[3])])[0] == -4
    assert oracle.decode(E, k, n, [(0, sh[0]), (0, sh[0]), (1, sh[1]), (2, sh[2])])[0] != 0


def test_simd_addmul_matches_scalar():
    rng = np.random.default_rng(5)
    for c in [0, 1, 2, 0x1D, 0x80, 0xFF, 77]:
        x = rng.integers(0, 256, 1000, dtype=np.uint8)
        z1 = rng.integers(0, 256, 1000, dtype=np.uint8)
        z2 = z1.copy()
        oracle.lib().orc_addmul(z1.ctypes.data, x.ctypes.data, c, 1000)
        oracle.lib().orc_addmul_simd(z2.ctypes.data, x.ctypes.data, c, 1000)
        assert (z1 == z2).all()
        assert (z1 == (z2 if c else z1)).all()


def test_batch_encode_matches_single():
    k, n, S, stripes = 10, 14, 1000, 5
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(stripes * k * S, 3)
    for simd, thr in [(False, 1), (True, 1), (True, 3)]:
        par = oracle.encode_batch(E, k, n, data, S, stripes, simd=simd, threads=thr)
        for s in range(stripes):
            ref = oracle.encode(E, k, n, data[s * k * S:(s + 1) * k * S].tobytes())
            assert par[s * (n - k) * S:(s + 1) * (n - k) * S].tobytes() == ref


def test_oracle_berlekamp_welch():
    k, n, S = 10, 14, 64
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, 17).tobytes()
    par = oracle.encode(E, k, n, data)
    sh = [bytearray(data[i * S:(i + 1) * S]) for i in range(k)] + \
         [bytearray(par[i * S:(i + 1) * S]) for i in range(n - k)]
    sh[4] = bytearray(b"\xAA" * S)     # whole data share wrong
    sh[13][5] ^= 0x11                  # one parity byte wrong
    rc, out = oracle.decode_correct(E, k, n, [(i, bytes(sh[i])) for i in range(n)][::-1])
    assert rc == 0 and out == data
    sh[9] = bytearray(S)               # third bad share: beyond floor(4/2)
    rc, _ = oracle.decode_correct(E, k, n, [(i, bytes(sh[i])) for i in range(n)])
    assert rc == -7
