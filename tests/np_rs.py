"""Independent numpy restatement of the infectious code (second checker).

Written differently from oracle/rs_oracle.c on purpose: log/exp arithmetic
over numpy arrays and a generic Gauss-Jordan inverse of the full Vandermonde
top block (instead of infectious's polynomial createInvertedVdm).  It follows
the same published algorithm: GF(2^8) poly 0x11D,
generator 2, systematic matrix V[k..n-1] . inv(V[0..k-1]) with V[r][c] =
x_r^c, x_0 = 0, x_r = 2^(r - 1 + point_offset) for r >= 1.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11D


def _tables():
    exp = np.zeros(512, dtype=np.int64)
    log = np.zeros(256, dtype=np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[:255]
    mul = np.zeros((256, 256), dtype=np.uint8)
    a = np.arange(1, 256)
    mul[1:, 1:] = exp[(log[a][:, None] + log[a][None, :]) % 255]
    return exp, log, mul


EXP, LOG, MUL = _tables()


def gmul(a, b):
    return MUL[a, b]


def ginv(a: int) -> int:
    return int(EXP[(255 - LOG[a]) % 255])


def matmul(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    A = np.asarray(A, dtype=np.uint8)
    B = np.asarray(B, dtype=np.uint8)
    out = np.zeros((A.shape[0], B.shape[1]), dtype=np.uint8)
    for i in range(A.shape[1]):
        out ^= MUL[A[:, i][:, None], B[i, :][None, :]]
    return out


def invert(M: np.ndarray):
    """Gauss-Jordan; returns None if singular."""
    k = M.shape[0]
    aug = np.concatenate([np.asarray(M, dtype=np.uint8), np.eye(k, dtype=np.uint8)], axis=1)
    for col in range(k):
        piv = next((r for r in range(col, k) if aug[r, col]), None)
        if piv is None:
            return None
        aug[[col, piv]] = aug[[piv, col]]
        aug[col] = MUL[ginv(int(aug[col, col])), aug[col]]
        for r in range(k):
            if r != col and aug[r, col]:
                aug[r] ^= MUL[aug[r, col], aug[col]]
    return aug[:, k:].copy()


def point(r: int, point_offset: int = 1) -> int:
    return 0 if r == 0 else int(EXP[(r - 1 + point_offset) % 255])


def vandermonde(n: int, k: int, point_offset: int = 1) -> np.ndarray:
    V = np.zeros((n, k), dtype=np.uint8)
    for r in range(n):
        x = point(r, point_offset)
        v = 1
        for c in range(k):
            V[r, c] = v
            v = int(MUL[v, x])
    return V


def fec_matrix(k: int, n: int, point_offset: int = 1) -> np.ndarray:
    V = vandermonde(n, k, point_offset)
    E = matmul(V, invert(V[:k]))
    return E


def encode(E: np.ndarray, k: int, data: bytes) -> np.ndarray:
    """Parity shares as an (m, S) array."""
    d = np.frombuffer(bytes(data), dtype=np.uint8).reshape(k, -1)
    m = E.shape[0] - k
    out = np.zeros((m, d.shape[1]), dtype=np.uint8)
    for t in range(m):
        for c in range(k):
            out[t] ^= MUL[E[k + t, c], d[c]]
    return out


def apply_rows(rows: np.ndarray, shards: np.ndarray) -> np.ndarray:
    out = np.zeros((rows.shape[0], shards.shape[1]), dtype=np.uint8)
    for t in range(rows.shape[0]):
        for c in range(rows.shape[1]):
            out[t] ^= MUL[rows[t, c], shards[c]]
    return out
