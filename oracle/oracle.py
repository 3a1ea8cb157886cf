"""ctypes loader for the CPU oracle (oracle/rs_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
(noise-erasurecode-plugin_amd/) never imports it.

Parity status: restatement of github.com/vivint/infectious (unpinned version,
absent from /root/reference); parity bytes are "parity unpinned" against
upstream -- see rs_oracle.h and DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_LIB = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i32, u8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint8
        L.orc_gf_mul.restype = u8
        L.orc_gf_mul.argtypes = [u8, u8]
        L.orc_gf_inv.restype = u8
        L.orc_gf_inv.argtypes = [u8]
        L.orc_gf_exp.restype = u8
        L.orc_gf_exp.argtypes = [i32]
        L.orc_gf_log.restype = i32
        L.orc_gf_log.argtypes = [u8]
        L.orc_fec_matrix.restype = i32
        L.orc_fec_matrix.argtypes = [i32, i32, i32, vp]
        L.orc_encode.restype = i32
        L.orc_encode.argtypes = [vp, i32, i32, vp, sz, vp]
        L.orc_decode.restype = i32
        L.orc_decode.argtypes = [vp, i32, i32, vp, vp, i32, sz, vp]
        L.orc_decode_correct.restype = i32
        L.orc_decode_correct.argtypes = [vp, i32, i32, vp, vp, i32, sz, vp]
        L.orc_bw_column.restype = i32
        L.orc_bw_column.argtypes = [vp, i32, i32, vp, vp, i32, vp]
        L.orc_invert.restype = i32
        L.orc_invert.argtypes = [vp, i32]
        L.orc_addmul.restype = None
        L.orc_addmul.argtypes = [vp, vp, u8, sz]
        L.orc_addmul_simd.restype = None
        L.orc_addmul_simd.argtypes = [vp, vp, u8, sz]
        L.orc_encode_batch.restype = i32
        L.orc_encode_batch.argtypes = [vp, i32, i32, vp, vp, sz, sz, i32, i32]
        L.orc_reconstruct_batch.restype = i32
        L.orc_reconstruct_batch.argtypes = [vp, i32, i32, vp, vp, sz, sz, vp, i32, i32]
        L.orc_matmul_stripe.restype = None
        L.orc_matmul_stripe.argtypes = [vp, i32, i32, vp, vp, sz, i32]
        L.orc_fill_splitmix.restype = None
        L.orc_fill_splitmix.argtypes = [vp, sz, ctypes.c_uint64]
        _LIB = L
    return _LIB


def _p(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def fec_matrix(k: int, n: int, point_offset: int = 1) -> np.ndarray:
    """infectious.NewFEC(k, n) encode matrix, shape (n, k)."""
    out = np.zeros((n, k), dtype=np.uint8) if 0 < k <= n <= 256 else np.zeros(1, np.uint8)
    rc = lib().orc_fec_matrix(k, n, point_offset, _p(out))
    if rc != 0:
        raise ValueError(f"orc_fec_matrix({k},{n}) -> {rc}")
    return out


def encode(enc: np.ndarray, k: int, n: int, data: bytes) -> bytes:
    """(*FEC).Encode parity shares k..n-1 concatenated."""
    src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    if len(src) % k:
        raise ValueError("input length must be a multiple of k")
    S = len(src) // k
    par = np.zeros((n - k) * S, dtype=np.uint8)
    rc = lib().orc_encode(_p(np.ascontiguousarray(enc)), k, n,
                          _p(src) if len(src) else None, len(src), _p(par) if len(par) else None)
    if rc != 0:
        raise ValueError(f"orc_encode -> {rc}")
    return par.tobytes()


def decode(enc: np.ndarray, k: int, n: int, shares: Sequence[Tuple[int, bytes]]) -> Tuple[int, bytes]:
    """(*FEC).Decode(nil, shares) -> (status, k*S bytes)."""
    cnt = len(shares)
    S = len(shares[0][1]) if cnt else 0
    nums = (ctypes.c_int * max(cnt, 1))(*[s[0] for s in shares])
    keep = [np.frombuffer(bytes(s[1]), dtype=np.uint8).copy() for s in shares]
    ptrs = (ctypes.c_void_p * max(cnt, 1))(*[_p(b) if len(b) else None for b in keep])
    dst = np.zeros(max(k * S, 1), dtype=np.uint8)
    rc = lib().orc_decode(_p(np.ascontiguousarray(enc)), k, n, ctypes.addressof(nums),
                          ctypes.addressof(ptrs), cnt, S, _p(dst))
    return rc, dst[:k * S].tobytes()


def decode_correct(enc: np.ndarray, k: int, n: int, shares: Sequence[Tuple[int, bytes]]) -> Tuple[int, bytes]:
    """(*FEC).Decode with Correct (Berlekamp-Welch) for more than k shares."""
    cnt = len(shares)
    S = len(shares[0][1]) if cnt else 0
    nums = (ctypes.c_int * max(cnt, 1))(*[s[0] for s in shares])
    keep = [np.frombuffer(bytes(s[1]), dtype=np.uint8).copy() for s in shares]
    ptrs = (ctypes.c_void_p * max(cnt, 1))(*[_p(b) if len(b) else None for b in keep])
    dst = np.zeros(max(k * S, 1), dtype=np.uint8)
    rc = lib().orc_decode_correct(_p(np.ascontiguousarray(enc)), k, n, ctypes.addressof(nums),
                                  ctypes.addressof(ptrs), cnt, S, _p(dst))
    return rc, dst[:k * S].tobytes()


def invert(a: np.ndarray) -> Tuple[int, np.ndarray]:
    m = np.ascontiguousarray(a, dtype=np.uint8).copy()
    rc = lib().orc_invert(_p(m), m.shape[0])
    return rc, m


def matmul_stripe(coef: np.ndarray, shards: List[np.ndarray], simd: bool = False) -> List[np.ndarray]:
    """out_t = sum_c coef[t, c] * shards[c] (Rebuild's inner loop)."""
    rows, k = coef.shape
    S = len(shards[0]) if shards else 0
    ins = [np.ascontiguousarray(s, dtype=np.uint8) for s in shards]
    outs = [np.zeros(S, dtype=np.uint8) for _ in range(rows)]
    inp = (ctypes.c_void_p * k)(*[_p(x) for x in ins])
    outp = (ctypes.c_void_p * max(rows, 1))(*[_p(x) for x in outs])
    lib().orc_matmul_stripe(_p(np.ascontiguousarray(coef, dtype=np.uint8)), rows, k,
                            ctypes.addressof(inp), ctypes.addressof(outp), S, int(simd))
    return outs


def encode_batch(enc: np.ndarray, k: int, n: int, data: np.ndarray, S: int, stripes: int,
                 simd: bool = True, threads: int = 1, out: np.ndarray = None) -> np.ndarray:
    """Parity of `stripes` stripes [stripes][k][S] -> [stripes][n-k][S], into
    `out` when given (a pre-touched buffer keeps page faults, which
    serialise threads, out of a timed loop)."""
    par = np.zeros(stripes * (n - k) * S, dtype=np.uint8) if out is None else out
    lib().orc_encode_batch(_p(np.ascontiguousarray(enc)), k, n, _p(data), _p(par), S, stripes,
                           int(simd), threads)
    return par


def reconstruct_batch(enc: np.ndarray, k: int, n: int, data: np.ndarray, parity: np.ndarray,
                      S: int, stripes: int, erased: np.ndarray, simd: bool = True,
                      threads: int = 1) -> int:
    """Regenerates every erased shard in place (Rebuild per stripe)."""
    er = np.ascontiguousarray(erased, dtype=np.uint8)
    return lib().orc_reconstruct_batch(_p(np.ascontiguousarray(enc)), k, n, _p(data), _p(parity),
                                       S, stripes, _p(er), int(simd), threads)


def splitmix_bytes(n: int, seed: int) -> np.ndarray:
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().orc_fill_splitmix(_p(out), n, seed & (2**64 - 1))
    return out[:n]


def gf_mul(a: int, b: int) -> int:
    return lib().orc_gf_mul(a, b)


def gf_exp(i: int) -> int:
    return lib().orc_gf_exp(i)
