#!/usr/bin/env python3
"""Randomised soak of the host-buffer C ABI (rs_encode / rs_decode, the cgo
calls replacing infectious Encode / Decode at main.go:262 / :77) against the
oracle: random (k, n), shard lengths from 1 byte to past the one-shot staging
threshold (aligned and ragged), k to n shares in random order, sometimes with
one corrupted share (Correct / Berlekamp-Welch), survivors in pageable
memory, in an engine-pinned rs_arena (read in place) or mixed, dst pageable
or engine-pinned.  Every fourth case also runs a batch of 1-40 messages of
that shape through rs_encode_batch and rs_decode_batch (own shares, drops,
corruptions and survivor placement per message).  Aliasing (infectious lets
Decode's shares alias dst; round 6): some single decodes put every share and
dst in one buffer (rows in a random order, dst at a random row and byte
shift, pinned or pageable), and some batches put each message's shares in a
block that its own or the next message's dst covers.  Every parity and every
decoded message is compared with the oracle's.  Prints one JSON line.

usage: tools/fuzz_host_api.py [--seconds 120 | --cases N] [--seed 1]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402

CODES = [(10, 14), (64, 80), (8, 14), (4, 6), (17, 49), (1, 3), (32, 40), (100, 120), (200, 256), (2, 4)]


def batch_case(rng, lib, f, E, k, n, S, stats, oracle, rsmi):
    """rs_encode_batch then rs_decode_batch over B messages of k*S bytes."""
    m = n - k
    P = ctypes.c_void_p
    B = int(rng.integers(1, 41))
    B = max(1, min(B, (24 << 20) // max(1, k * S)))
    datas = [oracle.splitmix_bytes(k * S, int(rng.integers(0, 2**32))) for _ in range(B)]
    pars = [np.zeros(m * S, dtype=np.uint8) for _ in range(B)]
    ins = (ctypes.c_void_p * B)(*[d.ctypes.data for d in datas])
    outs = (ctypes.c_void_p * B)(*[p_.ctypes.data for p_ in pars])
    st = (ctypes.c_int * B)()
    rc = lib.rs_encode_batch(f.handle, B, ins, k * S, outs, st)
    assert rc == 0 and not any(st), f"k={k} n={n} S={S} B={B} encode_batch rc {rc} {list(st)[:4]}"
    for b in range(B):
        assert pars[b].tobytes() == oracle.encode(E, k, n, datas[b].tobytes()), f"k={k} n={n} S={S} B={B} batch parity {b}"
    stats["encode_batch_msgs"] += B
    # decode: per message its own share set (k or more), maybe one corrupted share
    counts, nums, ptrs, keep, refs, arenas = [], [], [], [], [], []
    in_arena = rng.random() < 0.4
    arena = rsmi.Arena(B * n * (S + 256) + 4096) if in_arena else None
    # aliasing: message b's shares in rows of block b, its dst in block (b + off) % B
    alias = not in_arena and rng.random() < 0.15
    rows = n + 2
    blk_bytes = rows * S + S
    blk_pinned = alias and rng.random() < 0.5
    blk_keep = None
    if alias:
        if blk_pinned:
            base = lib.rs_pinned_alloc(B * blk_bytes)
        else:
            blk_keep = np.zeros(B * blk_bytes, dtype=np.uint8)
            base = blk_keep.ctypes.data
        off = int(rng.integers(0, 2))
        shift = int(rng.integers(0, S)) if rng.random() < 0.5 else 0
    for b in range(B):
        cnt = k if rng.random() < 0.7 else int(rng.integers(k, n + 1))
        ids = [int(v) for v in rng.choice(n, size=cnt, replace=False)]
        sh = {i: (datas[b][i * S:(i + 1) * S] if i < k else pars[b][(i - k) * S:(i - k + 1) * S]).copy() for i in ids}
        if cnt >= k + 2 and rng.random() < 0.5:
            v = ids[int(rng.integers(0, cnt))]
            sh[v][int(rng.integers(0, S))] ^= np.uint8(1 + int(rng.integers(0, 255)))
        shares = [(i, sh[i].tobytes()) for i in ids]
        refs.append(oracle.decode(E, k, n, shares) if cnt == k else oracle.decode_correct(E, k, n, shares))
        counts.append(cnt)
        perm = rng.permutation(rows)
        for j, i in enumerate(ids):
            nums.append(i)
            if alias:
                a = base + b * blk_bytes + int(perm[j]) * S
                ctypes.memmove(a, sh[i].tobytes(), S)
                ptrs.append(a)
            elif arena is not None:
                ptrs.append(arena.put(sh[i].tobytes()))
            else:
                keep.append(sh[i])
                ptrs.append(sh[i].ctypes.data)
    dsts = [np.zeros(k * S, dtype=np.uint8) for _ in range(B)]
    dptr = ([base + ((b + off) % B) * blk_bytes + shift for b in range(B)] if alias
            else [d.ctypes.data for d in dsts])
    cc = (ctypes.c_int * B)(*counts)
    nn = (ctypes.c_int * len(nums))(*nums)
    pp = (ctypes.c_void_p * len(ptrs))(*ptrs)
    dd = (ctypes.c_void_p * B)(*dptr)
    st = (ctypes.c_int * B)()
    lib.rs_decode_batch(f.handle, B, cc, nn, pp, S, dd, st)
    if alias:
        for b in range(B):
            dsts[b][:] = np.frombuffer(ctypes.string_at(dptr[b], k * S), dtype=np.uint8)
        if blk_pinned:
            lib.rs_pinned_free(base)
        stats["aliased_batch_msgs"] += B
    if arena is not None:
        arena.free()
    for b in range(B):
        ref_rc, ref = refs[b]
        assert (st[b] == 0) == (ref_rc == 0), f"k={k} n={n} S={S} B={B} alias={alias} decode_batch msg {b} rc {st[b]} vs {ref_rc}"
        if st[b] == 0:
            assert dsts[b].tobytes() == ref == datas[b].tobytes(), f"k={k} n={n} S={S} B={B} alias={alias} decode_batch msg {b} bytes"
    stats["decode_batch_msgs"] += B


def run(seconds=None, cases=None, seed=1):
    import rsmi
    from oracle import oracle

    rng = np.random.default_rng(seed)
    lib = rsmi.load()
    P = ctypes.c_void_p
    fecs, mats = {}, {}
    stats = {"cases": 0, "encode": 0, "decode_k": 0, "decode_more": 0, "corrupted": 0, "arena": 0,
             "pinned_dst": 0, "aliased": 0, "encode_batch_msgs": 0, "decode_batch_msgs": 0,
             "aliased_batch_msgs": 0, "failures": 0}
    first = []
    t0 = last_note = time.time()
    while (cases is None or stats["cases"] < cases) and (seconds is None or time.time() - t0 < seconds):
        if time.time() - last_note > 30:  # progress on stderr: a long run is seen to be alive
            last_note = time.time()
            print(f"fuzz_host_api: {stats['cases']} cases, {stats['failures']} failures, {last_note - t0:.0f} s",
                  file=sys.stderr, flush=True)
        k, n = CODES[int(rng.integers(0, len(CODES)))]
        m = n - k
        if (k, n) not in fecs:
            fecs[(k, n)] = rsmi.FEC(k, n)
            mats[(k, n)] = oracle.fec_matrix(k, n)
        f, E = fecs[(k, n)], mats[(k, n)]
        smax = max(1, min(300_000, 4_000_000 // k))
        S = int(np.exp(rng.uniform(0, np.log(smax))))
        if rng.random() < 0.3:
            S = max(16, S // 16 * 16)
        data = oracle.splitmix_bytes(k * S, int(rng.integers(0, 2**32)))
        par = np.zeros(m * S, dtype=np.uint8)
        case = f"k={k} n={n} S={S}"
        stats["cases"] += 1
        try:
            assert lib.rs_encode(f.handle, P(data.ctypes.data), k * S, P(par.ctypes.data)) == 0, case + " encode rc"
            assert par.tobytes() == oracle.encode(E, k, n, data.tobytes()), case + " parity"
            stats["encode"] += 1
            shard = lambda i: data[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S]
            cnt = k if rng.random() < 0.6 else int(rng.integers(k, n + 1))
            ids = [int(v) for v in rng.choice(n, size=cnt, replace=False)]
            bufs = {i: np.ascontiguousarray(shard(i)).copy() for i in ids}
            corrupt = cnt >= k + 2 and rng.random() < 0.5
            if corrupt:
                v = ids[int(rng.integers(0, cnt))]
                pos = int(rng.integers(0, S))
                bufs[v][pos] ^= np.uint8(1 + int(rng.integers(0, 255)))
                stats["corrupted"] += 1
            where = rng.random()
            arena = None
            ptr = {}
            # aliasing: the shares and dst in one buffer (random rows, dst at a
            # random row and byte shift), pinned or pageable
            alias = rng.random() < 0.15
            alias_keep = alias_pinned = None
            if alias:
                rows = n + 2
                size = rows * S + S
                alias_pinned = rng.random() < 0.5
                if alias_pinned:
                    blk = lib.rs_pinned_alloc(size)
                else:
                    alias_keep = np.zeros(size, dtype=np.uint8)
                    blk = alias_keep.ctypes.data
                perm = rng.permutation(rows)
                for j, i in enumerate(ids):
                    ptr[i] = blk + int(perm[j]) * S
                    ctypes.memmove(ptr[i], bufs[i].tobytes(), S)
                stats["aliased"] += 1
            elif where < 0.35:  # every survivor in an engine-pinned arena slot
                arena = rsmi.Arena(sum(S + 256 for _ in ids) + 4096)
                for i in ids:
                    ptr[i] = arena.put(bufs[i].tobytes())
                stats["arena"] += 1
            elif where < 0.5 and cnt > 1:  # mixed: some pinned, some pageable
                arena = rsmi.Arena(sum(S + 256 for _ in ids) + 4096)
                for j, i in enumerate(ids):
                    ptr[i] = arena.put(bufs[i].tobytes()) if j % 2 else bufs[i].ctypes.data
            else:
                for i in ids:
                    ptr[i] = bufs[i].ctypes.data
            pinned_dst = not alias and rng.random() < 0.25
            if alias:
                drow = int(rng.integers(0, rows - k + 1))
                dp = blk + drow * S + (int(rng.integers(0, S)) if rng.random() < 0.5 else 0)
            elif pinned_dst:
                dp = lib.rs_pinned_alloc(max(k * S, 16))
                ctypes.memset(dp, 0, max(k * S, 16))
                stats["pinned_dst"] += 1
            else:
                dst = np.zeros(k * S, dtype=np.uint8)
                dp = dst.ctypes.data
            nums = (ctypes.c_int * cnt)(*ids)
            ptrs = (ctypes.c_void_p * cnt)(*[ptr[i] for i in ids])
            rc = lib.rs_decode(f.handle, nums, ptrs, cnt, S, P(dp))
            got = ctypes.string_at(dp, k * S)
            shares = [(i, bufs[i].tobytes()) for i in ids]
            if cnt == k:
                ref_rc, ref = oracle.decode(E, k, n, shares)
                stats["decode_k"] += 1
            else:
                ref_rc, ref = oracle.decode_correct(E, k, n, shares)
                stats["decode_more"] += 1
            if pinned_dst:
                lib.rs_pinned_free(dp)
            if alias_pinned:
                lib.rs_pinned_free(blk)
            if arena is not None:
                arena.free()
            case += f" alias={alias}"
            assert (rc == 0) == (ref_rc == 0), f"{case} cnt={cnt} corrupt={corrupt} rc {rc} vs oracle {ref_rc}"
            if rc == 0:
                assert got == ref, f"{case} cnt={cnt} corrupt={corrupt} decode bytes"
                assert got == data.tobytes(), f"{case} cnt={cnt} corrupt={corrupt} not the message"
            if stats["cases"] % 4 == 0:
                batch_case(rng, lib, f, E, k, n, S, stats, oracle, rsmi)
        except AssertionError as e:
            stats["failures"] += 1
            if len(first) < 5:
                first.append(str(e))
    for fc in fecs.values():
        fc.close()
    stats["seconds"] = round(time.time() - t0, 1)
    stats["first_failures"] = first
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=None)
    ap.add_argument("--cases", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    if a.seconds is None and a.cases is None:
        a.seconds = 120.0
    st = run(a.seconds, a.cases, a.seed)
    print(json.dumps(st))
    return 1 if st["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
