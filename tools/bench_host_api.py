#!/usr/bin/env python3
"""Host-buffer (PCIe-inclusive) rates of the engine: the cgo path the plugin
uses (rs_encode / rs_decode: pageable host buffers, H2D, kernel, D2H) and
BASELINE config 1 end to end through the C++ ShardPlugin mirror, next to
the CPU oracle on the same inputs.  Not the bench.py headline (which is
device-resident); DESIGN.md quotes these as the PCIe-inclusive numbers.

    python tools/bench_host_api.py [--reps 20]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "noise-erasurecode-plugin_amd")]

import numpy as np  # noqa: E402


def timeit(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch-only", action="store_true", help="only the receive-batching section")
    ap.add_argument("--batch-reps", type=int, default=3)
    a = ap.parse_args()
    import rsmi
    from rsmi import host as h
    from oracle import oracle

    import ctypes
    lib = rsmi.load()
    out = {}
    k, n = 10, 14
    m = n - k
    f = rsmi.NewFEC(k, n)
    E = oracle.fec_matrix(k, n)
    P = ctypes.c_void_p
    sizes = (("config1_blob_1MiB+4", (1 << 20) + 4), ("msg_64KiB", 65540), ("msg_64MiB", 64 << 20),
             ("msg_640MiB", 640 << 20))
    for name, size in (() if a.batch_only else sizes):
        size -= size % k
        S = size // k
        blob = oracle.splitmix_bytes(size, 1)
        parity = np.zeros(m * S, dtype=np.uint8)
        reps = a.reps if size < (100 << 20) else 5
        # rs_encode on caller-owned pageable buffers (what the cgo shim passes)
        t_enc = timeit(lambda: lib.rs_encode(f.handle, P(blob.ctypes.data), size,
                                             P(parity.ctypes.data)), reps)
        lost = (0, 4, 6, 10)
        keep = [i for i in range(n) if i not in lost]
        shard = lambda i: (blob[i * S:(i + 1) * S] if i < k else parity[(i - k) * S:(i - k + 1) * S])
        bufs = [np.ascontiguousarray(shard(i)) for i in keep]
        dst = np.zeros(size, dtype=np.uint8)

        def dec():
            nums = (ctypes.c_int * len(keep))(*keep)
            ptrs = (ctypes.c_void_p * len(keep))(*[b.ctypes.data for b in bufs])
            rc = lib.rs_decode(f.handle, nums, ptrs, len(keep), S, P(dst.ctypes.data))
            assert rc == 0
        t_dec = timeit(dec, reps)
        assert (dst == blob).all()
        if size <= (64 << 20):
            assert parity.tobytes() == oracle.encode(E, k, n, blob.tobytes())
        rec = {"bytes": size,
               "encode_ms": round(t_enc * 1e3, 3),
               "encode_GBps_pcie_inclusive": round(size * n / k / t_enc / 1e9, 2),
               "decode4_ms": round(t_dec * 1e3, 3),
               "decode4_GBps_pcie_inclusive": round(size * n / k / t_dec / 1e9, 2)}
        # The same calls on engine-pinned buffers (16-byte shards): the
        # kernel reads and writes them in place over PCIe.
        Sp = S // 16 * 16
        if Sp:
            sp = Sp * k
            pin_in, pin_par, pin_dst = (lib.rs_pinned_alloc(sp), lib.rs_pinned_alloc(m * Sp),
                                        lib.rs_pinned_alloc(sp))
            ctypes.memmove(pin_in, blob.ctypes.data, sp)
            e0 = f.stat(f.STAT_ENCODES_IN_PLACE)
            t_penc = timeit(lambda: lib.rs_encode(f.handle, pin_in, sp, pin_par), reps)
            assert f.stat(f.STAT_ENCODES_IN_PLACE) > e0
            pkeep = [pin_in + i * Sp if i < k else pin_par + (i - k) * Sp for i in keep]

            def pdec():
                nums = (ctypes.c_int * len(keep))(*keep)
                ptrs = (ctypes.c_void_p * len(keep))(*pkeep)
                assert lib.rs_decode(f.handle, nums, ptrs, len(keep), Sp, P(pin_dst)) == 0
            t_pdec = timeit(pdec, reps)
            assert ctypes.string_at(pin_dst, sp) == blob[:sp].tobytes()
            for q in (pin_in, pin_par, pin_dst):
                lib.rs_pinned_free(q)
            rec.update({"pinned_encode_ms": round(t_penc * 1e3, 3),
                        "pinned_encode_GBps_pcie_inclusive": round(sp * n / k / t_penc / 1e9, 2),
                        "pinned_decode4_ms": round(t_pdec * 1e3, 3),
                        "pinned_decode4_GBps_pcie_inclusive": round(sp * n / k / t_pdec / 1e9, 2)})
        if size <= (64 << 20):
            t_cpu = timeit(lambda: oracle.encode(E, k, n, blob.tobytes()), 3)
            rec["cpu_oracle_scalar_encode_ms"] = round(t_cpu * 1e3, 3)
        out[name] = rec

    # config 1 through the plugin mirror: prepareShards -> Marshal -> drop 4 ->
    # Unmarshal -> Receive x10 -> Decode of the pooled shares.
    blob = oracle.splitmix_bytes(1 << 20, 0x5EED).tobytes() + b"\0" * 4
    me = h.PeerID("tcp://localhost:3000", b"\x11" * 32)
    sign = lambda m: hashlib.sha512(m).digest()  # ed25519 stand-in (out of scope)
    verify = lambda m, s: hashlib.sha512(m).digest() == s

    hf = h.NewFEC(k, n)

    def config1():
        p = h.NewShardPlugin(sign, verify, k, n)
        wires = [s.Marshal() for s in p.prepareShards(me, blob)]
        recv = h.NewShardPlugin(sign, verify, k, n)
        got = []
        for i in (1, 2, 3, 5, 7, 8, 9, 11, 12, 13):
            s = h.Shard()
            s.Unmarshal(wires[i])
            recv.Receive(me, s)
            got.append(h.Share(int(s.ShardNumber), s.ShardData))
        msg, _ = hf.Decode(None, got)
        assert msg == blob
    if not a.batch_only:
        out["config1_plugin_end_to_end_ms"] = round(timeit(config1, a.reps) * 1e3, 3)

    # receive-side batching at the C ABI: B messages, each arriving with 4 of
    # its 14 shards lost -> B rs_decode calls vs one rs_decode_batch.
    for label, B, S in (("receive_batch_256x1MiB", 256, 104858), ("receive_batch_2048x64KiB", 2048, 6554)):
        rng = np.random.default_rng(3)
        data = oracle.splitmix_bytes(k * S, 9)
        par = np.zeros(m * S, dtype=np.uint8)
        lib.rs_encode(f.handle, P(data.ctypes.data), k * S, P(par.ctypes.data))
        shard = lambda i: (data[i * S:(i + 1) * S] if i < k else par[(i - k) * S:(i - k + 1) * S])
        losts = [set(rng.choice(n, size=4, replace=False).tolist()) for _ in range(B)]
        keeps = [[i for i in range(n) if i not in lost] for lost in losts]
        bufs = [[np.ascontiguousarray(shard(i)) for i in kp] for kp in keeps]
        dsts = [np.zeros(k * S, dtype=np.uint8) for _ in range(B)]
        cnt = sum(len(kp) for kp in keeps)
        nums = (ctypes.c_int * cnt)()
        ptrs = (ctypes.c_void_p * cnt)()
        counts = (ctypes.c_int * B)(*[len(kp) for kp in keeps])
        outp = (ctypes.c_void_p * B)(*[d.ctypes.data for d in dsts])
        st = (ctypes.c_int * B)()

        def fill():
            j = 0
            for kp, bl in zip(keeps, bufs):
                for i, bb in zip(kp, bl):
                    nums[j] = i
                    ptrs[j] = bb.ctypes.data
                    j += 1

        def seq():
            fill()
            j = 0
            for b in range(B):
                c = counts[b]
                pn = ctypes.cast(ctypes.c_void_p(ctypes.addressof(nums) + 4 * j), ctypes.POINTER(ctypes.c_int))
                pp = ctypes.cast(ctypes.c_void_p(ctypes.addressof(ptrs) + 8 * j), ctypes.POINTER(ctypes.c_void_p))
                rc = lib.rs_decode(f.handle, pn, pp, c, S, P(dsts[b].ctypes.data))
                assert rc == 0
                j += c

        def bat():
            fill()
            rc = lib.rs_decode_batch(f.handle, B, counts, nums, ptrs, S, outp, st)
            assert rc == 0

        t_seq = timeit(seq, 3)
        t_bat = timeit(bat, a.batch_reps)
        assert all((d == data).all() for d in dsts)
        # Zero-copy receive: the same survivors in an engine-pinned arena
        # (where rs_shard_unmarshal_arena puts ShardData); the kernel reads
        # them in place over PCIe.
        arena = rsmi.Arena(B * n * ((S + 255) // 256 * 256) + 4096)
        abufs = [[arena.put(bb.tobytes()) for bb in bl] for bl in bufs]
        for d in dsts:
            d[:] = 0

        def arena_fill():
            j = 0
            for kp, bl in zip(keeps, abufs):
                for i, pa in zip(kp, bl):
                    nums[j] = i
                    ptrs[j] = pa
                    j += 1

        def bat_arena():
            arena_fill()
            rc = lib.rs_decode_batch(f.handle, B, counts, nums, ptrs, S, outp, st)
            assert rc == 0
        in0 = f.stat(f.STAT_BATCHES_IN_PLACE)
        t_arena = timeit(bat_arena, a.batch_reps)
        assert f.stat(f.STAT_BATCHES_IN_PLACE) > in0
        assert all((d == data).all() for d in dsts)
        arena.free()
        out[label] = {"per_message_ms": round(t_seq / B * 1e3, 4),
                      "batched_ms_per_message": round(t_bat / B * 1e3, 4),
                      "speedup": round(t_seq / t_bat, 2),
                      "batched_GBps_pcie_inclusive": round(B * n * S / t_bat / 1e9, 2),
                      "in_place_ms_per_message": round(t_arena / B * 1e3, 4),
                      "in_place_GBps_pcie_inclusive": round(B * n * S / t_arena / 1e9, 2),
                      "in_place_speedup_vs_staged": round(t_bat / t_arena, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
