"""Concurrent calls on one rs_ctx (SURVEY.md §8b threading row).

The reference's Receive runs once per peer connection, concurrently
(main.go:49-52, the sync.Map pool), and the Go shim shares one context per
(k, n) between all goroutines.  Each C-ABI call leases its own stream,
staging and device workspace, and only the decode-pattern cache is shared
(reader/writer lock).  These tests drive one context from several threads
(ctypes releases the GIL for the duration of each call) and check every
result bit-exact against the oracle; they also cover the cross-stream cases
the lease events order (a reconstruct on the NULL stream interleaved with
rs_decode_batch on the lease streams), eviction of the pattern cache without
a host sync, and that rs_free returns the lease buffers.
"""
import ctypes
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402


def _message(k, n, S, seed):
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, seed).tobytes()
    par = oracle.encode(E, k, n, data)
    sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
    return data, sh


def _fec_env(k, n, **env):
    old = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    try:
        return rsmi.FEC(k, n)
    finally:
        for key, v in old.items():
            if v is None:
                del os.environ[key]
            else:
                os.environ[key] = v


@pytest.mark.parametrize("k,n,S", [(10, 14, 104858), (64, 80, 4099)])
def test_concurrent_decode_one_fec(k, n, S):
    """8 threads call Decode on one FEC at once, each on its own messages
    with its own erasures; every output equals the oracle's Rebuild."""
    f = rsmi.FEC(k, n)
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(k + S)
    jobs = []
    for j in range(24):
        data, sh = _message(k, n, S, 1000 + j)
        keep = sorted(rng.choice(n, size=k, replace=False).tolist())
        rng.shuffle(keep)
        rc, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep])
        assert rc == 0 and ref == data
        jobs.append((keep, sh, ref))

    def run(job):
        keep, sh, ref = job
        out = []
        for _ in range(3):
            out.append(f.Decode(None, [rsmi.Share(i, sh[i]) for i in keep]))
        return all(o == ref for o in out)

    with ThreadPoolExecutor(8) as ex:
        assert all(ex.map(run, jobs))
    f.close()


def test_concurrent_encode_and_decode_batch():
    """Encode, DecodeBatch and EncodeBatch from different threads on one FEC."""
    k, n, S = 10, 14, 65536
    f = rsmi.FEC(k, n)
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(11)
    msgs = [_message(k, n, S, 50 + j) for j in range(12)]
    errors = []

    def encoder(j):
        data, sh = msgs[j]
        for _ in range(4):
            got = f.encode_parity(data)
            if got != b"".join(sh[k:]):
                errors.append(("encode", j))

    def batcher(j):
        batch = []
        for data, sh in msgs:
            keep = sorted(rng.choice(n, size=k, replace=False).tolist())
            batch.append([rsmi.Share(i, sh[i]) for i in keep])
        outs, st = f.DecodeBatch(batch)
        for (data, _), o, s in zip(msgs, outs, st):
            if s != 0 or o != data:
                errors.append(("batch", j))

    def enc_batcher(j):
        for _ in range(3):
            pars, st = f.EncodeBatch([data for data, _ in msgs])
            for (data, sh), p, s in zip(msgs, pars, st):
                if s != 0 or p != b"".join(sh[k:]):
                    errors.append(("encode_batch", j))

    with ThreadPoolExecutor(8) as ex:
        futs = ([ex.submit(encoder, j) for j in range(6)] + [ex.submit(batcher, j) for j in range(4)] +
                [ex.submit(enc_batcher, j) for j in range(4)])
        for fu in futs:
            fu.result()
    assert not errors, errors[:5]
    f.close()


def test_reconstruct_null_stream_interleaved_with_decode_batch():
    """rs_reconstruct_stripes on the NULL stream and
    rs_decode_batch on the lease streams of one ctx, alternating, with fresh
    RS(64,16) patterns (so both build decode rows and both reuse stripe
    descriptor buffers).  Each result equals the originals / the oracle."""
    k, n, S = 64, 80, 8192
    m = n - k
    f = rsmi.FEC(k, n)
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(2024)
    stripes = 16
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 3)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    msgs = [_message(k, n, 1000, 70 + j) for j in range(6)]
    for it in range(6):
        er = np.zeros((stripes, n), dtype=np.uint8)
        for s in range(stripes):
            er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
        data.copy_(d0)
        parity.copy_(p0)
        data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
        parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                              er.tobytes())  # NULL stream, no sync before the next call
        batch = []
        for data_b, sh in msgs:
            keep = sorted(rng.choice(n, size=k, replace=False).tolist())
            batch.append([rsmi.Share(i, sh[i]) for i in keep])
        outs, st = f.DecodeBatch(batch)
        assert st == [0] * len(msgs)
        assert all(o == d for o, (d, _) in zip(outs, msgs))
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0), it
    f.close()


def test_pattern_cache_eviction_without_sync():
    """With a pattern cap of 24, RS(64,16) calls with fresh patterns evict the
    cache again and again (no host sync); every reconstruct stays exact and
    two threads doing it at once on one ctx agree with the originals."""
    k, n, S = 64, 80, 4096
    m = n - k
    f = _fec_env(k, n, RSMI_PATTERN_CAP="24")
    stripes = 10
    bufs = []
    for t in range(2):
        data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
        parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
        f.fill_splitmix(data.data_ptr(), data.numel(), 40 + t)
        f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
        bufs.append((data, parity))
    f.sync()
    refs = [(d.clone(), p.clone()) for d, p in bufs]
    errors = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        data, parity = bufs[t]
        d0, p0 = refs[t]
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            for it in range(12):
                er = np.zeros((stripes, n), dtype=np.uint8)
                for s in range(stripes):
                    er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
                data.copy_(d0)
                parity.copy_(p0)
                data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
                parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
                f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes,
                                      er.tobytes(), stream.cuda_stream)
                stream.synchronize()
                if not (torch.equal(data, d0) and torch.equal(parity, p0)):
                    errors.append((t, it))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    assert f.pattern_evictions() >= 4
    assert f.pattern_count() <= 24 + stripes
    # rows built after evictions still match the oracle's Rebuild rows
    er = np.zeros(n, dtype=np.uint8)
    er[[0, 5, 70]] = 1
    rows, cnt = f.pattern_rows(er.tobytes())
    import np_rs
    from rsmi import distributed as rd
    E = oracle.fec_matrix(k, n)
    surv = rd.choose_survivors(er, k, n)
    rc, inv = oracle.invert(E[surv])
    assert rc == 0 and cnt == 3
    assert (np.frombuffer(rows, np.uint8).reshape(m, k)[:3] == np_rs.matmul(E[[0, 5, 70]], inv)).all()
    f.close()


@pytest.mark.parametrize("cap", [None, "40"])
def test_watermark_reuse_while_tables_move(cap):
    """launch_reconstruct skips its wait for the pattern builds
    when every pattern it reads is older than its lease's watermark and the
    tables have not moved (rsmi.cpp wait_patterns_for).  One thread reuses a
    fixed, long-cached pattern set over and over while another meets fresh
    patterns on every call, growing the device tables (cap None) or evicting
    and rebuilding them (cap 40); with two leases the callers keep trading
    leases.  Every reconstruct of both threads equals the originals."""
    k, n, S = 64, 80, 4096
    m = n - k
    env = {"RSMI_MAX_LEASES": "2"}
    if cap:
        env["RSMI_PATTERN_CAP"] = cap
    f = _fec_env(k, n, **env)
    stripes = [8, 48]  # reuser, builder
    bufs = []
    for t in range(2):
        data = torch.empty(stripes[t] * k * S, dtype=torch.uint8, device="cuda")
        parity = torch.empty(stripes[t] * m * S, dtype=torch.uint8, device="cuda")
        f.fill_splitmix(data.data_ptr(), data.numel(), 70 + t)
        f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes[t])
        bufs.append((data, parity))
    f.sync()
    refs = [(d.clone(), p.clone()) for d, p in bufs]
    fixed = np.zeros((stripes[0], n), dtype=np.uint8)
    rng0 = np.random.default_rng(5)
    for s in range(stripes[0]):
        fixed[s, rng0.choice(n, size=int(rng0.integers(1, m + 1)), replace=False)] = 1
    errors = []
    seen = set()  # the builder's distinct patterns

    def worker(t):
        rng = np.random.default_rng(200 + t)
        data, parity = bufs[t]
        d0, p0 = refs[t]
        st = stripes[t]
        stream = torch.cuda.Stream()
        with torch.cuda.stream(stream):
            for it in range(30):
                if t == 0:
                    er = fixed
                else:
                    er = np.zeros((st, n), dtype=np.uint8)
                    for s in range(st):
                        er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
                    seen.update(row.tobytes() for row in er)
                data.copy_(d0)
                parity.copy_(p0)
                data.view(st, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
                parity.view(st, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0
                f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, st,
                                      er.tobytes(), stream.cuda_stream)
                stream.synchronize()
                if not (torch.equal(data, d0) and torch.equal(parity, p0)):
                    errors.append((t, it))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    if cap:
        assert f.pattern_evictions() >= 10
    else:
        assert f.pattern_count() >= len(seen) > 1000  # every pattern kept: the tables grew again and again
    f.close()


def test_rs_free_releases_lease_buffers():
    """rs_free must free every lease's device and pinned buffers
    (the rs_decode_batch workspaces included).  Three create / batch-decode
    / free cycles leave device memory where it started."""
    k, n, S = 10, 14, 1 << 18
    msgs = [_message(k, n, S, 300 + j) for j in range(24)]
    rng = np.random.default_rng(4)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(3):
        f = rsmi.FEC(k, n)
        batch = []
        for data, sh in msgs:
            keep = sorted(rng.choice(n, size=k, replace=False).tolist())
            batch.append([rsmi.Share(i, sh[i]) for i in keep])
        outs, st = f.DecodeBatch(batch)
        assert st == [0] * len(msgs) and all(o == d for o, (d, _) in zip(outs, msgs))
        f.close()
    free1, _ = torch.cuda.mem_get_info()
    # one batch holds ~24 * 14 * 256 KiB * 2 = 168 MiB of device buffers
    assert free1 >= free0 - (32 << 20), (free0, free1)


def test_prepare_patterns_status_per_pattern():
    """rs_prepare_patterns / rs_pattern_rows report each pattern's own
    inversion status (the old shared status word was never
    cleared); a valid MDS pattern after many builds is RS_OK."""
    f = rsmi.FEC(10, 14)
    f.prepare_patterns(4)
    assert f.pattern_count() == 1470
    er = np.zeros(14, dtype=np.uint8)
    er[[1, 2, 12, 13]] = 1
    rows, cnt = f.pattern_rows(er.tobytes())
    assert cnt == 4
    f.close()


def test_lease_pool_bound():
    """RSMI_MAX_LEASES=2 with 6 concurrent callers: calls wait for a lease and
    all complete bit-exact."""
    k, n, S = 4, 6, 40000
    f = _fec_env(k, n, RSMI_MAX_LEASES="2")
    msgs = [_message(k, n, S, 900 + j) for j in range(6)]

    def run(j):
        data, sh = msgs[j]
        return f.Decode(None, [rsmi.Share(i, sh[i]) for i in (5, 0, 4, 2)]) == data

    with ThreadPoolExecutor(6) as ex:
        assert all(ex.map(run, range(6)))
    f.close()


def _erase(data, parity, er, k, m, S, stripes):
    data.view(stripes, k, S)[torch.from_numpy(er[:, :k].astype(bool)).cuda()] = 0
    parity.view(stripes, m, S)[torch.from_numpy(er[:, k:].astype(bool)).cuda()] = 0


def test_failed_pattern_build_rolls_back():
    """a build that fails after a call created patterns
    must not leave them in the cache.  RSMI_TEST_FAIL_FLUSH=1 makes the
    context's first build fail (RS_ENOMEM, as an allocation failure would);
    the call reports it and the cache is empty again.  The same patterns
    then reconstruct exactly -- through the exclusive path (which rebuilds
    them) and through a second call that only finds them (shared path)."""
    k, n, S, stripes = 64, 80, 4096, 12
    m = n - k
    f = _fec_env(k, n, RSMI_TEST_FAIL_FLUSH="1")
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 91)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    rng = np.random.default_rng(91)
    er = np.zeros((stripes, n), dtype=np.uint8)
    for s in range(stripes):
        er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
    _erase(data, parity, er, k, m, S, stripes)
    with pytest.raises(rsmi.RSError) as ei:
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
    assert ei.value.code == rsmi.RS_ENOMEM
    assert f.pattern_count() == 0  # rolled back, nothing half-built stays findable
    for _ in range(2):  # 1st: patterns created and built again; 2nd: found (shared path)
        data.copy_(d0)
        parity.copy_(p0)
        _erase(data, parity, er, k, m, S, stripes)
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0)
    assert f.pattern_count() == len({row.tobytes() for row in er})
    f.close()


def test_eviction_counts_distinct_new_patterns():
    """near the cap, a batch whose many stripes share ONE
    new pattern must not evict the cache (the check counts distinct new
    patterns, not stripes)."""
    k, n, S, stripes = 10, 14, 4096, 64
    m = n - k
    f = _fec_env(k, n, RSMI_PATTERN_CAP="8")
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda")
    f.fill_splitmix(data.data_ptr(), data.numel(), 5)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    f.sync()
    d0, p0 = data.clone(), parity.clone()
    for ids in ([0], [1], [2], [0, 1], [2, 3], [12]):  # 6 cached patterns, cap 8
        er = np.zeros((stripes, n), dtype=np.uint8)
        er[:, ids] = 1
        data.copy_(d0)
        parity.copy_(p0)
        _erase(data, parity, er, k, m, S, stripes)
        f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
        f.sync()
        assert torch.equal(data, d0) and torch.equal(parity, p0), ids
    assert f.pattern_count() == 6 and f.pattern_evictions() == 0
    # 64 stripes, one new pattern: 6 + 1 <= 8, no eviction
    er = np.zeros((stripes, n), dtype=np.uint8)
    er[:, [3, 9, 11]] = 1
    data.copy_(d0)
    parity.copy_(p0)
    _erase(data, parity, er, k, m, S, stripes)
    f.reconstruct_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes, er.tobytes())
    f.sync()
    assert torch.equal(data, d0) and torch.equal(parity, p0)
    assert f.pattern_count() == 7 and f.pattern_evictions() == 0
    f.close()


def test_lease_buffers_grow_concurrently():
    """lease buffers (device workspaces, pinned staging, the
    host pipeline's slots) grow without a device-wide sync.  8 threads on one
    context call DecodeBatch and Decode with monotonically growing messages,
    so every call outgrows the buffers of the lease it gets; every result is
    bit-exact against the oracle."""
    k, n = 10, 14
    f = rsmi.FEC(k, n)
    E = oracle.fec_matrix(k, n)
    sizes = [160 * (2 ** (i / 2)) for i in range(16)]  # 160 B .. ~29 KiB per shard
    errors = []

    def worker(t):
        rng = np.random.default_rng(500 + t)
        for i, sz in enumerate(sizes):
            S = int(sz) + t  # ragged, distinct per thread
            msgs = [_message(k, n, S, 10_000 * t + 100 * i + j) for j in range(1 + (i + t) % 4)]
            batch = []
            for data, sh in msgs:
                keep = rng.choice(n, size=k, replace=False).tolist()
                batch.append([rsmi.Share(x, sh[x]) for x in keep])
            outs, st = f.DecodeBatch(batch)
            if st != [0] * len(msgs) or any(o != d for o, (d, _) in zip(outs, msgs)):
                errors.append(("batch", t, i))
            data, sh = msgs[0]
            keep = rng.choice(n, size=k, replace=False).tolist()
            rc, ref = oracle.decode(E, k, n, [(x, sh[x]) for x in keep])
            if rc != 0 or f.Decode(None, [rsmi.Share(x, sh[x]) for x in keep]) != ref:
                errors.append(("decode", t, i))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    f.close()
