"""Multi-process (gloo, world_size 2 and 3, CPU) tests of the shard-distributed
survivor gather (rsmi/distributed.py): the exchange plan
delivers exactly the k survivors of every owned stripe that Rebuild would
read, the shard table points at them where they landed (receive buffer or
local holder buffer), and reconstructing from exactly those bytes gives the
original stripes (the reconstruct is done here by the oracle; on the GPU it
is rs_reconstruct_ptrs through the same table, tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rsmi import distributed as rd

K, N, S, STRIPES = 10, 14, 64, 23


def dataset(seed=7):
    from oracle import oracle
    E = oracle.fec_matrix(K, N)
    data = oracle.splitmix_bytes(STRIPES * K * S, seed)
    par = oracle.encode_batch(E, K, N, data, S, STRIPES, simd=False)
    full = np.concatenate([data.reshape(STRIPES, K, S), par.reshape(STRIPES, N - K, S)], axis=1)
    rng = np.random.default_rng(seed)
    er = np.zeros((STRIPES, N), dtype=np.uint8)
    for s in range(STRIPES):
        er[s, rng.choice(N, size=int(rng.integers(1, N - K + 1)), replace=False)] = 1
    return E, full, er


def test_choose_survivors_matches_oracle_rule():
    rng = np.random.default_rng(0)
    for _ in range(300):
        er = np.zeros(N, dtype=np.uint8)
        er[rng.choice(N, size=int(rng.integers(0, 5)), replace=False)] = 1
        surv = rd.choose_survivors(er, K, N)
        assert len(set(surv)) == K and not any(er[i] for i in surv)
        assert all(surv[i] == i for i in range(K) if not er[i])


def _plan_reference(erased, k, n, rank, world, S):
    """The round-2 loop plan (one chunk), kept as the reference of the
    vectorised plan: per stripe, Rebuild's survivors (in id order), then
    holder/owner bookkeeping one shard at a time."""
    stripes = erased.shape[0]
    nloc = len(rd.local_shard_ids(rank, n, world))
    owned = [s for s in range(stripes) if rd.owner(s, world) == rank]
    send = {p: [] for p in range(world) if p != rank}
    recv_rows = {p: [] for p in range(world) if p != rank}
    kind = np.full((len(owned), n), rd.UNUSED, dtype=np.int8)
    row = np.zeros((len(owned), n), dtype=np.int64)
    n_out = 0
    opos = {s: j for j, s in enumerate(owned)}
    for s in range(stripes):
        o = rd.owner(s, world)
        surv = sorted(rd.choose_survivors(erased[s], k, n))
        if o == rank:
            for i in range(n):
                if erased[s, i]:
                    kind[opos[s], i] = rd.OUTPUT
                    row[opos[s], i] = n_out
                    n_out += 1
        for i in surv:
            hd = rd.holder(i, world)
            if hd == rank and o == rank:
                kind[opos[s], i] = rd.LOCAL
                row[opos[s], i] = s * nloc + i // world
            elif hd == rank:
                send[o].append(s * nloc + i // world)
            elif o == rank:
                recv_rows[hd].append((opos[s], i))
    recv, recv_off, off = {}, {}, 0
    for p in sorted(recv_rows):
        recv_off[p] = off
        for r, (j, i) in enumerate(recv_rows[p]):
            kind[j, i] = rd.REMOTE
            row[j, i] = off + r
        recv[p] = len(recv_rows[p])
        off += recv[p]
    return owned, kind, row, send, recv, recv_off, n_out, off * S


def test_survivor_mask_matches_rebuild_rule():
    rng = np.random.default_rng(3)
    for k, n in ((10, 14), (64, 80), (4, 6), (3, 3), (17, 49)):
        er = np.zeros((400, n), dtype=np.uint8)
        for s in range(400):
            er[s, rng.choice(n, size=int(rng.integers(0, n - k + 1)), replace=False)] = 1
        mask = rd.survivor_mask(er, k, n)
        for s in range(400):
            assert sorted(np.nonzero(mask[s])[0].tolist()) == sorted(rd.choose_survivors(er[s], k, n))
    with pytest.raises(ValueError):
        rd.survivor_mask(np.ones((1, N), dtype=np.uint8), K, N)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_vectorised_plan_equals_loop_plan(world):
    """the numpy plan equals the round-2 loop plan (one
    chunk): same owned stripes, kinds, rows, send lists, receive counts and
    offsets, output count and gathered bytes."""
    rng = np.random.default_rng(world)
    er = np.zeros((211, N), dtype=np.uint8)
    for s in range(211):
        er[s, rng.choice(N, size=int(rng.integers(0, N - K + 1)), replace=False)] = 1
    for rank in range(world):
        owned, kind, row, send, recv, recv_off, n_out, bytes_in = _plan_reference(er, K, N, rank, world, S)
        p = rd.plan_exchange(er, K, N, rank, world, S)
        assert p.owned.tolist() == owned
        assert np.array_equal(p.kind, kind) and np.array_equal(p.row, row)
        assert {q: v.tolist() for q, v in p.send.items()} == send
        assert p.recv == recv and p.recv_off == recv_off
        assert p.n_out == n_out and p.bytes_in == bytes_in


def test_vectorised_plan_is_fast():
    """The config-4 plan at N = 8 (52,424 global stripes) takes well under a
    second (the loop plan took seconds per step)."""
    import time
    rng = np.random.default_rng(0)
    G = 6553 * 8
    er = np.zeros((G, N), dtype=np.uint8)
    e = rng.integers(1, 5, size=G)
    pos = np.argsort(rng.random((G, N)), axis=1)
    for t in range(4):
        sel = e > t
        er[np.nonzero(sel)[0], pos[sel, t]] = 1
    t0 = time.perf_counter()
    p = rd.plan_exchange(er, K, N, 3, 8, 1 << 20, chunks=8)
    assert time.perf_counter() - t0 < 2.0
    assert len(p.chunks) == 8 and p.n_out == int(er[3::8].sum())


@pytest.mark.parametrize("world,chunks", [(1, 3), (2, 4), (3, 5), (8, 7)])
def test_plan_covers_each_survivor_once(world, chunks):
    _, _, er = dataset()
    got = {}
    plans = [rd.plan_exchange(er, K, N, r, world, S, chunks=chunks) for r in range(world)]
    for rank, p in enumerate(plans):
        for j in range(len(p.owned)):
            for i in range(N):
                if p.kind[j, i] in (rd.LOCAL, rd.REMOTE):
                    got.setdefault((rank, j, i), []).append(int(p.kind[j, i]))
        # what peers send to `rank` equals what `rank` expects from them, chunk by chunk
        for peer in range(world):
            if peer == rank:
                continue
            for c in range(len(p.chunks)):
                assert len(plans[peer].chunks[c].send[rank]) == p.chunks[c].recv[peer]
        # chunks tile the owned stripes in order
        assert [ch.lo for ch in p.chunks][0] == 0 and p.chunks[-1].hi == len(p.owned)
        assert all(a.hi == b.lo for a, b in zip(p.chunks, p.chunks[1:]))
    assert len(got) == STRIPES * K and all(len(v) == 1 for v in got.values())


def test_hbm_budget_arithmetic():
    """The per-rank budget of the shard-distributed step, before allocation:
    holder buffer, two chunk slots of send / receive rows, the output rows,
    tables and the setup batch; more chunks shrink only the slots."""
    G, world, Sb = 6553 * 8, 8, 1 << 20
    rng = np.random.default_rng(1)
    er = np.zeros((G, N), dtype=np.uint8)
    e = rng.integers(1, 5, size=G)
    pos = np.argsort(rng.random((G, N)), axis=1)
    for t in range(4):
        sel = e > t
        er[np.nonzero(sel)[0], pos[sel, t]] = 1
    nloc = len(rd.local_shard_ids(0, N, world))
    b1 = rd.hbm_budget(G, nloc, Sb, [rd.plan_exchange(er, K, N, 0, world, Sb, chunks=1)], N, k=K)
    b8 = rd.hbm_budget(G, nloc, Sb, [rd.plan_exchange(er, K, N, 0, world, Sb, chunks=8)], N, k=K)
    assert b1["held"] == b8["held"] == G * nloc * Sb / 1e9
    assert abs(b1["out"] - int(er[0::8].sum()) * Sb / 1e9) < 1e-9
    assert b8["send"] < b1["send"] / 3 and b8["recv"] < b1["recv"] / 3  # 2 slots of 1/8 vs 1 slot of all
    assert abs(b8["total"] - sum(v for key, v in b8.items() if key != "total")) < 1e-6
    assert b1["total"] > 200 and b8["total"] < 170  # GB: the round-2 sizing vs chunked slots


def test_buffers_require_16_byte_rows():
    """shard rows must stay 16-byte aligned for the kernels."""
    _, _, er = dataset()
    p = rd.plan_exchange(er, K, N, 0, 1, 100)
    with pytest.raises(ValueError):
        rd.make_buffers([p], 100, "cpu")


def _check_gathered(plan, held, bufs, full, er, E, rank, chunk=None):
    """Every survivor Rebuild reads is where the shard table says; the
    erased shards, reconstructed (by the oracle here; by rs_reconstruct_ptrs
    on the GPU) from exactly those bytes, equal the originals.  With `chunk`,
    only that chunk's owned stripes (whose slot was just filled)."""
    from oracle import oracle
    lo, hi = (0, len(plan.owned)) if chunk is None else (plan.chunks[chunk].lo, plan.chunks[chunk].hi)
    owned = list(plan.owned[lo:hi])
    data = np.zeros((len(owned), K, S), dtype=np.uint8)
    par = np.zeros((len(owned), N - K, S), dtype=np.uint8)
    for j, s in enumerate(owned):
        surv = rd.choose_survivors(er[s], K, N)
        for i in range(N):
            if i in surv:
                got = rd.shard_bytes_at(plan, held, bufs, lo + j, i).numpy()
                assert (got == full[s, i]).all(), (rank, s, i)
                (data[j, i] if i < K else par[j, i - K])[:] = got
            else:
                assert er[s, i] or plan.kind[lo + j, i] == rd.UNUSED
                (data[j, i] if i < K else par[j, i - K])[:] = 0xEE
    erw = np.ascontiguousarray(er[owned])
    assert oracle.reconstruct_batch(E, K, N, data, par, S, len(owned), erw) == 0
    for j, s in enumerate(owned):
        for i in np.nonzero(erw[j])[0]:
            assert plan.kind[lo + j, i] == rd.OUTPUT
            got = data[j, i] if i < K else par[j, i - K]
            assert (got == full[s, i]).all(), (rank, s, i)


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle
        E, full, er = dataset()
        ids = rd.local_shard_ids(rank, N, world)
        held = torch.from_numpy(np.ascontiguousarray(full[:, ids, :]))
        for chunks in (1, 3):
            plan = rd.plan_exchange(er, K, N, rank, world, S, chunks=chunks)
            bufs = rd.make_buffers([plan], S, "cpu")
            if chunks == 1:
                rd.gather_survivors(held, plan, bufs)
                _check_gathered(plan, held, bufs, full, er, E, rank)
                continue
            # chunk by chunk: each chunk's survivors are in its slot right after its exchange
            for c in range(len(plan.chunks)):
                rd.gather_survivors(held, plan, bufs, chunk=c)
                _check_gathered(plan, held, bufs, full, er, E, rank, chunk=c)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", plan.bytes_in))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), 0))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_gather_and_reconstruct_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def test_gather_single_rank_all_local():
    """N = 1: every survivor is local, nothing moves, and the shard table
    points each survivor at its holder row and each erased shard at its own
    output row (addresses checked by reading them back)."""
    import ctypes
    E, full, er = dataset()
    held = torch.from_numpy(np.ascontiguousarray(full[:, rd.local_shard_ids(0, N, 1), :]))
    plan = rd.plan_exchange(er, K, N, 0, 1, S)
    assert plan.bytes_in == 0 and plan.n_send == 0 and not (plan.kind == rd.REMOTE).any()
    bufs = rd.make_buffers([plan], S, "cpu")
    bufs.out.fill_(0x5A)
    table = rd.shard_table(plan, held, bufs)
    for j, s in enumerate(plan.owned):
        surv = rd.choose_survivors(er[s], K, N)
        for i in range(N):
            if i in surv:
                assert ctypes.string_at(int(table[j, i]), S) == full[s, i].tobytes()
            elif er[s, i]:
                assert ctypes.string_at(int(table[j, i]), S) == b"\x5a" * S
    outs = table[plan.kind == rd.OUTPUT]
    assert len(set(outs.tolist())) == plan.n_out == int(er.sum())
    _check_gathered(plan, held, bufs, full, er, E, 0)


def test_plan_send_recv_orders_agree():
    """What p packs for o, row by row, is what o expects from p at each
    receive-buffer row (same survivor of the same stripe)."""
    _, full, er = dataset()
    world = 3
    plans = [rd.plan_exchange(er, K, N, r, world, S) for r in range(world)]
    for o in range(world):
        po = plans[o]
        for p in range(world):
            if p == o:
                continue
            rows = plans[p].send[o]
            nloc = len(rd.local_shard_ids(p, N, world))
            assert len(rows) == po.recv[p]
            for r, hrow in enumerate(rows):
                s, slot = divmod(int(hrow), nloc)
                i = p + slot * world
                j = po.owned.tolist().index(s)
                assert po.kind[j, i] == rd.REMOTE and po.row[j, i] == po.recv_off[p] + r


class _FakeEvent:
    n = 0

    def __init__(self, enable_timing=False):
        _FakeEvent.n += 1
        self.id = _FakeEvent.n
        self.stream = None

    def record(self, stream):
        self.stream = stream
        stream.log.append(("record", stream.name, self.id))


class _FakeStream:
    def __init__(self, name, log):
        self.name, self.log, self.cuda_stream = name, log, 0

    def wait_event(self, ev):
        self.log.append(("wait", self.name, ev.id))


def test_run_step_orders_slot_reuse_across_steps(monkeypatch):
    """Back-to-back steps with a communication stream (the RCCL path, no
    host sync between steps): every exchange into receive slot s after its
    first use waits for the event recorded after the last reconstruct that
    read slot s -- including step i + 1's first chunks against step i's
    last reconstructs (the write-after-read race of round 3)."""
    import contextlib
    log = []
    comm, compute = _FakeStream("comm", log), _FakeStream("compute", log)
    current = {"s": compute}

    @contextlib.contextmanager
    def fake_stream(st):
        prev, current["s"] = current["s"], st
        yield
        current["s"] = prev

    monkeypatch.setattr(torch.cuda, "Event", _FakeEvent)
    monkeypatch.setattr(torch.cuda, "stream", fake_stream)
    monkeypatch.setattr(rd, "gather_survivors",
                        lambda held, plan, bufs, group, c: log.append(("gather", current["s"].name, c % bufs.slots)))
    monkeypatch.setattr(rd, "reconstruct_owned",
                        lambda fec, plan, table, er, S_, stream, c: log.append(("rec", "compute", c % 2)))
    _, _, er = dataset()
    for chunks in (1, 2, 3, 4):
        log.clear()
        plan = rd.plan_exchange(er, K, N, 0, 2, S, chunks=chunks)
        bufs = rd.GatherBuffers([None] * min(2, chunks), [None] * min(2, chunks), [None])
        for _ in range(3):
            start, end = rd.run_step(None, None, plan, bufs, None, er, S, compute, comm)
            assert start is not None and end is not None
        last_rec_event = {}   # slot -> event recorded after its latest reconstruct
        waited = set()
        pending_slot = None
        for op in log:
            if op[0] == "wait" and op[1] == "comm":
                waited.add(op[2])
            elif op[0] == "gather":
                assert op[1] == "comm"
                slot = op[2]
                if slot in last_rec_event:
                    assert last_rec_event[slot] in waited, (chunks, op, log)
            elif op[0] == "rec":
                pending_slot = op[2] % bufs.slots
            elif op[0] == "record" and op[1] == "compute" and pending_slot is not None:
                last_rec_event[pending_slot] = op[2]
                pending_slot = None
        assert sum(1 for op in log if op[0] == "gather") == 3 * len(plan.chunks)


def test_output_ring_tables_point_at_their_own_buffer():
    """Step i writes output buffer i mod outs: the tables of two steps
    differ only in the erased entries, which lie in different buffers."""
    _, full, er = dataset()
    held = torch.from_numpy(np.ascontiguousarray(full[:, rd.local_shard_ids(0, N, 1), :]))
    plan = rd.plan_exchange(er, K, N, 0, 1, S)
    bufs = rd.make_buffers([plan], S, "cpu", outs=2)
    assert len(bufs.outs) == 2 and bufs.out is bufs.outs[0]
    t0, t1 = rd.shard_table(plan, held, bufs, 0), rd.shard_table(plan, held, bufs, 1)
    out = plan.kind == rd.OUTPUT
    assert (t0[~out] == t1[~out]).all()
    assert (t1[out] - t0[out] == bufs.outs[1].data_ptr() - bufs.outs[0].data_ptr()).all()
    b1 = rd.hbm_budget(STRIPES, 14, S, [plan], N, k=K, outs=1)
    b2 = rd.hbm_budget(STRIPES, 14, S, [plan], N, k=K, outs=2)
    assert abs(b2["out"] - 2 * b1["out"]) < 1e-12
