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


def test_plan_covers_each_survivor_once():
    _, _, er = dataset()
    for world in (1, 2, 3, 4, 8):
        got = {}
        for rank in range(world):
            p = rd.plan_exchange(er, K, N, rank, world, S)
            for j in range(len(p.owned)):
                for i in range(N):
                    if p.kind[j, i] in (rd.LOCAL, rd.REMOTE):
                        got.setdefault((rank, j, i), []).append(int(p.kind[j, i]))
            # what peers send to `rank` equals what `rank` expects from them
            for peer in range(world):
                if peer == rank:
                    continue
                q = rd.plan_exchange(er, K, N, peer, world, S)
                assert len(q.send[rank]) == p.recv[peer]
        want = 0
        for s in range(STRIPES):
            want += K
        assert len(got) == want and all(len(v) == 1 for v in got.values())


def _check_gathered(plan, held, bufs, full, er, E, rank):
    """Every survivor Rebuild reads is where the shard table says; the
    erased shards, reconstructed (by the oracle here; by rs_reconstruct_ptrs
    on the GPU) from exactly those bytes, equal the originals."""
    from oracle import oracle
    owned = plan.owned
    data = np.zeros((len(owned), K, S), dtype=np.uint8)
    par = np.zeros((len(owned), N - K, S), dtype=np.uint8)
    for j, s in enumerate(owned):
        surv = rd.choose_survivors(er[s], K, N)
        for i in range(N):
            if i in surv:
                got = rd.shard_bytes_at(plan, held, bufs, j, i).numpy()
                assert (got == full[s, i]).all(), (rank, s, i)
                (data[j, i] if i < K else par[j, i - K])[:] = got
            else:
                assert er[s, i] or plan.kind[j, i] == rd.UNUSED
                (data[j, i] if i < K else par[j, i - K])[:] = 0xEE
    erw = np.ascontiguousarray(er[owned])
    assert oracle.reconstruct_batch(E, K, N, data, par, S, len(owned), erw) == 0
    for j, s in enumerate(owned):
        for i in np.nonzero(erw[j])[0]:
            assert plan.kind[j, i] == rd.OUTPUT
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
        plan = rd.plan_exchange(er, K, N, rank, world, S)
        bufs = rd.make_buffers([plan], S, "cpu")
        rd.gather_survivors(held, plan, bufs)
        _check_gathered(plan, held, bufs, full, er, E, rank)
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
                j = po.owned.index(s)
                assert po.kind[j, i] == rd.REMOTE and po.row[j, i] == po.recv_off[p] + r
