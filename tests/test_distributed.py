"""Multi-process (gloo, world_size 2 and 3, CPU) tests of the shard-distributed
survivor gather (rsmi/distributed.py): the exchange plan
delivers exactly the k survivors of every owned stripe that Rebuild would
read, and the gathered owner buffers reconstruct the original stripes (the
reconstruct itself is done here by the oracle; on the GPU it is
rs_reconstruct_stripes, covered by tests/test_gpu_parity.py)."""
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
            for peer, rows in p.recv.items():
                for r in rows:
                    got.setdefault((rank, int(r)), []).append(peer)
            for r in p.local_dst:
                got.setdefault((rank, int(r)), []).append(rank)
            # what peers send to `rank` equals what `rank` expects from them
            for peer in range(world):
                if peer == rank:
                    continue
                q = rd.plan_exchange(er, K, N, peer, world, S)
                assert len(q.send[rank]) == len(p.recv[peer])
        want = 0
        for s in range(STRIPES):
            want += K
        assert len(got) == want and all(len(v) == 1 for v in got.values())


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import oracle
        E, full, er = dataset()
        ids = rd.local_shard_ids(rank, N, world)
        held = torch.from_numpy(np.ascontiguousarray(full[:, ids, :]))
        plan = rd.plan_exchange(er, K, N, rank, world, S)
        out = rd.gather_survivors(held, plan, N).numpy()
        owned = plan.owned
        # survivors landed where Rebuild reads them
        for j, s in enumerate(owned):
            for i in rd.choose_survivors(er[s], K, N):
                assert (out[j, i] == full[s, i]).all(), (rank, s, i)
        # reconstruct the owned stripes (oracle stands in for the GPU here)
        data = np.ascontiguousarray(out[:, :K, :])
        par = np.ascontiguousarray(out[:, K:, :])
        erw = np.ascontiguousarray(er[owned])
        for j in range(len(owned)):  # poison the erased slots
            for i in np.nonzero(erw[j])[0]:
                (data[j, i] if i < K else par[j, i - K])[:] = 0xEE
        rc = oracle.reconstruct_batch(E, K, N, data, par, S, len(owned), erw)
        assert rc == 0
        for j, s in enumerate(owned):
            for i in np.nonzero(erw[j])[0]:
                got = data[j, i] if i < K else par[j, i - K]
                assert (got == full[s, i]).all(), (rank, s, i)
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


def test_gather_single_rank_in_place():
    """N = 1: the holder buffer is already the owner layout, so the gather
    moves nothing and returns it (the bench's sharded placement at N = 1)."""
    E, full, er = dataset()
    held = torch.from_numpy(np.ascontiguousarray(full[:, rd.local_shard_ids(0, N, 1), :]))
    plan = rd.plan_exchange(er, K, N, 0, 1, S)
    out = rd.gather_survivors(held, plan, N)
    assert out.data_ptr() == held.data_ptr() and plan.bytes_in == 0
    for j, s in enumerate(plan.owned):
        for i in rd.choose_survivors(er[s], K, N):
            assert (out[j, i].numpy() == full[s, i]).all()
