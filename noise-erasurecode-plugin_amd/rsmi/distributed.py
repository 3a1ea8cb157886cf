"""Multi-GPU placement of the shard path.

Two placements:

* stripe-local (the default and the bench headline): stripe s lives entirely
  on rank s mod G; encode and reconstruct are local, no collective.
* shard-distributed (the p2p analogue of "shards spread over peers",
  main.go:207 broadcasts every shard to every peer): shard i of every stripe
  is held by rank i mod G.  To reconstruct stripe s its owner (rank s mod G)
  gathers the k survivors it will read -- chosen with infectious Rebuild's
  rule, the same rule the engine applies -- from their holders in ONE grouped
  point-to-point exchange (torch.distributed batch_isend_irecv = RCCL
  ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd over xGMI), then regenerates
  the erased shards locally with rs_reconstruct_stripes.  Traffic per stripe
  is the survivors not already on the owner (about k*S*(G-1)/G bytes), so
  this variant is bound by xGMI, not HBM.

The exchange plan is a pure function of (n, k, G, erasure flags) and is
computed identically on every rank; the erasure map is metadata every peer
knows (the plugin learns it from which Shard messages arrived).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np


def choose_survivors(erased_row: Sequence[int], k: int, n: int) -> List[int]:
    """infectious Rebuild's choice (restated in csrc/gf256.cpp
    choose_survivors): slot i takes shard i if present, otherwise the
    highest-numbered present shard not yet used."""
    present = [not erased_row[i] for i in range(n)]
    used = [False] * n
    out: List[int] = []
    hi = n - 1
    for i in range(k):
        if present[i] and not used[i]:
            out.append(i)
            used[i] = True
            continue
        while hi >= 0 and (not present[hi] or used[hi]):
            hi -= 1
        if hi < 0:
            raise ValueError("not enough shares")
        out.append(hi)
        used[hi] = True
    return out


def holder(shard_id: int, world: int) -> int:
    return shard_id % world


def owner(stripe: int, world: int) -> int:
    return stripe % world


def local_shard_ids(rank: int, n: int, world: int) -> List[int]:
    """Shard ids held by `rank` (its slot j holds id rank + j*G)."""
    return list(range(rank, n, world))


@dataclass
class ExchangePlan:
    """Row indices for one rank's part of the survivor gather.

    send[peer]: rows of this rank's holder buffer ([stripes * nloc, S] view)
                to send to `peer`, in order.
    recv[peer]: rows of this rank's owner buffer ([owned * n, S] view) that
                the data received from `peer` lands in, in the same order.
    local_src/local_dst: survivors this rank both holds and owns.
    """
    owned: List[int]
    send: Dict[int, np.ndarray]
    recv: Dict[int, np.ndarray]
    local_src: np.ndarray
    local_dst: np.ndarray
    bytes_in: int = 0


def plan_exchange(erased: np.ndarray, k: int, n: int, rank: int, world: int,
                  shard_bytes: int) -> ExchangePlan:
    stripes = erased.shape[0]
    nloc = len(local_shard_ids(rank, n, world))
    owned = [s for s in range(stripes) if owner(s, world) == rank]
    opos = {s: j for j, s in enumerate(owned)}
    send: Dict[int, List[int]] = {p: [] for p in range(world) if p != rank}
    recv: Dict[int, List[int]] = {p: [] for p in range(world) if p != rank}
    lsrc: List[int] = []
    ldst: List[int] = []
    for s in range(stripes):
        o = owner(s, world)
        for i in choose_survivors(erased[s], k, n):
            hd = holder(i, world)
            if hd == rank and o == rank:
                lsrc.append(s * nloc + i // world)
                ldst.append(opos[s] * n + i)
            elif hd == rank:
                send[o].append(s * nloc + i // world)
            elif o == rank:
                recv[hd].append(opos[s] * n + i)
    as_arr = lambda d: {p: np.asarray(v, dtype=np.int64) for p, v in d.items()}
    rb = sum(len(v) for v in recv.values()) * shard_bytes
    return ExchangePlan(owned, as_arr(send), as_arr(recv), np.asarray(lsrc, dtype=np.int64),
                        np.asarray(ldst, dtype=np.int64), rb)


def gather_survivors(held, plan: ExchangePlan, n: int, group=None):
    """Runs the exchange.  `held` is this rank's holder buffer, a
    [stripes, nloc, S] uint8 tensor; returns the owner buffer [owned, n, S]
    with every survivor of every owned stripe in place (other slots
    undefined).  One batch_isend_irecv: RCCL groups it into a single
    ncclGroupStart/End of point-to-point sends and receives."""
    import torch
    import torch.distributed as dist

    stripes, nloc, S = held.shape
    if (nloc == n and len(plan.owned) == stripes and not any(len(r) for r in plan.send.values())
            and not any(len(r) for r in plan.recv.values())
            and np.array_equal(plan.local_src, plan.local_dst)):
        # One rank holds and owns everything in the owner layout already
        # (N = 1): the survivors are in place, nothing moves.
        return held
    flat = held.reshape(stripes * nloc, S)
    out = torch.empty((len(plan.owned), n, S), dtype=held.dtype, device=held.device)
    oflat = out.view(len(plan.owned) * n, S)
    dev = held.device
    ops = []
    recv_bufs = {}
    for p, rows in plan.send.items():
        if len(rows):
            buf = flat.index_select(0, torch.from_numpy(rows).to(dev))
            ops.append(dist.P2POp(dist.isend, buf, p, group))
    for p, rows in plan.recv.items():
        if len(rows):
            recv_bufs[p] = torch.empty((len(rows), S), dtype=held.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, recv_bufs[p], p, group))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    if len(plan.local_src):
        oflat.index_copy_(0, torch.from_numpy(plan.local_dst).to(dev),
                          flat.index_select(0, torch.from_numpy(plan.local_src).to(dev)))
    for r in reqs:
        r.wait()
    for p, buf in recv_bufs.items():
        oflat.index_copy_(0, torch.from_numpy(plan.recv[p]).to(dev), buf)
    return out


def reconstruct_owned(fec, owned_buf, erased_owned: np.ndarray, stream: int = 0) -> None:
    """Regenerates the erased shards of the owner buffer [owned, n, S] in
    place with the engine (data region = slots 0..k-1, parity = k..n-1)."""
    stripes, n, S = owned_buf.shape
    k = fec.k
    base = owned_buf.data_ptr()
    fec.reconstruct_stripes(base, n * S, base + k * S, n * S, S, S, stripes,
                            np.ascontiguousarray(erased_owned, dtype=np.uint8).tobytes(), stream)
