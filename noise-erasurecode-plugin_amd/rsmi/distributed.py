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
  the erased shards with rs_reconstruct_ptrs.  Traffic per stripe is the
  survivors not already on the owner (about k*S*(G-1)/G bytes), so this
  variant is bound by xGMI, not HBM.

Data path of one exchange (no unpack pass, no per-peer temporaries):
  * sender: the rows a peer needs are packed once into that peer's
    contiguous segment of one reusable send buffer (one gather per peer;
    sending exactly the survivors moves n/k = 1.4x fewer xGMI bytes for
    RS(10,4) than shipping whole holder slices);
  * receiver: each peer's rows land by irecv in a contiguous segment of one
    receive buffer, in the order the plan fixed;
  * reconstruct: a [owned][n] table of device addresses points each survivor
    at its row in the receive buffer (or the local holder buffer) and each
    erased shard at a row of the output buffer; the engine reads and writes
    through it (rs_reconstruct_ptrs), so nothing is copied into an owner
    layout first.

The exchange plan is a pure function of (n, k, G, erasure flags) and is
computed identically on every rank; the erasure map is metadata every peer
knows (the plugin learns it from which Shard messages arrived).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

# Shard table entry kinds ([owned][n] per plan).
LOCAL, REMOTE, OUTPUT, UNUSED = 0, 1, 2, 3


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
    """One rank's part of the survivor gather.

    send[peer]:     rows of this rank's holder buffer ([stripes * nloc, S]
                    view) that `peer` needs, in the order it expects them.
    recv[peer]:     rows this rank receives from `peer`; they occupy rows
                    [recv_off[peer], recv_off[peer] + recv[peer]) of the
                    receive buffer.
    kind/row:       [owned, n] where shard i of owned stripe j is: LOCAL
                    (holder-buffer row), REMOTE (receive-buffer row), OUTPUT
                    (erased: output-buffer row) or UNUSED (present but not
                    read by Rebuild).
    """
    owned: List[int]
    send: Dict[int, np.ndarray]
    recv: Dict[int, int]
    recv_off: Dict[int, int]
    kind: np.ndarray
    row: np.ndarray
    n_recv: int = 0
    n_send: int = 0
    n_out: int = 0
    bytes_in: int = 0
    send_off: Dict[int, int] = field(default_factory=dict)


def plan_exchange(erased: np.ndarray, k: int, n: int, rank: int, world: int,
                  shard_bytes: int) -> ExchangePlan:
    stripes = erased.shape[0]
    nloc = len(local_shard_ids(rank, n, world))
    owned = [s for s in range(stripes) if owner(s, world) == rank]
    send: Dict[int, List[int]] = {p: [] for p in range(world) if p != rank}
    recv_rows: Dict[int, List[tuple]] = {p: [] for p in range(world) if p != rank}
    kind = np.full((len(owned), n), UNUSED, dtype=np.int8)
    row = np.zeros((len(owned), n), dtype=np.int64)
    n_out = 0
    opos = {s: j for j, s in enumerate(owned)}
    for s in range(stripes):
        o = owner(s, world)
        surv = choose_survivors(erased[s], k, n)
        if o == rank:
            j = opos[s]
            for i in range(n):
                if erased[s, i]:
                    kind[j, i] = OUTPUT
                    row[j, i] = n_out
                    n_out += 1
        for i in surv:
            hd = holder(i, world)
            if hd == rank and o == rank:
                kind[opos[s], i] = LOCAL
                row[opos[s], i] = s * nloc + i // world
            elif hd == rank:
                send[o].append(s * nloc + i // world)
            elif o == rank:
                recv_rows[hd].append((opos[s], i))
    recv: Dict[int, int] = {}
    recv_off: Dict[int, int] = {}
    off = 0
    for p in sorted(recv_rows):
        recv_off[p] = off
        for r, (j, i) in enumerate(recv_rows[p]):
            kind[j, i] = REMOTE
            row[j, i] = off + r
        recv[p] = len(recv_rows[p])
        off += recv[p]
    send_off: Dict[int, int] = {}
    soff = 0
    for p in sorted(send):
        send_off[p] = soff
        soff += len(send[p])
    return ExchangePlan(owned, {p: np.asarray(v, dtype=np.int64) for p, v in send.items()}, recv, recv_off,
                        kind, row, n_recv=off, n_send=soff, n_out=n_out, bytes_in=off * shard_bytes,
                        send_off=send_off)


@dataclass
class GatherBuffers:
    """Reusable per-rank buffers of the exchange (allocate once, pass to
    every step): send [rows, S], receive [rows, S], output [rows, S]."""
    send: object
    recv: object
    out: object


def make_buffers(plans: Sequence[ExchangePlan], shard_bytes: int, device) -> GatherBuffers:
    import torch
    mk = lambda rows: torch.empty((max(rows, 1), shard_bytes), dtype=torch.uint8, device=device)
    return GatherBuffers(mk(max(p.n_send for p in plans)), mk(max(p.n_recv for p in plans)),
                         mk(max(p.n_out for p in plans)))


def shard_table(plan: ExchangePlan, held, bufs: GatherBuffers) -> np.ndarray:
    """[owned, n] int64 device addresses for rs_reconstruct_ptrs: every
    survivor where it lies, every erased shard at its output row."""
    S = held.shape[-1]
    base = {LOCAL: held.data_ptr(), REMOTE: bufs.recv.data_ptr(), OUTPUT: bufs.out.data_ptr(),
            UNUSED: held.data_ptr()}
    t = np.empty(plan.kind.shape, dtype=np.int64)
    for kd, b in base.items():
        m = plan.kind == kd
        t[m] = b + plan.row[m] * S if kd != UNUSED else b
    return t


def gather_survivors(held, plan: ExchangePlan, bufs: GatherBuffers, group=None):
    """Runs the exchange: packs what each peer needs into its segment of
    bufs.send, and receives every peer's rows into bufs.recv (contiguous
    segments in plan.recv_off order).  `held` is this rank's holder buffer, a
    [stripes, nloc, S] uint8 tensor.  One batch_isend_irecv: RCCL groups it
    into a single ncclGroupStart/End of point-to-point sends and receives."""
    import torch
    import torch.distributed as dist

    stripes, nloc, S = held.shape
    flat = held.view(stripes * nloc, S)
    dev = held.device
    # gloo (CPU tests, and the bench's one-GPU rehearsal of N ranks) moves
    # host tensors only: device segments are staged through host copies.
    staged = held.is_cuda and dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "gloo"
    ops, landing = [], []
    for p, rows in sorted(plan.send.items()):
        if len(rows):
            seg = bufs.send[plan.send_off[p]:plan.send_off[p] + len(rows)]
            torch.index_select(flat, 0, torch.from_numpy(rows).to(dev, non_blocking=True), out=seg)
            ops.append(dist.P2POp(dist.isend, seg.cpu() if staged else seg, p, group))
    for p, cnt in sorted(plan.recv.items()):
        if cnt:
            seg = bufs.recv[plan.recv_off[p]:plan.recv_off[p] + cnt]
            tgt = torch.empty(seg.shape, dtype=seg.dtype) if staged else seg
            if staged:
                landing.append((seg, tgt))
            ops.append(dist.P2POp(dist.irecv, tgt, p, group))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    for r in reqs:
        r.wait()
    for seg, tgt in landing:
        seg.copy_(tgt)
    return bufs


def reconstruct_owned(fec, plan: ExchangePlan, table_dev, erased_owned: np.ndarray, shard_bytes: int,
                      stream: int = 0) -> None:
    """Regenerates the erased shards of the owned stripes into bufs.out
    through the shard table (a device int64 tensor from shard_table)."""
    fec.reconstruct_ptrs(table_dev.data_ptr(), shard_bytes, len(plan.owned),
                         np.ascontiguousarray(erased_owned, dtype=np.uint8).tobytes(), stream)


def shard_bytes_at(plan: ExchangePlan, held, bufs: GatherBuffers, j: int, i: int):
    """The bytes of shard i of owned stripe j as the reconstruct sees them
    (tests)."""
    kd, r = int(plan.kind[j, i]), int(plan.row[j, i])
    S = held.shape[-1]
    if kd == LOCAL:
        return held.reshape(-1, S)[r]
    if kd == REMOTE:
        return bufs.recv[r]
    if kd == OUTPUT:
        return bufs.out[r]
    return None
