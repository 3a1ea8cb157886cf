"""Multi-GPU placement of the shard path.

Two placements:

* stripe-local (the default and the bench headline): stripe s lives entirely
  on rank s mod G; encode and reconstruct are local, no collective.
* shard-distributed (the p2p analogue of "shards spread over peers",
  main.go:207 broadcasts every shard to every peer): shard i of every stripe
  is held by rank i mod G.  To reconstruct stripe s its owner (rank s mod G)
  gathers the k survivors it will read -- chosen with infectious Rebuild's
  rule, the same rule the engine applies -- from their holders in grouped
  point-to-point exchanges (torch.distributed batch_isend_irecv = RCCL
  ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd over xGMI), then regenerates
  the erased shards with rs_reconstruct_ptrs.  Traffic per stripe is the
  survivors not already on the owner (about k*S*(G-1)/G bytes), so this
  variant is bound by xGMI, not HBM.

Data path of one step (no unpack pass, no per-peer temporaries):
  * the owned stripes are split into chunks (global stripe ranges, so every
    rank agrees on them); chunk c's exchange uses send/receive slot c mod 2,
    so two chunks' buffers are live at a time, not a whole step's;
  * sender: the rows a peer needs are packed once into that peer's
    contiguous segment of the slot's send buffer (one gather per peer;
    sending exactly the survivors moves n/k = 1.4x fewer xGMI bytes for
    RS(10,4) than shipping whole holder slices);
  * receiver: each peer's rows land by irecv in a contiguous segment of the
    slot's receive buffer, in the order the plan fixed;
  * reconstruct: a [owned][n] table of device addresses points each survivor
    at its row in the receive slot (or the local holder buffer) and each
    erased shard at a row of the output buffer; the engine reads and writes
    through it (rs_reconstruct_ptrs), so nothing is copied into an owner
    layout first.  With RCCL, chunk c + 1's exchange (a communication
    stream) overlaps chunk c's reconstruct (the compute stream).

The exchange plan is a pure function of (n, k, G, erasure flags, chunks),
computed identically on every rank with numpy (vectorised over stripes); the
erasure map is metadata every peer knows (the plugin learns it from which
Shard messages arrived).
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


def survivor_mask(erased: np.ndarray, k: int, n: int) -> np.ndarray:
    """[stripes, n] bool: the shards Rebuild reads, for every stripe at once.

    Every present data shard keeps its own slot; the d erased data slots are
    filled from the top down, and every parity id exceeds every data id, so
    they take the d highest-numbered present parity shards."""
    present = np.asarray(erased)[:, :n] == 0
    d = (~present[:, :k]).sum(axis=1)
    par = present[:, k:]
    higher = np.cumsum(par[:, ::-1], axis=1)[:, ::-1] - par  # present parity with a larger id
    use_par = par & (higher < d[:, None])
    if (use_par.sum(axis=1) != d).any():
        raise ValueError("not enough shares")
    return np.concatenate([present[:, :k], use_par], axis=1)


def holder(shard_id: int, world: int) -> int:
    return shard_id % world


def owner(stripe: int, world: int) -> int:
    return stripe % world


def local_shard_ids(rank: int, n: int, world: int) -> List[int]:
    """Shard ids held by `rank` (its slot j holds id rank + j*G)."""
    return list(range(rank, n, world))


@dataclass
class ChunkPlan:
    """One chunk's exchange: owned stripes [lo, hi) of the plan (a global
    stripe range).  send[peer] are rows of this rank's holder buffer
    ([stripes * nloc, S] view) that `peer` needs, packed at send_off[peer]
    of the slot's send buffer; recv[peer] rows arrive from `peer` at rows
    [recv_off[peer], recv_off[peer] + recv[peer]) of the slot's receive
    buffer."""
    lo: int
    hi: int
    send: Dict[int, np.ndarray]
    send_off: Dict[int, int]
    recv: Dict[int, int]
    recv_off: Dict[int, int]
    n_send: int
    n_recv: int


@dataclass
class ExchangePlan:
    """One rank's part of the survivor gather of one step.

    owned:     global ids of the stripes this rank owns (ascending).
    kind/row:  [owned, n] where shard i of owned stripe j is LOCAL
               (holder-buffer row), REMOTE (row of its chunk's receive
               slot), OUTPUT (erased: output-buffer row) or UNUSED (present
               but not read by Rebuild).
    chunks:    the exchanges, in order; chunk c uses buffer slot c mod slots.
    """
    owned: np.ndarray
    kind: np.ndarray
    row: np.ndarray
    chunks: List[ChunkPlan]
    n_out: int = 0
    bytes_in: int = 0

    def _one(self) -> ChunkPlan:
        if len(self.chunks) != 1:
            raise ValueError("plan has several chunks: use plan.chunks[c]")
        return self.chunks[0]

    # Single-chunk views (the whole step in one exchange).
    send = property(lambda self: self._one().send)
    send_off = property(lambda self: self._one().send_off)
    recv = property(lambda self: self._one().recv)
    recv_off = property(lambda self: self._one().recv_off)
    n_send = property(lambda self: sum(c.n_send for c in self.chunks))
    n_recv = property(lambda self: sum(c.n_recv for c in self.chunks))

    def chunk_of(self, j: int) -> int:
        for c, ch in enumerate(self.chunks):
            if ch.lo <= j < ch.hi:
                return c
        raise IndexError(j)


def chunk_bounds(stripes: int, chunks: int) -> np.ndarray:
    """Global stripe ranges of the chunks: chunk c = [b[c], b[c+1])."""
    chunks = max(1, min(chunks, max(stripes, 1)))
    return (np.arange(chunks + 1, dtype=np.int64) * stripes) // chunks


def _segments(keys: np.ndarray, nkeys: int):
    """(counts, starts) of a sorted key array over 0..nkeys-1."""
    counts = np.bincount(keys, minlength=nkeys) if len(keys) else np.zeros(nkeys, dtype=np.int64)
    starts = np.zeros(nkeys, dtype=np.int64)
    np.cumsum(counts[:-1], out=starts[1:])
    return counts, starts


def plan_exchange(erased: np.ndarray, k: int, n: int, rank: int, world: int, shard_bytes: int,
                  chunks: int = 1) -> ExchangePlan:
    """The exchange plan of one step for `rank`, vectorised over stripes.
    Within a chunk, rows for one peer are ordered by (stripe, shard id) on
    both sides, so what p packs for o is what o expects from p."""
    erased = np.asarray(erased)
    G = erased.shape[0]
    used = survivor_mask(erased, k, n)
    ids = np.arange(n)
    hold = ids % world
    slot = ids // world
    nloc = len(local_shard_ids(rank, n, world))
    bounds = chunk_bounds(G, chunks)
    C = len(bounds) - 1
    chunk_of_stripe = np.searchsorted(bounds, np.arange(G), side="right") - 1
    owned = np.arange(rank, G, world, dtype=np.int64)
    er_own = erased[owned, :n] != 0
    used_own = used[owned]
    kind = np.full((len(owned), n), UNUSED, dtype=np.int8)
    row = np.zeros((len(owned), n), dtype=np.int64)
    # erased shards: output rows in (owned stripe, shard id) order
    kind[er_own] = OUTPUT
    n_out = int(er_own.sum())
    row[er_own] = np.arange(n_out, dtype=np.int64)
    # survivors held here
    loc = used_own & (hold == rank)[None, :]
    kind[loc] = LOCAL
    row[loc] = (owned[:, None] * nloc + slot[None, :])[loc]
    # survivors held by peers: receive rows, chunk by chunk, peer segments
    rem = used_own & (hold != rank)[None, :]
    kind[rem] = REMOTE
    J, I = np.nonzero(rem)  # row-major: (owned stripe, shard id) ascending
    rc = chunk_of_stripe[owned[J]]
    rp = hold[I]
    order = np.lexsort((rp, rc))  # stable: (stripe, id) order kept inside (chunk, peer)
    rcs, rps = rc[order], rp[order]
    _, cstart = _segments(rcs, C)
    pos = np.arange(len(order), dtype=np.int64) - cstart[rcs]
    row[J[order], I[order]] = pos
    # rows this rank sends: survivors it holds of stripes owned elsewhere
    mine = ids[hold == rank]
    sub = used[:, mine]
    sub[np.arange(G) % world == rank, :] = False
    S_, M_ = np.nonzero(sub)  # (stripe, id) ascending
    sdst = S_ % world
    sc = chunk_of_stripe[S_]
    srow = S_.astype(np.int64) * nloc + slot[mine[M_]]
    sorder = np.lexsort((sdst, sc))
    sdst, sc, srow = sdst[sorder], sc[sorder], srow[sorder]
    peers = [p for p in range(world) if p != rank]
    plans: List[ChunkPlan] = []
    o_lo = np.searchsorted(owned, bounds, side="left")
    for c in range(C):
        rsel = rcs == c
        send: Dict[int, np.ndarray] = {}
        send_off: Dict[int, int] = {}
        recv: Dict[int, int] = {}
        recv_off: Dict[int, int] = {}
        cs = np.nonzero(sc == c)[0]
        soff = 0
        roff = 0
        rcnt = np.bincount(rps[rsel], minlength=world)
        for p in peers:
            sel = cs[sdst[cs] == p]
            send[p] = srow[sel]
            send_off[p] = soff
            soff += len(sel)
            recv_off[p] = roff
            recv[p] = int(rcnt[p])
            roff += recv[p]
        plans.append(ChunkPlan(int(o_lo[c]), int(o_lo[c + 1]), send, send_off, recv, recv_off, soff, roff))
    return ExchangePlan(owned, kind, row, plans, n_out=n_out, bytes_in=int(rem.sum()) * shard_bytes)


# -------------------------------------------------------------- memory ----
def hbm_budget(gstripes: int, nloc: int, shard_bytes: int, plans: Sequence[ExchangePlan], n: int,
               slots: int = 2, setup_batch: int = 64, k: int = 0, outs: int = 1) -> Dict[str, float]:
    """Per-rank device bytes of the shard-distributed step (GB), computed
    before anything is allocated: the holder buffer, the send / receive
    slots (sized by the largest chunk of any step), the `outs` output
    buffers (each sized by the largest step), the shard tables and the setup
    batch."""
    S = shard_bytes
    send = max((c.n_send for p in plans for c in p.chunks), default=0)
    recv = max((c.n_recv for p in plans for c in p.chunks), default=0)
    out = max((p.n_out for p in plans), default=0)
    owned = max((len(p.owned) for p in plans), default=0)
    nslots = min(slots, max(len(p.chunks) for p in plans)) if plans else 1
    b = {
        "held": gstripes * nloc * S,
        "send": nslots * max(send, 1) * S,
        "recv": nslots * max(recv, 1) * S,
        "out": max(1, outs) * max(out, 1) * S,
        "tables": owned * n * 8 * 2,
        "setup": setup_batch * max(k, 1) * S * 2,
    }
    gb = {key: v / 1e9 for key, v in b.items()}
    gb["total"] = sum(b.values()) / 1e9
    return gb


@dataclass
class GatherBuffers:
    """Reusable per-rank buffers of the exchange (allocate once, pass to
    every step): `slots` send and receive buffers [rows, S] (chunk c uses
    slot c mod slots) and a ring of output buffers [rows, S] (step i of a
    run writes outs[i mod len(outs)], so the last len(outs) steps' outputs
    survive the run and can be checked).

    slot_free[s] is the compute-stream event after the last reconstruct that
    read receive slot s (None: free).  It is carried from step to step:
    the next exchange into slot s -- in this step or the next one -- waits
    for it on the communication stream, so a receive never overwrites
    survivors a queued reconstruct has yet to read."""
    send: List[object]
    recv: List[object]
    outs: List[object]
    slot_free: List[object] = field(default_factory=list)

    def __post_init__(self):
        if not self.slot_free:
            self.slot_free = [None] * len(self.recv)

    @property
    def slots(self) -> int:
        return len(self.recv)

    @property
    def out(self):
        return self.outs[0]


def make_buffers(plans: Sequence[ExchangePlan], shard_bytes: int, device, slots: int = 2,
                 outs: int = 1) -> GatherBuffers:
    """Buffers sized for the largest chunk and the largest step of `plans`,
    with `outs` output buffers.  Shard rows must stay 16-byte aligned for
    the engine's vector loads, so shard_bytes must be a multiple of 16."""
    import torch
    if shard_bytes % 16:
        raise ValueError(f"shard_bytes {shard_bytes} is not a multiple of 16 (the kernels load 16-byte vectors)")
    nslots = max(1, min(slots, max(len(p.chunks) for p in plans)))
    mk = lambda rows: torch.empty((max(rows, 1), shard_bytes), dtype=torch.uint8, device=device)
    send = max(c.n_send for p in plans for c in p.chunks)
    recv = max(c.n_recv for p in plans for c in p.chunks)
    n_out = max(p.n_out for p in plans)
    return GatherBuffers([mk(send) for _ in range(nslots)], [mk(recv) for _ in range(nslots)],
                         [mk(n_out) for _ in range(max(1, outs))])


def shard_table(plan: ExchangePlan, held, bufs: GatherBuffers, out: int = 0) -> np.ndarray:
    """[owned, n] int64 device addresses for rs_reconstruct_ptrs: every
    survivor where it lies (its chunk's receive slot for REMOTE), every
    erased shard at its row of output buffer `out`."""
    S = held.shape[-1]
    if S % 16:
        raise ValueError(f"shard bytes {S} is not a multiple of 16")
    t = np.empty(plan.kind.shape, dtype=np.int64)
    m = plan.kind == LOCAL
    t[m] = held.data_ptr() + plan.row[m] * S
    m = plan.kind == OUTPUT
    t[m] = bufs.outs[out].data_ptr() + plan.row[m] * S
    t[plan.kind == UNUSED] = held.data_ptr()
    for c, ch in enumerate(plan.chunks):
        blk = slice(ch.lo, ch.hi)
        m = plan.kind[blk] == REMOTE
        tb = t[blk]
        tb[m] = bufs.recv[c % bufs.slots].data_ptr() + plan.row[blk][m] * S
    return t


def gather_survivors(held, plan: ExchangePlan, bufs: GatherBuffers, group=None, chunk: int = 0):
    """Runs chunk `chunk`'s exchange: packs what each peer needs into its
    segment of the slot's send buffer, and receives every peer's rows into
    the slot's receive buffer (contiguous segments in recv_off order).
    `held` is this rank's holder buffer, a [stripes, nloc, S] uint8 tensor.
    One batch_isend_irecv: RCCL groups it into a single ncclGroupStart/End
    of point-to-point sends and receives.  Issued on the current stream; the
    waits make the current stream wait for the transfers (RCCL), so the
    caller orders the reconstruct after it with an event."""
    import torch
    import torch.distributed as dist

    ch = plan.chunks[chunk]
    stripes, nloc, S = held.shape
    flat = held.view(stripes * nloc, S)
    dev = held.device
    sbuf = bufs.send[chunk % bufs.slots]
    rbuf = bufs.recv[chunk % bufs.slots]
    # gloo (CPU tests, and the bench's one-GPU rehearsal of N ranks) moves
    # host tensors only: device segments are staged through host copies.
    staged = held.is_cuda and dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "gloo"
    ops, landing = [], []
    for p, rows in sorted(ch.send.items()):
        if len(rows):
            seg = sbuf[ch.send_off[p]:ch.send_off[p] + len(rows)]
            idx = torch.from_numpy(rows)
            if held.is_cuda:
                idx = idx.pin_memory().to(dev, non_blocking=True)
            torch.index_select(flat, 0, idx, out=seg)
            ops.append(dist.P2POp(dist.isend, seg.cpu() if staged else seg, p, group))
    for p, cnt in sorted(ch.recv.items()):
        if cnt:
            seg = rbuf[ch.recv_off[p]:ch.recv_off[p] + cnt]
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
                      stream: int = 0, chunk: Optional[int] = None) -> None:
    """Regenerates the erased shards of the owned stripes (all, or one
    chunk's) into the output buffer the shard table (a device int64 tensor
    from shard_table) points at."""
    n = plan.kind.shape[1]
    lo, hi = (0, len(plan.owned)) if chunk is None else (plan.chunks[chunk].lo, plan.chunks[chunk].hi)
    if hi <= lo:
        return
    er = np.ascontiguousarray(np.asarray(erased_owned)[lo:hi], dtype=np.uint8)
    fec.reconstruct_ptrs(table_dev.data_ptr() + lo * n * 8, shard_bytes, hi - lo, er.tobytes(), stream)


def run_step(fec, held, plan: ExchangePlan, bufs: GatherBuffers, table_dev, erased_owned: np.ndarray,
             shard_bytes: int, compute_stream, comm_stream=None, group=None):
    """One pipelined step: chunk c's exchange on comm_stream, its
    reconstruct on compute_stream after the exchange's event.  Before an
    exchange lands in receive slot s, comm_stream waits for bufs.slot_free[s]
    -- the reconstruct that last read slot s, in this step or in the step
    before (steps are queued back to back with no host sync, so without the
    carried event step i + 1's first receives would overwrite survivors that
    step i's last reconstructs still read).  Without a comm stream the
    chunks run one after the other on the current stream.

    Returns (start, end): compute-stream events recorded before the step's
    first reconstruct is queued and after its last one (None, None without a
    comm stream)."""
    import torch
    slots = bufs.slots
    if comm_stream is None:
        for c in range(len(plan.chunks)):
            gather_survivors(held, plan, bufs, group, c)
            reconstruct_owned(fec, plan, table_dev, erased_owned, shard_bytes, compute_stream.cuda_stream, c)
        return None, None
    start = torch.cuda.Event(enable_timing=True)
    start.record(compute_stream)
    for c in range(len(plan.chunks)):
        slot = c % slots
        if bufs.slot_free[slot] is not None:
            comm_stream.wait_event(bufs.slot_free[slot])
        with torch.cuda.stream(comm_stream):
            gather_survivors(held, plan, bufs, group, c)
            got = torch.cuda.Event()
            got.record(comm_stream)
        compute_stream.wait_event(got)
        reconstruct_owned(fec, plan, table_dev, erased_owned, shard_bytes, compute_stream.cuda_stream, c)
        ev = torch.cuda.Event()
        ev.record(compute_stream)
        bufs.slot_free[slot] = ev
    end = torch.cuda.Event(enable_timing=True)
    end.record(compute_stream)
    return start, end


def shard_bytes_at(plan: ExchangePlan, held, bufs: GatherBuffers, j: int, i: int):
    """The bytes of shard i of owned stripe j as the reconstruct sees them
    (tests)."""
    kd, r = int(plan.kind[j, i]), int(plan.row[j, i])
    S = held.shape[-1]
    if kd == LOCAL:
        return held.reshape(-1, S)[r]
    if kd == REMOTE:
        return bufs.recv[plan.chunk_of(j) % bufs.slots][r]
    if kd == OUTPUT:
        return bufs.out[r]
    return None
