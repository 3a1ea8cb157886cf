"""Zero-copy receive: survivors that lie in
engine-pinned memory (rs_arena / rs_pinned_alloc) are read in place over
PCIe by rs_decode_batch's reconstruct kernel -- no staging memcpy, no H2D of
survivors.  The reference copies ShardData at Unmarshal (shard.pb.go:468-503)
and DeepCopies every share (main.go:255-258); rs_shard_unmarshal_arena makes
that one copy land in an aligned arena slot.  Results are checked bit-exact
against the oracle and against the staged path."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402


def _messages(k, n, S, B, seed):
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(seed)
    msgs = []
    for b in range(B):
        data = oracle.splitmix_bytes(k * S, seed * 1000 + b).tobytes()
        par = oracle.encode(E, k, n, data)
        sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
        keep = sorted(rng.choice(n, size=k, replace=False).tolist())
        msgs.append((data, sh, keep))
    return msgs


def _decode_batch(f, msgs, ptr_of):
    lib = rsmi.load()
    k = f.k
    S = len(msgs[0][1][0])
    B = len(msgs)
    counts = (ctypes.c_int * B)(*[k] * B)
    nums = (ctypes.c_int * (B * k))(*[i for _, _, keep in msgs for i in keep])
    ptrs = (ctypes.c_void_p * (B * k))(*[ptr_of(b, i) for b, (_, _, keep) in enumerate(msgs) for i in keep])
    outs = [ctypes.create_string_buffer(k * S) for _ in range(B)]
    dsts = (ctypes.c_void_p * B)(*[ctypes.addressof(o) for o in outs])
    st = (ctypes.c_int * B)()
    rc = lib.rs_decode_batch(f.handle, B, counts, nums, ptrs, S, dsts, st)
    return rc, [o.raw for o in outs], list(st)


@pytest.mark.parametrize("k,n,S,B", [(10, 14, 104858, 24), (10, 14, 6554, 200), (64, 80, 4099, 12),
                                     (4, 6, 17, 50)])
def test_decode_batch_reads_arena_survivors_in_place(k, n, S, B):
    f = rsmi.FEC(k, n)
    msgs = _messages(k, n, S, B, k + S)
    arena = rsmi.Arena(B * n * ((S + 255) // 256 * 256) + 4096)
    addr = {}
    for b, (_, sh, keep) in enumerate(msgs):
        for i in keep:
            addr[(b, i)] = arena.put(sh[i])
    rc, outs, st = _decode_batch(f, msgs, lambda b, i: addr[(b, i)])
    assert rc == 0 and st == [0] * B
    assert f.stat(f.STAT_BATCHES_IN_PLACE) == 1 and f.stat(f.STAT_BATCHES_STAGED) == 0
    E = oracle.fec_matrix(k, n)
    for (data, sh, keep), o in zip(msgs, outs):
        rc2, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep])
        assert rc2 == 0 and o == ref == data
    # a survivor outside engine-pinned memory: the whole batch is staged
    keepalive = [bytes(msgs[0][1][msgs[0][2][0]])]
    ptr = ctypes.cast(ctypes.c_char_p(keepalive[0]), ctypes.c_void_p).value
    rc, outs2, st = _decode_batch(f, msgs, lambda b, i: ptr if (b, i) == (0, msgs[0][2][0]) else addr[(b, i)])
    assert rc == 0 and outs2 == outs and f.stat(f.STAT_BATCHES_STAGED) == 1
    arena.free()
    f.close()


def test_unaligned_pinned_survivor_is_staged():
    """Pinned but not 16-byte aligned (a ShardData view inside a marshalled
    message): staged, still exact."""
    k, n, S, B = 10, 14, 1000, 8
    f = rsmi.FEC(k, n)
    msgs = _messages(k, n, S, B, 5)
    arena = rsmi.Arena(B * n * 2048)
    addr = {(b, i): arena.put(b"\0" * 3 + sh[i]) + 3 for b, (_, sh, keep) in enumerate(msgs) for i in keep}
    rc, outs, st = _decode_batch(f, msgs, lambda b, i: addr[(b, i)])
    assert rc == 0 and all(o == d for o, (d, _, _) in zip(outs, msgs))
    assert f.stat(f.STAT_BATCHES_STAGED) == 1 and f.stat(f.STAT_BATCHES_IN_PLACE) == 0
    arena.free()
    f.close()


def test_unmarshal_into_arena_then_decode_in_place():
    """Marshalled Shards (the wire bytes a peer sends) unmarshalled with
    rs_shard_unmarshal_arena: ShardData lands 16-byte aligned in the arena
    and the batch decodes in place, bit-exact."""
    from rsmi import host as h
    lib = rsmi.load()

    class View(ctypes.Structure):
        _fields_ = [("file_signature", ctypes.c_void_p), ("file_signature_len", ctypes.c_size_t),
                    ("shard_data", ctypes.c_void_p), ("shard_data_len", ctypes.c_size_t),
                    ("shard_number", ctypes.c_uint64), ("total_shards", ctypes.c_uint64),
                    ("minimum_needed_shards", ctypes.c_uint64)]

    k, n, S, B = 10, 14, 104858, 6
    f = rsmi.FEC(k, n)
    msgs = _messages(k, n, S, B, 77)
    arena = rsmi.Arena(B * k * 105 * 1024)
    wires, addr = [], {}
    for b, (_, sh, keep) in enumerate(msgs):
        for i in keep:
            w = h.Shard(b"\x42" * 64, sh[i], i, n, k).Marshal()
            wires.append(w)
            v = View()
            assert lib.rs_shard_unmarshal_arena(ctypes.c_char_p(w), len(w), arena._a, ctypes.byref(v)) == 0
            assert v.shard_number == i and v.shard_data_len == S and v.shard_data % 16 == 0
            assert ctypes.string_at(v.shard_data, S) == sh[i]
            addr[(b, i)] = v.shard_data
    rc, outs, st = _decode_batch(f, msgs, lambda b, i: addr[(b, i)])
    assert rc == 0 and all(o == d for o, (d, _, _) in zip(outs, msgs))
    assert f.stat(f.STAT_BATCHES_IN_PLACE) == 1
    full = rsmi.Arena(1024)  # too small: RS_ENOMEM, nothing written
    v = View()
    assert lib.rs_shard_unmarshal_arena(ctypes.c_char_p(wires[0]), len(wires[0]), full._a,
                                        ctypes.byref(v)) == rsmi.RS_ENOMEM
    arena.free()
    full.free()
    f.close()


@pytest.mark.parametrize("k,n,S", [(10, 14, 65536), (4, 6, 4096), (10, 14, 1 << 20)])
def test_host_api_in_place_encode_decode(k, n, S):
    """rs_encode with input and parity in engine-pinned memory runs the
    split-table kernel on them in place (no staging); rs_decode of k pinned
    survivors reads them in place too (rsmi.cpp decode_in_place: one launch,
    pattern and shard table read from pinned staging), writing the missing
    shares straight into a pinned dst or through staging into a pageable one.
    Bit-exact vs oracle."""
    lib = rsmi.load()
    f = rsmi.FEC(k, n)
    m = n - k
    E = oracle.fec_matrix(k, n)
    data = oracle.splitmix_bytes(k * S, 31 + S).tobytes()
    pin_in, pin_par, pin_dst = lib.rs_pinned_alloc(k * S), lib.rs_pinned_alloc(m * S), lib.rs_pinned_alloc(k * S)
    try:
        ctypes.memmove(pin_in, data, k * S)
        assert lib.rs_encode(f.handle, pin_in, k * S, pin_par) == rsmi.RS_OK
        assert f.stat(f.STAT_ENCODES_IN_PLACE) == 1
        assert ctypes.string_at(pin_par, m * S) == oracle.encode(E, k, n, data)
        keep = list(range(m, k)) + list(range(k, n))  # first m data shards lost
        nums = (ctypes.c_int * k)(*keep[::-1])
        ptrs = (ctypes.c_void_p * k)(*[pin_in + i * S if i < k else pin_par + (i - k) * S for i in keep[::-1]])
        d0 = f.stat(f.STAT_DECODES_IN_PLACE)
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, pin_dst) == rsmi.RS_OK
        assert f.stat(f.STAT_DECODES_IN_PLACE) == d0 + 1
        assert ctypes.string_at(pin_dst, k * S) == data
        assert list(nums) == sorted(keep)
        # pageable dst: the regenerated shares go through pinned staging
        pdst = ctypes.create_string_buffer(k * S)
        nums = (ctypes.c_int * k)(*keep)
        ptrs = (ctypes.c_void_p * k)(*[pin_in + i * S if i < k else pin_par + (i - k) * S for i in keep])
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, ctypes.cast(pdst, ctypes.c_void_p)) == rsmi.RS_OK
        assert f.stat(f.STAT_DECODES_IN_PLACE) == d0 + 2 and pdst.raw == data
        # one survivor pageable: the staged path, same bytes
        lone = ctypes.create_string_buffer(ctypes.string_at(ptrs[0], S), S)
        ptrs[0] = ctypes.cast(lone, ctypes.c_void_p)
        pdst2 = ctypes.create_string_buffer(k * S)
        assert lib.rs_decode(f.handle, nums, ptrs, k, S, ctypes.cast(pdst2, ctypes.c_void_p)) == rsmi.RS_OK
        assert f.stat(f.STAT_DECODES_IN_PLACE) == d0 + 2 and pdst2.raw == data
        # pageable parity: staged pipeline, same bytes
        pageable = ctypes.create_string_buffer(m * S)
        assert lib.rs_encode(f.handle, pin_in, k * S, ctypes.cast(pageable, ctypes.c_void_p)) == rsmi.RS_OK
        assert f.stat(f.STAT_ENCODES_IN_PLACE) == 1 and pageable.raw == ctypes.string_at(pin_par, m * S)
    finally:
        for p in (pin_in, pin_par, pin_dst):
            lib.rs_pinned_free(p)
    f.close()


@pytest.mark.parametrize("cross", [False, True])
@pytest.mark.parametrize("k,n,S,B", [(10, 14, 104858, 6), (10, 14, 4096, 9), (64, 80, 4099, 3)])
def test_decode_batch_dst_aliasing_survivors(k, n, S, B, cross):
    """The batched twin of test_decode_dst_overlapping_survivors (VERDICT r05
    weak #4): arena (engine-pinned) survivors that the dsts alias.  Message
    b's kept shares sit one row before their own inside a block of pinned
    memory; its dst is that block (cross=False: the decode overwrites its own
    survivors) or the next message's block (cross=True: message b's outputs
    land on message b+1's survivors while later chunks still read them).
    Every message decodes to its data, against the oracle."""
    lib = rsmi.load()
    f = rsmi.FEC(k, n)
    msgs = _messages(k, n, S, B, 31 * k + S + cross)
    blk = (n + 2) * S
    base = lib.rs_pinned_alloc(B * blk)
    assert base
    try:
        def row_addr(b, r):  # row r of message b's block (r = -1 just before its dst)
            return base + b * blk + (r + 1) * S
        ptr = {}
        for b, (_, sh, keep) in enumerate(msgs):
            for i in keep:
                ptr[(b, i)] = row_addr(b, i - 1)
                ctypes.memmove(ptr[(b, i)], sh[i], S)
        counts = (ctypes.c_int * B)(*[k] * B)
        order = [list(reversed(keep)) for _, _, keep in msgs]  # arrival order: sorted in place
        nums = (ctypes.c_int * (B * k))(*[i for o in order for i in o])
        ptrs = (ctypes.c_void_p * (B * k))(*[ptr[(b, i)] for b, o in enumerate(order) for i in o])
        dst_of = [row_addr((b + 1) % B if cross else b, 0) for b in range(B)]
        dsts = (ctypes.c_void_p * B)(*dst_of)
        st = (ctypes.c_int * B)()
        assert lib.rs_decode_batch(f.handle, B, counts, nums, ptrs, S, dsts, st) == rsmi.RS_OK
        assert list(st) == [0] * B
        E = oracle.fec_matrix(k, n)
        for b, (data, sh, keep) in enumerate(msgs):
            assert ctypes.string_at(dst_of[b], k * S) == data, b
            rc2, ref = oracle.decode(E, k, n, [(i, sh[i]) for i in keep])
            assert rc2 == 0 and ref == data
            # the caller's arrays sorted in place, pointers still the caller's
            got = [(nums[b * k + j], ptrs[b * k + j]) for j in range(k)]
            assert got == sorted((i, ptr[(b, i)]) for i in keep)
    finally:
        lib.rs_pinned_free(base)
        f.close()
