"""GPU: device-set contexts (rs_new_devices) against the oracle.

north_star partitions stripes across the GPUs of one node, with the plugin's
Go host code calling HIP through the C ABI; a device-set context is that
partition behind the same ABI (VERDICT r05 "next" #1).  The pool's boxes have
one GPU, so the sets here are {0} and {0, 0} -- two members, two contexts and
two host threads on one GPU, which exercises every host path of the set
(partition, per-member threads, per-member streams and leases, the spread
reconstruct's per-owner tables) except xGMI itself.  Everything is checked
bit-exact against the oracle on config-2 geometry (RS(10,4), 1 MiB shards)
and config-5 geometry (RS(64,16), 64 KiB shards).
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

SETS = [[0], [0, 0]]


def _erasures(stripes, n, m, seed):
    rng = np.random.default_rng(seed)
    er = np.zeros((stripes, n), dtype=np.uint8)
    for s in range(stripes):
        er[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 1
    return er


@pytest.mark.parametrize("devices", SETS, ids=["set0", "set00"])
@pytest.mark.parametrize("k,n,S,stripes", [(10, 14, 1 << 20, 21), (64, 80, 65536, 37)])
def test_stripe_parts_encode_and_reconstruct(devices, k, n, S, stripes):
    """Stripe-local placement: rs_partition splits the stripes over the
    members, each member's part lives in its own buffers, one
    rs_encode_stripes_parts / rs_reconstruct_stripes_parts call runs every
    part (member threads at once).  Parity = oracle; every erased shard (1..m
    per stripe, data and parity) regenerated = oracle Rebuild = original."""
    m = n - k
    f = rsmi.FEC(k, n, devices=devices)
    G = f.member_count()
    assert G == len(devices)
    ranges = [rsmi.partition(stripes, G, g) for g in range(G)]
    data = [torch.empty(c * k * S, dtype=torch.uint8, device="cuda:0") for _, c in ranges]
    par = [torch.zeros(c * m * S, dtype=torch.uint8, device="cuda:0") for _, c in ranges]
    for g, (first, c) in enumerate(ranges):
        # stripe s's bytes are the splitmix stream of seed s, whichever member holds it
        for j in range(c):
            f.member(g).fill_splitmix(data[g].data_ptr() + j * k * S, k * S, 1000 + first + j)
    torch.cuda.synchronize()
    parts = [(data[g].data_ptr(), k * S, par[g].data_ptr(), m * S, c, 0) for g, (_, c) in enumerate(ranges)]
    f.encode_stripes_parts(parts, S, S)
    torch.cuda.synchronize()
    E = oracle.fec_matrix(k, n)
    hd = np.concatenate([d.cpu().numpy() for d in data])
    hp = np.concatenate([p.cpu().numpy() for p in par])
    for s in range(stripes):
        assert np.array_equal(hd[s * k * S:(s + 1) * k * S], oracle.splitmix_bytes(k * S, 1000 + s)), s
    ref = oracle.encode_batch(E, k, n, hd, S, stripes, threads=8)
    assert np.array_equal(hp, ref)
    # reconstruct: erase, zero, regenerate; the oracle regenerates the same
    er = _erasures(stripes, n, m, 77 + k)
    d0 = [x.clone() for x in data]
    p0 = [x.clone() for x in par]
    for g, (first, c) in enumerate(ranges):
        e = torch.from_numpy(er[first:first + c].astype(bool)).cuda()
        data[g].view(c, k, S)[e[:, :k]] = 0
        par[g].view(c, m, S)[e[:, k:]] = 0
    f.reconstruct_stripes_parts(parts, S, S, er.tobytes())
    torch.cuda.synchronize()
    for g in range(G):
        assert torch.equal(data[g], d0[g]) and torch.equal(par[g], p0[g]), g
    od, op = hd.copy(), hp.copy()
    for s in range(stripes):
        for i in np.flatnonzero(er[s]):
            (od[(s * k + i) * S:(s * k + i + 1) * S] if i < k else op[(s * m + i - k) * S:(s * m + i - k + 1) * S])[:] = 0
    assert oracle.reconstruct_batch(E, k, n, od, op, S, stripes, er, threads=8) == 0
    assert np.array_equal(od, hd) and np.array_equal(op, hp)
    f.close()


def _config1_messages(k, n, S, B, seed):
    E = oracle.fec_matrix(k, n)
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        data = oracle.splitmix_bytes(k * S, seed * 100 + b).tobytes()
        par = oracle.encode(E, k, n, data)
        sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
        keep = rng.choice(n, size=k, replace=False).tolist()  # arrival order
        out.append((data, par, [rsmi.Share(i, sh[i]) for i in keep]))
    return out


@pytest.mark.parametrize("devices", SETS, ids=["set0", "set00"])
def test_batches_split_over_members(devices):
    """rs_encode_batch / rs_decode_batch on a set: 9 config-1 messages split
    into contiguous ranges (4 + 5 on two members), each member one batched
    GPU pass; per-message results equal the oracle."""
    k, n, S, B = 10, 14, 104858, 9
    f = rsmi.FEC(k, n, devices=devices)
    msgs = _config1_messages(k, n, S, B, 5)
    pars, st = f.EncodeBatch([d for d, _, _ in msgs])
    assert st == [0] * B
    assert pars == [p for _, p, _ in msgs]
    for g in range(f.member_count()):
        assert f.member(g).stat(rsmi.FEC.STAT_ENCODE_BATCHES) == 1, g
    outs, st = f.DecodeBatch([list(sh) for _, _, sh in msgs])
    assert st == [0] * B
    assert outs == [d for d, _, _ in msgs]
    assert f.stat(rsmi.FEC.STAT_BATCHES_STAGED) == f.member_count()  # summed over the members
    f.close()


@pytest.mark.parametrize("devices", SETS, ids=["set0", "set00"])
def test_single_messages_from_threads_spread_over_members(devices):
    """rs_encode / rs_decode on a set from 8 threads (noise's concurrent
    Receive, main.go:49-52): every result oracle-exact, and with two members
    both serve calls (the least-busy pick)."""
    k, n, S = 10, 14, 104858
    f = rsmi.FEC(k, n, devices=devices)
    msgs = _config1_messages(k, n, S, 16, 9)
    errors = []

    def worker(t):
        try:
            for data, par, sh in msgs[t::8]:
                assert f.encode_parity(data) == par
                assert f.Decode(None, list(sh)) == data
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for g in range(f.member_count()):
        assert f.member(g).stat(rsmi.FEC.STAT_LEASES) >= 1, g  # member g served calls
    f.close()


@pytest.mark.parametrize("devices", SETS, ids=["set0", "set00"])
@pytest.mark.parametrize("k,n,S,stripes", [(10, 14, 1 << 20, 16), (64, 80, 65536, 24)])
def test_spread_reconstruct(devices, k, n, S, stripes):
    """Shard-distributed placement (main.go:207 sends every
    shard to a different peer): shard i of each stripe lives in holder i mod H
    (H = 2 separate allocations), stripe s is reconstructed by member s mod G
    reading its survivors where they lie (peer HBM on a multi-GPU node) and
    writing every erased shard back into its holder.  Bit-exact vs the
    originals, with the members' own streams and with NULL streams."""
    m = n - k
    f = rsmi.FEC(k, n, devices=devices)
    G = f.member_count()
    H = 2
    per = [(n - h + H - 1) // H for h in range(H)]  # shards per stripe in holder h
    holders = [torch.empty(stripes * per[h] * S, dtype=torch.uint8, device="cuda:0") for h in range(H)]
    # encode the stripes contiguously, then scatter shard i to holder i % H
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda:0")
    parity = torch.empty(stripes * m * S, dtype=torch.uint8, device="cuda:0")
    f.fill_splitmix(data.data_ptr(), data.numel(), 4242 + k)
    f.encode_stripes(data.data_ptr(), k * S, parity.data_ptr(), m * S, S, S, stripes)
    torch.cuda.synchronize()
    full = torch.cat([data.view(stripes, k, S), parity.view(stripes, m, S)], dim=1)  # [stripes][n][S]
    for h in range(H):
        holders[h].view(stripes, per[h], S).copy_(full[:, h::H, :])
    ptrs = np.zeros((stripes, n), dtype=np.uint64)
    for s in range(stripes):
        for i in range(n):
            h = i % H
            ptrs[s, i] = holders[h].data_ptr() + (s * per[h] + i // H) * S
    owner = [s % G for s in range(stripes)]
    ref = [x.clone() for x in holders]
    for use_streams in (False, True):
        er = _erasures(stripes, n, m, 11 + use_streams)
        for s in range(stripes):
            for i in np.flatnonzero(er[s]):
                h = int(i) % H
                holders[h].view(stripes, per[h], S)[s, int(i) // H].zero_()
        torch.cuda.synchronize()
        streams = None
        if use_streams:
            ss = [torch.cuda.Stream() for _ in range(G)]
            streams = [x.cuda_stream for x in ss]
        f.reconstruct_spread(ptrs.reshape(-1).tolist(), owner, S, stripes, er.tobytes(), streams)
        torch.cuda.synchronize()
        for h in range(H):
            assert torch.equal(holders[h], ref[h]), (use_streams, h)
    f.close()


def test_single_device_context_is_a_set_of_one():
    """The set calls on a plain context: member 0 is the context itself, the
    parts and spread calls take one part / owner 0."""
    k, n, S, stripes = 10, 14, 65536, 6
    m = n - k
    f = rsmi.FEC(k, n)
    assert f.member_count() == 1 and f.member(0).handle.value == f.handle.value
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda:0")
    par = torch.zeros(stripes * m * S, dtype=torch.uint8, device="cuda:0")
    f.fill_splitmix(data.data_ptr(), data.numel(), 3)
    f.encode_stripes_parts([(data.data_ptr(), k * S, par.data_ptr(), m * S, stripes, 0)], S, S)
    torch.cuda.synchronize()
    E = oracle.fec_matrix(k, n)
    assert np.array_equal(par.cpu().numpy(), oracle.encode_batch(E, k, n, data.cpu().numpy(), S, stripes))
    f.close()


def test_set_routes_device_resident_calls_by_buffer():
    """rs_encode_stripes / rs_reconstruct_stripes on a set run on a member on
    the device that holds the data; a set naming a device that does not exist
    is refused."""
    k, n, S, stripes = 10, 14, 65536, 4
    m = n - k
    f = rsmi.FEC(k, n, devices=[0, 0])
    data = torch.empty(stripes * k * S, dtype=torch.uint8, device="cuda:0")
    par = torch.zeros(stripes * m * S, dtype=torch.uint8, device="cuda:0")
    f.fill_splitmix(data.data_ptr(), data.numel(), 21)
    f.encode_stripes(data.data_ptr(), k * S, par.data_ptr(), m * S, S, S, stripes)
    torch.cuda.synchronize()
    E = oracle.fec_matrix(k, n)
    assert np.array_equal(par.cpu().numpy(), oracle.encode_batch(E, k, n, data.cpu().numpy(), S, stripes))
    d0 = data.clone()
    er = np.zeros((stripes, n), dtype=np.uint8)
    er[:, 3] = 1
    data.view(stripes, k, S)[:, 3] = 0
    f.reconstruct_stripes(data.data_ptr(), k * S, par.data_ptr(), m * S, S, S, stripes, er.tobytes())
    torch.cuda.synchronize()
    assert torch.equal(data, d0)
    f.prepare_patterns(2)  # every member
    assert f.pattern_count() >= 2 * (n + n * (n - 1) // 2)
    # a member belongs to its set: rs_free on it does nothing, the set still works
    rsmi.load().rs_free(f.member(1).handle)
    msgs = _config1_messages(k, n, 4096, 4, 3)
    pars, st = f.EncodeBatch([d for d, _, _ in msgs])
    assert st == [0] * 4 and pars == [p for _, p, _ in msgs]
    f.close()
    with pytest.raises(rsmi.RSError) as ei:
        rsmi.FEC(k, n, devices=[0, torch.cuda.device_count() + 7])
    assert ei.value.code == rsmi.RS_EDEVICE
