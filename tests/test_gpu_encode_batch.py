"""GPU: rs_encode_batch (send-side batching) against the oracle.

Many messages' Encode (main.go:262, called once per message by shardInput,
main.go:243-267) in one GPU pass: every message's parity must equal the
oracle's encode of it, and equal what rs_encode gives one message at a time.
Covers the split-table codes and the bit-sliced ones, ragged shard lengths
(the staging pitch pads them), batches staged in one chunk and in several,
and the error statuses (length not a multiple of k, a null message).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

_FECS = {}


def fec(k, n):
    if (k, n) not in _FECS:
        _FECS[(k, n)] = rsmi.NewFEC(k, n)
    return _FECS[(k, n)]


def _messages(k, S, B, seed):
    return [oracle.splitmix_bytes(k * S, seed + 977 * b).tobytes() for b in range(B)]


@pytest.mark.parametrize("k,n,S,B", [
    (10, 14, 1, 5), (10, 14, 17, 9), (10, 14, 4099, 33), (10, 14, 104858, 7),
    (4, 6, 4096, 64), (8, 14, 6553, 11), (64, 80, 4099, 6), (17, 49, 1000, 5), (1, 2, 333, 4),
])
def test_encode_batch_matches_oracle(k, n, S, B):
    f = fec(k, n)
    E = oracle.fec_matrix(k, n)
    msgs = _messages(k, S, B, 100 * k + S)
    before = f.stat(rsmi.FEC.STAT_ENCODE_BATCHES)
    par, st = f.EncodeBatch(msgs)
    assert st == [0] * B
    for b in range(B):
        assert par[b] == oracle.encode(E, k, n, msgs[b]), b
    assert f.stat(rsmi.FEC.STAT_ENCODE_BATCHES) == before + 1


def test_encode_batch_chunked_config1_messages():
    """20 config-1 messages (>= 16 MiB staged: four chunks, each coded while
    the next is copied in), against rs_encode one message at a time."""
    k, n = 10, 14
    f = fec(k, n)
    S = 104858
    msgs = _messages(k, S, 20, 7)
    par, st = f.EncodeBatch(msgs)
    assert st == [0] * 20
    E = oracle.fec_matrix(k, n)
    for b in (0, 5, 19):
        assert par[b] == oracle.encode(E, k, n, msgs[b])
    for b in range(20):
        assert par[b] == f.encode_parity(msgs[b])


def test_encode_batch_large_shards_past_a_group():
    """Messages whose staging exceeds one group's budget go through several
    groups (RS(10,4), 4 MiB shards: 56 MiB per message)."""
    k, n = 10, 14
    f = fec(k, n)
    S = 4 << 20
    msgs = _messages(k, S, 10, 3)
    par, st = f.EncodeBatch(msgs)
    assert st == [0] * 10
    E = oracle.fec_matrix(k, n)
    for b in (0, 9):  # the first group and the last
        assert par[b] == oracle.encode(E, k, n, msgs[b])
    for b in range(10):
        assert par[b] == f.encode_parity(msgs[b])


def test_encode_batch_errors_and_edges():
    k, n = 10, 14
    f = fec(k, n)
    lib = rsmi.load()
    # len not a multiple of k: every message fails the same way
    par, st = f.EncodeBatch([b"x" * 13, b"y" * 13])
    assert st == [rsmi.RS_ELEN_NOT_MULTIPLE] * 2 and par == [None, None]
    # empty messages: nothing to code
    par, st = f.EncodeBatch([b"", b""])
    assert st == [0, 0] and par == [b"", b""]
    # an empty batch
    assert f.EncodeBatch([]) == ([], [])
    # a null message among good ones: only it fails
    S = 4096
    msgs = _messages(k, S, 3, 11)
    keep = [bytes(m) for m in msgs]
    ins = (ctypes.c_void_p * 3)(ctypes.cast(ctypes.c_char_p(keep[0]), ctypes.c_void_p).value, None,
                                ctypes.cast(ctypes.c_char_p(keep[2]), ctypes.c_void_p).value)
    outs = [bytearray(4 * S) for _ in range(3)]
    outp = (ctypes.c_void_p * 3)(*[ctypes.addressof((ctypes.c_char * len(o)).from_buffer(o)) for o in outs])
    st = (ctypes.c_int * 3)()
    rc = lib.rs_encode_batch(f.handle, 3, ins, k * S, outp, st)
    assert rc == rsmi.RS_EINVAL and list(st) == [0, rsmi.RS_EINVAL, 0]
    E = oracle.fec_matrix(k, n)
    assert bytes(outs[0]) == oracle.encode(E, k, n, keep[0])
    assert bytes(outs[2]) == oracle.encode(E, k, n, keep[2])
    # bad arguments
    assert lib.rs_encode_batch(None, 1, ins, k * S, outp, st) == rsmi.RS_EINVAL
    assert lib.rs_encode_batch(f.handle, -1, ins, k * S, outp, st) == rsmi.RS_EINVAL


def test_encode_batch_messages_alias_nothing_between_calls():
    """Back-to-back batches on one context (the lease's staging reused) give
    each batch its own parity."""
    k, n = 10, 14
    f = fec(k, n)
    E = oracle.fec_matrix(k, n)
    for rep in range(4):
        msgs = _messages(k, 6554 + 16 * rep, 24, 1000 + rep)
        par, st = f.EncodeBatch(msgs)
        assert st == [0] * 24
        assert par[rep] == oracle.encode(E, k, n, msgs[rep])
        assert par[-1] == oracle.encode(E, k, n, msgs[-1])


def test_batches_split_into_staging_groups():
    """A batch larger than the pinned-staging cap goes in groups of messages
    (both batch calls; RSMI_BATCH_STAGE_MB=2 in a child process): every
    message still matches the oracle, and rs_decode_batch returns the first
    failing status in message order across groups."""
    import os
    import subprocess
    import sys
    code = r'''
import sys; sys.path[:0] = ['.', 'noise-erasurecode-plugin_amd']
import numpy as np, rsmi
from oracle import oracle
k, n, S, B = 10, 14, 8192, 40
f = rsmi.NewFEC(k, n); E = oracle.fec_matrix(k, n)
msgs = [oracle.splitmix_bytes(k * S, 300 + b).tobytes() for b in range(B)]
b0 = f.stat(f.STAT_ENCODE_BATCHES)
par, st = f.EncodeBatch(msgs)
assert st == [0] * B
assert all(par[b] == oracle.encode(E, k, n, msgs[b]) for b in range(B))
assert f.stat(f.STAT_ENCODE_BATCHES) - b0 >= 2, "one group only"
rng = np.random.default_rng(9); batch = []
for b in range(B):
    sh = [msgs[b][i*S:(i+1)*S] for i in range(k)] + [par[b][i*S:(i+1)*S] for i in range(n - k)]
    keep = rng.choice(n, size=k, replace=False).tolist()
    batch.append([rsmi.Share(i, sh[i]) for i in keep])
batch[33] = batch[33][:k - 1]       # not enough shares, in a later group
s0 = f.stat(f.STAT_BATCHES_STAGED)
outs, st = f.DecodeBatch(batch)
assert st[33] == rsmi.RS_ENOT_ENOUGH and outs[33] is None
assert all(st[b] == 0 and outs[b] == msgs[b] for b in range(B) if b != 33)
assert f.stat(f.STAT_BATCHES_STAGED) - s0 >= 3, "one group only"
print('ok')
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, RSMI_BATCH_STAGE_MB="2"))
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_decode_batch_failure_marks_its_messages():
    """A failing batched pass (the context's first pattern build made to fail,
    RSMI_TEST_FAIL_FLUSH=1) fails every message it carried -- none keeps a
    stale RS_OK -- while a Correct-path message in the same call decodes;
    the next call on the context decodes everything."""
    import os
    k, n, S = 10, 14, 4096
    old = os.environ.get("RSMI_TEST_FAIL_FLUSH")
    os.environ["RSMI_TEST_FAIL_FLUSH"] = "1"
    try:
        f = rsmi.FEC(k, n)
    finally:
        if old is None:
            del os.environ["RSMI_TEST_FAIL_FLUSH"]
        else:
            os.environ["RSMI_TEST_FAIL_FLUSH"] = old
    E = oracle.fec_matrix(k, n)
    msgs = _messages(k, S, 6, 77)
    batch = []
    for b, data in enumerate(msgs):
        par = oracle.encode(E, k, n, data)
        sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
        keep = [i for i in range(n) if i != b % k][: k + (2 if b == 2 else 0)]  # message 2: Correct path
        batch.append([rsmi.Share(i, sh[i]) for i in keep])
    outs, st = f.DecodeBatch(batch)
    assert st[2] == 0 and outs[2] == msgs[2]
    assert all(st[b] != 0 and outs[b] is None for b in range(6) if b != 2), st
    outs, st = f.DecodeBatch(batch)
    assert st == [0] * 6 and outs == msgs
    f.close()


@pytest.mark.parametrize("nt", ["1", "0"])
def test_staging_copy_modes_match_oracle(nt):
    """Small staged messages (rs_encode / rs_decode, both staging chunks) and
    a batch, with the non-temporal staging copy (default) and with memcpy
    (RSMI_STAGE_NT=0; the knob is read once per process: a child)."""
    import os
    import subprocess
    import sys
    code = r'''
import sys; sys.path[:0] = ['.', 'noise-erasurecode-plugin_amd']
import numpy as np, rsmi
from oracle import oracle
k, n = 10, 14
f = rsmi.NewFEC(k, n); E = oracle.fec_matrix(k, n)
for S in (1, 4095, 104858, 65543):
    data = oracle.splitmix_bytes(k * S, S).tobytes()
    par = f.encode_parity(data)
    assert par == oracle.encode(E, k, n, data), S
    sh = [data[i*S:(i+1)*S] for i in range(k)] + [par[i*S:(i+1)*S] for i in range(n - k)]
    keep = [13, 2, 11, 4, 5, 6, 10, 8, 9, 12]
    got = f.Decode(None, [rsmi.Share(i, sh[i]) for i in keep])
    assert got == data, S
msgs = [oracle.splitmix_bytes(k * 70001, 9 + b).tobytes() for b in range(30)]
pars, st = f.EncodeBatch(msgs)
assert st == [0] * 30 and all(p == oracle.encode(E, k, n, m) for p, m in zip(pars, msgs))
print('ok')
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, RSMI_STAGE_NT=nt))
    assert r.returncode == 0 and "ok" in r.stdout, (nt, r.stdout, r.stderr[-2000:])


def test_one_message_batches_take_the_single_message_path():
    """A batch of one message is coded by rs_encode / rs_decode's two-chunk
    staged path (no batched pass counted), bit-exact; two messages already
    go through the batched pass."""
    k, n, S = 10, 14, 104858
    f = fec(k, n)
    E = oracle.fec_matrix(k, n)
    msgs = _messages(k, S, 2, 4242)
    b0 = f.stat(rsmi.FEC.STAT_ENCODE_BATCHES)
    par, st = f.EncodeBatch(msgs[:1])
    assert st == [0] and par[0] == oracle.encode(E, k, n, msgs[0])
    assert f.stat(rsmi.FEC.STAT_ENCODE_BATCHES) == b0
    par2, st = f.EncodeBatch(msgs)
    assert st == [0, 0] and par2[1] == oracle.encode(E, k, n, msgs[1])
    assert f.stat(rsmi.FEC.STAT_ENCODE_BATCHES) == b0 + 1
    s0 = f.stat(rsmi.FEC.STAT_BATCHES_STAGED)
    batch = []
    for data, p in zip(msgs, par2):
        sh = [data[i * S:(i + 1) * S] for i in range(k)] + [p[i * S:(i + 1) * S] for i in range(n - k)]
        batch.append([rsmi.Share(i, sh[i]) for i in (13, 1, 12, 3, 4, 11, 6, 7, 8, 10)])
    outs, st = f.DecodeBatch(batch[:1])
    assert st == [0] and outs == msgs[:1] and f.stat(rsmi.FEC.STAT_BATCHES_STAGED) == s0
    outs, st = f.DecodeBatch(batch)
    assert st == [0, 0] and outs == msgs and f.stat(rsmi.FEC.STAT_BATCHES_STAGED) == s0 + 1
