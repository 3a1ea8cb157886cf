"""Mailbox grid (rsmi.cpp MailboxCall, rs_kernels.hip rs_mailbox_kernel).

A staged single message of two column chunks -- rs_encode / rs_decode of a
config-1 message (main.go:262 / main.go:77) -- is coded by one grid launched
before the first chunk is staged; the chunks are posted to it through pinned
memory.  Checked bit-exact against the oracle: on the mailbox path (its
counter moves, nothing recovered), with it off (RSMI_MAILBOX=0), with grids
that give up before the host posts (RSMI_MAILBOX_TIMEOUT_US=1: the caller
launches the undone chunks itself), and from concurrent callers, each with a
grid of its own.
"""
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shards(k, n, S, seed):
    data = oracle.splitmix_bytes(k * S, seed).tobytes()
    par = oracle.encode(oracle.fec_matrix(k, n), k, n, data)
    sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
    return data, par, sh


def _roundtrips(f, k, n, S, seed, patterns):
    """encode_parity + Decode for each keep-pattern; returns the GPU calls made."""
    data, par, sh = _shards(k, n, S, seed)
    assert f.encode_parity(data) == par
    calls = 1
    rng = np.random.default_rng(seed)
    for _ in range(patterns):
        keep = sorted(rng.choice(n, size=k, replace=False).tolist())
        rng.shuffle(keep)
        assert f.Decode(None, [rsmi.Share(i, sh[i]) for i in keep]) == data, keep
        calls += any(i >= k for i in keep)  # a decode with every data share present copies only
    return calls


# Shard lengths whose k shards fit the one-shot staging (<= 2 MiB) in two
# chunks (>= 256 KiB): the config-1 message (1,048,580 B / 10), the chunk
# threshold, odd lengths and the largest staged RS(10,4) message.
@pytest.mark.parametrize("k,n,S", [(10, 14, 104858), (10, 14, 26215), (10, 14, 33333), (10, 14, 209700),
                                   (4, 6, 65536), (4, 6, 99999), (4, 6, 524000)])
def test_mailbox_parity(k, n, S):
    f = rsmi.NewFEC(k, n)
    c0 = f.stat(f.STAT_MAILBOX_CALLS)
    calls = _roundtrips(f, k, n, S, k * 7919 + S, 12)
    assert f.stat(f.STAT_MAILBOX_CALLS) - c0 == calls
    assert f.stat(f.STAT_MAILBOX_RECOVERED) == 0


@pytest.mark.skipif(os.environ.get("RSMI_MAILBOX_MIN_JOBS", "2") != "2", reason="one-chunk calls use the grid too")
def test_mailbox_not_used_below_two_chunks_or_for_bitslice_codes():
    f = rsmi.NewFEC(10, 14)
    c0 = f.stat(f.STAT_MAILBOX_CALLS)
    _roundtrips(f, 10, 14, 1000, 5, 4)  # one chunk: ordinary launch
    assert f.stat(f.STAT_MAILBOX_CALLS) == c0
    g = rsmi.NewFEC(8, 14)  # no mailbox variant (k = 8)
    _roundtrips(g, 8, 14, 40000, 6, 4)
    assert g.stat(g.STAT_MAILBOX_CALLS) == 0


def test_mailbox_concurrent_callers():
    k, n, S = 10, 14, 104858
    f = rsmi.NewFEC(k, n)
    errors = []

    def worker(t):
        try:
            _roundtrips(f, k, n, S, 1000 + t, 6)
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    assert f.stat(f.STAT_MAILBOX_CALLS) > 0
    assert f.stat(f.STAT_MAILBOX_RECOVERED) == 0


_CHILD = r"""
import sys
root = sys.argv[1]
sys.path[:0] = [root, root + "/noise-erasurecode-plugin_amd"]
import numpy as np
import rsmi
from oracle import oracle
k, n, S, seed = 10, 14, 104858, 77
data = oracle.splitmix_bytes(k * S, seed).tobytes()
par = oracle.encode(oracle.fec_matrix(k, n), k, n, data)
sh = [data[i * S:(i + 1) * S] for i in range(k)] + [par[i * S:(i + 1) * S] for i in range(n - k)]
f = rsmi.NewFEC(k, n)
assert f.encode_parity(data) == par
calls = 1
for keep in ([0, 2, 3, 4, 5, 7, 8, 9, 10, 11], [13, 12, 11, 10, 0, 1, 2, 3, 4, 5], [1, 3, 5, 7, 9, 10, 11, 12, 13, 0]):
    assert f.Decode(None, [rsmi.Share(i, sh[i]) for i in keep]) == data, keep
    calls += 1
print(calls, f.stat(f.STAT_MAILBOX_CALLS), f.stat(f.STAT_MAILBOX_RECOVERED))
"""


def _child(**env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return [int(v) for v in r.stdout.split()[-3:]]


def test_mailbox_off():
    calls, mb, rec = _child(RSMI_MAILBOX="0")
    assert calls > 0 and mb == 0 and rec == 0


def test_mailbox_grid_gives_up_and_caller_recovers():
    # Block 0 waits 1 us for each post: the grid leaves before (most of) the
    # chunks are staged, and the caller launches them itself -- same bytes.
    calls, mb, rec = _child(RSMI_MAILBOX_TIMEOUT_US="1")
    assert mb == calls and rec > 0


@pytest.mark.parametrize("split", ["50", "20,45,75"])
def test_mailbox_other_chunk_splits(split):
    # Two and four column chunks (RSMI_CHUNK_SPLIT): a group per chunk, the
    # same bytes.
    calls, mb, rec = _child(RSMI_CHUNK_SPLIT=split)
    assert mb == calls and rec == 0
