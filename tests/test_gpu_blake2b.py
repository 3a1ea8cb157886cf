"""GPU BLAKE2b: the plugin's hash policy
(defaultHashPolicy = blake2b.New(), main.go:38-41) applied to
serializeMessage(id, message) when signing (main.go:219-223) and verifying
(main.go:82-89).  Every digest is checked bit-exact against Python's
hashlib.blake2b (an independent RFC 7693 implementation) for 32- and 64-byte
digests (noise's policy is recalled to be the 32-byte Sum256; both are
covered), edge lengths around the 128-byte block, a config-1-sized message,
ragged batches, and unaligned device-resident messages.
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import rsmi  # noqa: E402
from oracle import oracle  # noqa: E402

_F = {}


def fec():
    if "f" not in _F:
        _F["f"] = rsmi.FEC(10, 14)
    return _F["f"]


def _msg(n, seed):
    return oracle.splitmix_bytes(n, seed).tobytes()


EDGE = [0, 1, 3, 16, 31, 32, 33, 64, 127, 128, 129, 255, 256, 257, 1000, 4096, 65540]


@pytest.mark.parametrize("digest_len", [32, 64, 1, 20, 48])
def test_blake2b_edge_lengths(digest_len):
    msgs = [_msg(n, 100 + n) for n in EDGE]
    got = fec().blake2b_batch(msgs, digest_len)
    for m, g in zip(msgs, got):
        assert g == hashlib.blake2b(m, digest_size=digest_len).digest(), (len(m), digest_len)


def test_blake2b_rfc7693_abc():
    """RFC 7693 Appendix A: BLAKE2b-512("abc")."""
    want = bytes.fromhex(
        "ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
        "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert fec().blake2b_batch([b"abc"], 64)[0] == want


@pytest.mark.parametrize("digest_len", [32, 64])
def test_blake2b_config1_serialized_message(digest_len):
    """The hash the send side signs for BASELINE config 1:
    serializeMessage(id, 1 MiB blob + 4 zero bytes)."""
    from rsmi import host as h
    blob = _msg(1 << 20, 0x5EED) + b"\0" * 4
    me = h.PeerID("tcp://localhost:3000", b"\x11" * 32)
    ser = h.serializeMessage(me, blob)
    assert len(ser) == 4 + len("tcp://localhost:3000") + 4 + 32 + len(blob)
    got = fec().blake2b_batch([ser, blob, ser[:1048580]], digest_len)
    for m, g in zip([ser, blob, ser[:1048580]], got):
        assert g == hashlib.blake2b(m, digest_size=digest_len).digest()


def test_blake2b_ragged_batch():
    """2,000 messages of random lengths 0..5,000 (one launch, sorted longest
    first inside the engine, digests back in caller order)."""
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 5000, size=2000)
    msgs = [_msg(int(n), 9000 + i) for i, n in enumerate(lens)]
    for dl in (32, 64):
        got = fec().blake2b_batch(msgs, dl)
        assert all(g == hashlib.blake2b(m, digest_size=dl).digest() for m, g in zip(msgs, got))


def test_blake2b_device_unaligned_messages():
    """rs_blake2b_device over messages at every byte alignment in one device
    buffer (the dword-aligned funnel-shift path and its zero-padded tail)."""
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(0, 700, size=96)] + [128, 129, 1, 0]
    msgs = [_msg(n, 500 + i) for i, n in enumerate(lens)]
    offs, pos = [], 0
    for i, m in enumerate(msgs):
        pos += i % 16  # misalign by 0..15 bytes
        offs.append(pos)
        pos += len(m)
    buf = np.zeros(pos + 64, dtype=np.uint8)
    for o, m in zip(offs, msgs):
        buf[o:o + len(m)] = np.frombuffer(m, dtype=np.uint8)
    dbuf = torch.from_numpy(buf).cuda()
    base = dbuf.data_ptr()
    ptrs = torch.tensor([base + o for o in offs], dtype=torch.int64, device="cuda")
    dlen = torch.tensor(lens, dtype=torch.int64, device="cuda")
    for dl in (32, 64):
        out = torch.zeros(len(msgs) * dl, dtype=torch.uint8, device="cuda")
        fec().blake2b_device(len(msgs), ptrs.data_ptr(), dlen.data_ptr(), 0, dl, out.data_ptr())
        fec().sync()
        got = out.cpu().numpy().tobytes()
        for i, m in enumerate(msgs):
            assert got[i * dl:(i + 1) * dl] == hashlib.blake2b(m, digest_size=dl).digest(), (i, offs[i] % 16)


def test_blake2b_batch_of_large_messages_chunked():
    """64 messages of 300-400 KiB: > 16 MiB staged, so the input crosses PCIe
    in chunks overlapped with the staging copies."""
    rng = np.random.default_rng(3)
    msgs = [_msg(int(n), 77 + i) for i, n in enumerate(rng.integers(300 << 10, 400 << 10, size=64))]
    got = fec().blake2b_batch(msgs, 32)
    assert all(g == hashlib.blake2b(m, digest_size=32).digest() for m, g in zip(msgs, got))


def test_blake2b_batch_split_into_staging_groups():
    """Beyond the pinned-staging cap (RSMI_BATCH_STAGE_MB=1, a child
    process) the batch is hashed in groups of consecutive messages, one of
    them larger than the cap by itself; every digest matches hashlib."""
    import subprocess
    import sys
    code = r"""
import sys, hashlib; sys.path[:0] = ['.', 'noise-erasurecode-plugin_amd']
import numpy as np, rsmi
from oracle import oracle
f = rsmi.NewFEC(10, 14)
lens = [300 << 10] * 6 + [3 << 20] + [1000, 0, 700 << 10] * 3
msgs = [oracle.splitmix_bytes(n, 40 + i).tobytes() for i, n in enumerate(lens)]
got = f.blake2b_batch(msgs, 32)
assert all(g == hashlib.blake2b(m, digest_size=32).digest() for m, g in zip(msgs, got))
print('ok')
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, RSMI_BATCH_STAGE_MB="1"))
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_blake2b_bad_arguments():
    lib = rsmi.load()
    import ctypes
    out = ctypes.create_string_buffer(64)
    ptrs = (ctypes.c_void_p * 1)(None)
    lens = (ctypes.c_size_t * 1)(0)
    for dl in (0, 65):
        assert lib.rs_blake2b_batch(fec().handle, 1, ptrs, lens, dl, ctypes.cast(out, ctypes.c_void_p)) == rsmi.RS_EINVAL
    lens[0] = 5  # NULL message with a length
    assert lib.rs_blake2b_batch(fec().handle, 1, ptrs, lens, 32, ctypes.cast(out, ctypes.c_void_p)) == rsmi.RS_EINVAL


def test_hash_policy_crossover_bit_exact():
    """rs_blake2b: one message -- or a few long ones -- is
    hashed on the host, many short ones on the GPU; the digests equal
    hashlib's on both sides of the crossover, for 32- and 64-byte digests."""
    f = fec()
    rng = np.random.default_rng(3)
    cases = [
        ([_msg(1048580 + 40, 1)], 0),                                    # config-1 message: host
        ([_msg(65536, 10 + i) for i in range(4)], 0),                     # 4 long chains: host
        ([_msg(int(rng.integers(0, 2048)), 100 + i) for i in range(8192)], 1),  # many short: GPU
    ]
    for msgs, want_where in cases:
        for dl in (32, 64):
            got, where = f.blake2b(msgs, dl)
            assert where == want_where, (len(msgs), dl)
            assert got == [hashlib.blake2b(m, digest_size=dl).digest() for m in msgs]


def test_host_and_gpu_sides_agree_on_edges():
    msgs = [_msg(n, 7 + n) for n in EDGE]
    f = fec()
    for dl in (1, 32, 64):
        assert rsmi.blake2b_host(msgs, dl) == f.blake2b_batch(msgs, dl)
