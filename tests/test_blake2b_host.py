"""Host BLAKE2b (rs_blake2b_host, csrc/blake2b_host.cpp): the host side of
the hash policy the plugin applies to serializeMessage (main.go:38-41,
:219-223, :82-89).  Runs on the CPU: the C ABI's host hash needs no context
and no GPU.  Checked against Python's hashlib.blake2b (an independent RFC
7693 implementation) at every length around the 128-byte block boundaries,
digest lengths 1..64, one and many threads, and the RFC 7693 Appendix A
vector."""
import hashlib

import numpy as np
import pytest

import rsmi


def _ref(m, d):
    return hashlib.blake2b(m, digest_size=d).digest()


def test_rfc7693_appendix_a():
    got = rsmi.blake2b_host([b"abc"], 64)[0]
    assert got.hex().startswith("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1")
    assert got == _ref(b"abc", 64)


@pytest.mark.parametrize("digest_len", [1, 20, 32, 48, 64])
def test_lengths_around_block_boundaries(digest_len):
    rng = np.random.default_rng(digest_len)
    lens = sorted({0, 1, 2, 63, 64, 65, 111, 112, 127, 128, 129, 255, 256, 257, 383, 384, 385, 1000, 4096, 65537})
    msgs = [rng.integers(0, 256, size=L, dtype=np.uint8).tobytes() for L in lens]
    for threads in (1, 4):
        got = rsmi.blake2b_host(msgs, digest_len, threads)
        assert got == [_ref(m, digest_len) for m in msgs], threads


def test_many_messages_many_threads():
    rng = np.random.default_rng(7)
    msgs = [rng.integers(0, 256, size=int(rng.integers(0, 3000)), dtype=np.uint8).tobytes() for _ in range(2000)]
    assert rsmi.blake2b_host(msgs, 32, 8) == [_ref(m, 32) for m in msgs]  # joined-buffer path (> 1024 msgs)
    assert rsmi.blake2b_host(msgs[:37], 64, 0) == [_ref(m, 64) for m in msgs[:37]]


def test_config1_message():
    """A config-1-sized serialized message (1 MiB blob + framing)."""
    m = np.random.default_rng(1).integers(0, 256, size=1048580 + 40, dtype=np.uint8).tobytes()
    assert rsmi.blake2b_host([m], 32)[0] == _ref(m, 32)


def test_errors():
    with pytest.raises(rsmi.RSError):
        rsmi.blake2b_host([b"x"], 0)
    with pytest.raises(rsmi.RSError):
        rsmi.blake2b_host([b"x"], 65)
