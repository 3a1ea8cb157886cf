"""The C ABI driven from C (tests/capi/abi_check.c), the way the cgo shim
drives it: encode/decode of the config-1 blob vs the oracle, receive batching
from an arena, BLAKE2b known answers, error classes, 8 concurrent threads.
Built by __graft_entry__.build(); run on the GPU box.  Also the host-only
ThreadSanitizer / AddressSanitizer builds of the shared copy pool
(tests/capi/copypool_stress.cpp), which run on the CPU."""
import os
import subprocess

import pytest

from conftest import ROOT

BUILD = os.path.join(ROOT, "tests", "capi", "build")
BIN = os.path.join(BUILD, "abi_check")


def test_abi_check_builds():
    assert os.path.exists(BIN), "run __graft_entry__.build() (make -C tests/capi)"


@pytest.mark.gpu
def test_abi_check_runs_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_check: ok" in r.stdout


@pytest.mark.parametrize("spin_us,part_min", [("0", "0"), ("200", "65536")])
@pytest.mark.parametrize("variant,iters", [("copypool_tsan", 3), ("copypool_asan", 20)])
def test_copy_pool_concurrent_callers_under_sanitizer(variant, iters, spin_us, part_min):
    """Also with the workers' spin phase (RSMI_COPY_SPIN_US: the lock-free
    job counter they poll must not race the queue they then lock) and with
    64 KiB parts (RSMI_COPY_PART_MIN: many small hand-offs)."""
    exe = os.path.join(BUILD, variant)
    assert os.path.exists(exe), "run __graft_entry__.build() (make -C tests/capi)"
    env = dict(os.environ, RSMI_COPY_THREADS="8", RSMI_COPY_SPIN_US=spin_us)
    if part_min != "0":
        env["RSMI_COPY_PART_MIN"] = part_min
    r = subprocess.run([exe, str(iters), "8"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "copypool_stress: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr


def test_pattern_index_under_sanitizer():
    """The pattern cache's host index (csrc/pattern_index.cpp): the 8-at-a-time
    key builder against a byte loop for every n <= 256, and the open-addressing
    index against std::unordered_map across rehashes and clears (ASan/UBSan)."""
    exe = os.path.join(BUILD, "pattern_index_test")
    assert os.path.exists(exe), "run __graft_entry__.build() (make -C tests/capi)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pattern_index_test: ok" in r.stdout


def test_shard_wire_fuzz_under_sanitizer():
    """The Shard codec on peer input (tests/capi/wire_fuzz.cpp, ASan/UBSan):
    round trips, mutated and random encodings from exact-size buffers --
    no read past the input, views inside it, error codes negative."""
    exe = os.path.join(BUILD, "wire_fuzz")
    assert os.path.exists(exe), "run __graft_entry__.build() (make -C tests/capi)"
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wire_fuzz: ok" in r.stdout


def test_xcd_block_order_is_a_bijection():
    """csrc/xcd.hpp's block renumbering, host build under
    ASan/UBSan: a permutation of the grid for 165 (region, grid) sizes, each
    full group of 8 regions spread one region per XCD, in order, and the
    tail left in place."""
    exe = os.path.join(BUILD, "xcd_check")
    assert os.path.exists(exe), "run __graft_entry__.build() (make -C tests/capi)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cases ok" in r.stdout
