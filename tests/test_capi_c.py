"""The C ABI driven from C (tests/capi/abi_check.c), the way the cgo shim
drives it: encode/decode of the config-1 blob vs the oracle, receive batching
from an arena, BLAKE2b known answers, error classes, 8 concurrent threads.
Built by __graft_entry__.build(); run on the GPU box."""
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "capi", "build", "abi_check")


def test_abi_check_builds():
    assert os.path.exists(BIN), "run __graft_entry__.build() (make -C tests/capi)"


@pytest.mark.gpu
def test_abi_check_runs_on_gpu():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_check: ok" in r.stdout
