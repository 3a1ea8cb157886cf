"""Seeded random cases of the host-buffer C ABI against the oracle
(tools/fuzz_host_api.py): random codes, shard lengths from 1 byte past the
one-shot staging threshold, k..n shares in random order (Correct when more
than k, one corrupted share sometimes), survivors pageable / in an rs_arena /
mixed, dst pageable or engine-pinned.  Reference: Encode main.go:262,
Decode main.go:77."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import fuzz_host_api  # noqa: E402


@pytest.mark.parametrize("seed", [11, 12])
def test_host_api_random_cases(seed):
    st = fuzz_host_api.run(cases=60, seed=seed)
    assert st["failures"] == 0, st["first_failures"]
    assert st["encode"] == 60 and st["decode_k"] + st["decode_more"] == 60
    assert st["aliased"] > 0  # shares inside dst (round 6)
