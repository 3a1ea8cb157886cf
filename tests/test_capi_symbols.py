"""CPU: the C-ABI library loads and exports every symbol include/rsmi.h
declares; the product library does not link or embed the oracle."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, gpu_available

HEADERS = [os.path.join(ROOT, "include", n) for n in ("rsmi.h", "rsmi_wire.h")]


def header_functions(headers=HEADERS):
    names = set()
    for hp in headers:
        src = open(hp).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(rs_[a-z_0-9]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_header_symbol():
    import rsmi
    lib = ctypes.CDLL(rsmi.LIB_PATH)
    names = header_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(rsmi.EXPORTS) == header_functions(HEADERS[:1])


def test_product_does_not_contain_oracle():
    import rsmi
    out = subprocess.run(["nm", "-D", rsmi.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in out
    ldd = subprocess.run(["ldd", rsmi.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd


def test_strerror_and_no_gpu_behaviour():
    import rsmi
    assert rsmi.strerror(rsmi.RS_EINVAL_KN) == "requires 1 <= k <= n <= 256"
    with pytest.raises(rsmi.RSError) as ei:
        rsmi.NewFEC(0, 4)
    assert ei.value.code == rsmi.RS_EINVAL_KN
    if not gpu_available():
        # No CPU fallback: without a gfx950 device the engine refuses to start.
        with pytest.raises(rsmi.RSError) as ei:
            rsmi.NewFEC(10, 14)
        assert ei.value.code == rsmi.RS_EDEVICE


def test_null_context_is_rejected_without_a_device():
    """Every host-API entry point that takes a context refuses a NULL one
    with RS_EINVAL before touching HIP (the cgo shim may pass a nil *FEC's
    context); callable on a CPU-only machine."""
    import ctypes
    import rsmi
    lib = rsmi.load()
    i32 = ctypes.c_int
    st = (i32 * 1)()
    ptrs = (ctypes.c_void_p * 1)(None)
    nums = (i32 * 1)(0)
    lens = (ctypes.c_size_t * 1)(0)
    out = ctypes.create_string_buffer(64)
    assert lib.rs_encode(None, None, 0, None) == rsmi.RS_EINVAL
    assert lib.rs_encode_batch(None, 1, ptrs, 10, ptrs, st) == rsmi.RS_EINVAL
    assert lib.rs_decode_batch(None, 1, nums, nums, ptrs, 10, ptrs, st) == rsmi.RS_EINVAL
    assert lib.rs_decode(None, nums, ptrs, 1, 10, out) == rsmi.RS_EINVAL
    assert lib.rs_blake2b_batch(None, 1, ptrs, lens, 32, out) == rsmi.RS_EINVAL
