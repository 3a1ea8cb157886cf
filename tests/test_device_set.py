"""CPU: the device-set layer's host logic (include/rsmi.h rs_new_devices,
csrc/device_set.cpp) -- no compute calls.

north_star partitions stripes over the GPUs of one node ("stripes are
independent, so they are partitioned across the 8 GPUs of one node with no
collectives on the encode path"); rs_partition is the arithmetic every set
call uses to split stripes and messages into contiguous per-member ranges.
The GPU behaviour (bit-exact parts, batches and the spread reconstruct) is in
tests/test_gpu_device_set.py.
"""
import ctypes

import pytest

from conftest import gpu_available


@pytest.mark.parametrize("parts", [1, 2, 4, 8])
@pytest.mark.parametrize("units", [0, 1, 2, 3, 7, 8, 9, 64, 6553, 6553 * 8 + 5, 2**40 + 3])
def test_partition_tiles_in_order(units, parts):
    import rsmi
    ranges = [rsmi.partition(units, parts, p) for p in range(parts)]
    pos = 0
    for first, count in ranges:
        assert first == pos  # contiguous, in member order
        pos += count
    assert pos == units  # every unit exactly once
    sizes = [c for _, c in ranges]
    assert max(sizes) - min(sizes) <= 1  # balanced
    # first = units * part / parts, as include/rsmi.h documents
    assert all(f == units * p // parts for p, (f, _) in enumerate(ranges))


def test_partition_of_the_headline_over_8_gpus():
    """configs[3]: the 6,553 x 8 stripes of an 8-GPU run, 6,553 per GPU."""
    import rsmi
    assert [rsmi.partition(6553 * 8, 8, p) for p in range(8)] == [(6553 * p, 6553) for p in range(8)]


def test_partition_rejects_bad_arguments():
    import rsmi
    lib = rsmi.load()
    first, count = ctypes.c_size_t(), ctypes.c_size_t()
    for units, parts, part in ((10, 0, 0), (10, 2, 2), (10, 2, -1)):
        assert lib.rs_partition(units, parts, part, ctypes.byref(first), ctypes.byref(count)) == rsmi.RS_EINVAL
    assert lib.rs_partition(10, 2, 0, None, ctypes.byref(count)) == rsmi.RS_EINVAL


def test_new_devices_argument_errors_and_no_gpu():
    """rs_new_devices validates like NewFEC, then needs every listed device:
    without a gfx950 GPU it refuses (no CPU fallback)."""
    import rsmi
    lib = rsmi.load()
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.rs_new_devices(0, 4, devs, 2, ctypes.byref(h)) == rsmi.RS_EINVAL_KN
    assert lib.rs_new_devices(10, 14, devs, 0, ctypes.byref(h)) == rsmi.RS_EINVAL
    assert lib.rs_new_devices(10, 14, None, 2, ctypes.byref(h)) == rsmi.RS_EINVAL
    assert lib.rs_new_devices(10, 14, devs, 2, None) == rsmi.RS_EINVAL
    if not gpu_available():
        with pytest.raises(rsmi.RSError) as ei:
            rsmi.FEC(10, 14, devices=[0, 0])
        assert ei.value.code == rsmi.RS_EDEVICE


def test_set_entry_points_reject_null_context():
    import rsmi
    lib = rsmi.load()
    parts = (rsmi.StripePart * 1)()
    assert lib.rs_member_count(None) == rsmi.RS_EINVAL
    assert lib.rs_member(None, 0) is None
    assert lib.rs_encode_stripes_parts(None, parts, 16, 16) == rsmi.RS_EINVAL
    assert lib.rs_reconstruct_stripes_parts(None, parts, 16, 16, None) == rsmi.RS_EINVAL
    assert lib.rs_reconstruct_spread(None, None, None, 16, 1, None, None) == rsmi.RS_EINVAL
