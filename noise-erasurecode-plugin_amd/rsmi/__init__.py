"""ctypes binding of the MI355X Reed-Solomon engine (include/rsmi.h).

Mirrors the github.com/vivint/infectious API the reference plugin calls
(/root/reference/main.go:24 import, :73/:248 NewFEC, :262 Encode, :77 Decode,
:57-69/:254-258 Share + DeepCopy) so Python callers and the tests read like
the plugin.  The shared library lib/librsmi.so is built in-tree by
``__graft_entry__.build()`` (or ``make -C noise-erasurecode-plugin_amd/csrc``);
importing this module without it raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
# RSMI_LIB points at another build of the engine (same-box A/B runs of build variants).
LIB_PATH = os.environ.get("RSMI_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librsmi.so")

# rs_status codes (include/rsmi.h)
RS_OK = 0
RS_EINVAL_KN = -1
RS_ELEN_NOT_MULTIPLE = -2
RS_ENOT_ENOUGH = -3
RS_EBAD_SHARE_ID = -4
RS_ESINGULAR = -5
RS_ENO_SHARES = -6
RS_ESHARE_LEN = -7
RS_EINVAL = -8
RS_EDEVICE = -9
RS_ENOMEM = -10
RS_ETOO_MANY_ERRORS = -16

# Every symbol include/rsmi.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = (
    "rs_new", "rs_new_on_device", "rs_free", "rs_k", "rs_n", "rs_device",
    "rs_encode_matrix", "rs_strerror", "rs_encode", "rs_decode", "rs_decode_batch", "rs_encode_batch",
    "rs_encode_stripes", "rs_reconstruct_stripes", "rs_reconstruct_ptrs", "rs_pattern_count",
    "rs_pattern_evictions",
    "rs_prepare_patterns",
    "rs_pattern_rows",
    "rs_pinned_alloc", "rs_pinned_free", "rs_device_alloc", "rs_device_free",
    "rs_stream_sync", "rs_fill_splitmix", "rs_kernel_name",
    "rs_blake2b_batch", "rs_blake2b_device", "rs_blake2b", "rs_blake2b_host",
    "rs_stat", "rs_arena_new", "rs_arena_alloc", "rs_arena_put", "rs_arena_reset", "rs_arena_used", "rs_arena_free",
    "rs_new_devices", "rs_member_count", "rs_member", "rs_partition",
    "rs_encode_stripes_parts", "rs_reconstruct_stripes_parts", "rs_reconstruct_spread",
)


class StripePart(ctypes.Structure):
    """rs_stripe_part (include/rsmi.h): the stripes one member holds."""

    _fields_ = [("data", ctypes.c_void_p), ("data_stripe_stride", ctypes.c_size_t),
                ("parity", ctypes.c_void_p), ("parity_stripe_stride", ctypes.c_size_t),
                ("stripes", ctypes.c_size_t), ("stream", ctypes.c_void_p)]


class RSError(Exception):
    """Error from the engine; .code is the rs_status value."""

    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _lib().rs_strerror(code).decode() if _LIB is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class NotEnoughShares(RSError):
    """infectious NotEnoughShares (Rebuild/Correct with fewer than k shares)."""


_LIB: Optional[ctypes.CDLL] = None


def _lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                "(the engine has no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        u8p = ctypes.POINTER(ctypes.c_uint8)
        sig = {
            "rs_new": (i32, [i32, i32, ctypes.POINTER(vp)]),
            "rs_new_on_device": (i32, [i32, i32, i32, ctypes.POINTER(vp)]),
            "rs_free": (None, [vp]),
            "rs_k": (i32, [vp]),
            "rs_n": (i32, [vp]),
            "rs_device": (i32, [vp]),
            "rs_encode_matrix": (i32, [vp, u8p]),
            "rs_strerror": (ctypes.c_char_p, [i32]),
            "rs_kernel_name": (ctypes.c_char_p, [vp, i32]),
            "rs_encode": (i32, [vp, vp, sz, vp]),
            "rs_decode": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(vp), i32, sz, vp]),
            "rs_decode_batch": (i32, [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                      ctypes.POINTER(vp), sz, ctypes.POINTER(vp), ctypes.POINTER(i32)]),
            "rs_encode_batch": (i32, [vp, i32, ctypes.POINTER(vp), sz, ctypes.POINTER(vp), ctypes.POINTER(i32)]),
            "rs_encode_stripes": (i32, [vp, vp, sz, vp, sz, sz, sz, sz, vp]),
            "rs_reconstruct_stripes": (i32, [vp, vp, sz, vp, sz, sz, sz, sz, vp, vp]),
            "rs_reconstruct_ptrs": (i32, [vp, vp, sz, sz, vp, vp]),
            "rs_pattern_count": (i32, [vp]),
            "rs_pattern_evictions": (ctypes.c_int64, [vp]),
            "rs_prepare_patterns": (i32, [vp, i32, vp]),
            "rs_pattern_rows": (i32, [vp, vp, vp, ctypes.POINTER(i32)]),
            "rs_pinned_alloc": (vp, [sz]),
            "rs_pinned_free": (None, [vp]),
            "rs_device_alloc": (i32, [vp, sz, ctypes.POINTER(vp)]),
            "rs_device_free": (i32, [vp, vp]),
            "rs_stream_sync": (i32, [vp, vp]),
            "rs_fill_splitmix": (i32, [vp, vp, sz, ctypes.c_uint64, vp]),
            "rs_stat": (ctypes.c_int64, [vp, i32]),
            "rs_arena_new": (vp, [sz]),
            "rs_arena_alloc": (vp, [vp, sz]),
            "rs_arena_put": (vp, [vp, vp, sz]),
            "rs_arena_reset": (None, [vp]),
            "rs_arena_used": (sz, [vp]),
            "rs_arena_free": (None, [vp]),
            "rs_shard_unmarshal_arena": (i32, [vp, sz, vp, vp]),
            "rs_blake2b_batch": (i32, [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp]),
            "rs_blake2b_device": (i32, [vp, i32, vp, vp, vp, i32, vp, vp]),
            "rs_blake2b": (i32, [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp, ctypes.POINTER(i32)]),
            "rs_blake2b_host": (i32, [i32, ctypes.POINTER(vp), ctypes.POINTER(sz), i32, vp, i32]),
            "rs_new_devices": (i32, [i32, i32, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]),
            "rs_member_count": (i32, [vp]),
            "rs_member": (vp, [vp, i32]),
            "rs_partition": (i32, [sz, i32, i32, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
            "rs_encode_stripes_parts": (i32, [vp, ctypes.POINTER(StripePart), sz, sz]),
            "rs_reconstruct_stripes_parts": (i32, [vp, ctypes.POINTER(StripePart), sz, sz, vp]),
            "rs_reconstruct_spread": (i32, [vp, vp, vp, sz, sz, vp, vp]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("RSMI_LIB") and not hasattr(lib, name):
                continue  # an older build selected for an A/B run
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def load() -> ctypes.CDLL:
    """The loaded engine library (raises ImportError if it was not built)."""
    return _lib()


def _check(code: int, what: str) -> None:
    if code == RS_OK:
        return
    if code == RS_ENOT_ENOUGH:
        raise NotEnoughShares(code, what)
    raise RSError(code, what)


@dataclass
class Share:
    """infectious.Share{Number int; Data []byte} (main.go:57-69, :254-258)."""

    Number: int
    Data: bytes

    def DeepCopy(self) -> "Share":
        return Share(self.Number, bytes(self.Data))


def partition(units: int, parts: int, part: int):
    """rs_partition: (first, count) of part `part` of `units` split into
    `parts` contiguous ranges."""
    first, count = ctypes.c_size_t(), ctypes.c_size_t()
    _check(_lib().rs_partition(units, parts, part, ctypes.byref(first), ctypes.byref(count)), "rs_partition")
    return first.value, count.value


class FEC:
    """Handle of an rs_ctx: the engine-side infectious *FEC for (k, n).
    devices=[...] builds a device-set context (rs_new_devices): one member
    per listed GPU, every call spread over them."""

    def __init__(self, k: int, n: int, device: Optional[int] = None,
                 devices: Optional[Sequence[int]] = None, _handle=None):
        lib = _lib()
        self.k = k
        self.n = n
        self._owner = _handle is None
        if _handle is not None:  # a member of a device set: owned by the set
            self._h = ctypes.c_void_p(_handle)
            return
        h = ctypes.c_void_p()
        if devices is not None:
            devs = (ctypes.c_int * max(len(devices), 1))(*devices)
            code = lib.rs_new_devices(k, n, devs, len(devices), ctypes.byref(h))
        elif device is None:
            code = lib.rs_new(k, n, ctypes.byref(h))
        else:
            code = lib.rs_new_on_device(k, n, device, ctypes.byref(h))
        _check(code, f"NewFEC({k}, {n})")
        self._h = h

    # -- device sets (rs_new_devices) --------------------------------------------
    def member_count(self) -> int:
        return _lib().rs_member_count(self._h)

    def member(self, i: int) -> "FEC":
        """Member i (a single-device context owned by the set; self for i = 0
        of a single-device context)."""
        h = _lib().rs_member(self._h, i)
        if not h:
            raise RSError(RS_EINVAL, f"rs_member({i})")
        m = FEC(self.k, self.n, _handle=h)
        m._set = self  # keep the set alive while the member is used
        return m

    def encode_stripes_parts(self, parts: Sequence[tuple], pitch: int, shard_len: int) -> None:
        """rs_encode_stripes_parts: parts[i] = (data_ptr, data_stride,
        parity_ptr, parity_stride, stripes, stream) on member i's device."""
        arr = (StripePart * max(len(parts), 1))(*[StripePart(*p) for p in parts])
        _check(_lib().rs_encode_stripes_parts(self._h, arr, pitch, shard_len), "rs_encode_stripes_parts")

    def reconstruct_stripes_parts(self, parts: Sequence[tuple], pitch: int, shard_len: int,
                                  erased: bytes) -> None:
        arr = (StripePart * max(len(parts), 1))(*[StripePart(*p) for p in parts])
        buf = ctypes.c_char_p(bytes(erased))
        _check(_lib().rs_reconstruct_stripes_parts(self._h, arr, pitch, shard_len,
                                                   ctypes.cast(buf, ctypes.c_void_p)),
               "rs_reconstruct_stripes_parts")

    def reconstruct_spread(self, shard_ptrs: Sequence[int], owner: Sequence[int], shard_len: int,
                           stripes: int, erased: bytes, streams: Optional[Sequence[int]] = None) -> None:
        """rs_reconstruct_spread: shard i of stripe s at device address
        shard_ptrs[s * n + i] on any member's GPU; owner[s] reconstructs."""
        import numpy as np
        if len(erased) != stripes * self.n or len(shard_ptrs) != stripes * self.n or len(owner) != stripes:
            raise RSError(RS_EINVAL, "reconstruct_spread: table sizes")
        tab = np.ascontiguousarray(np.asarray(shard_ptrs, dtype=np.uint64))
        own = np.ascontiguousarray(np.asarray(owner, dtype=np.int32))
        buf = ctypes.c_char_p(bytes(erased))
        st = None
        if streams is not None:
            st = (ctypes.c_void_p * max(len(streams), 1))(*[x or None for x in streams])
        _check(_lib().rs_reconstruct_spread(self._h, tab.ctypes.data, own.ctypes.data, shard_len, stripes,
                                            ctypes.cast(buf, ctypes.c_void_p), st), "rs_reconstruct_spread")

    # -- infectious accessors -------------------------------------------------
    def Required(self) -> int:
        return self.k

    def Total(self) -> int:
        return self.n

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def close(self) -> None:
        if getattr(self, "_h", None):
            if getattr(self, "_owner", True):
                _lib().rs_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def kernel_name(self, which: int = 0) -> str:
        """Kernel serving encode (0) or reconstruct (1): diagnostics."""
        return _lib().rs_kernel_name(self._h, which).decode()

    def matrix(self) -> bytes:
        buf = (ctypes.c_uint8 * (self.n * self.k))()
        _check(_lib().rs_encode_matrix(self._h, buf), "rs_encode_matrix")
        return bytes(buf)

    # -- (*FEC).Encode (main.go:262) ------------------------------------------
    def Encode(self, input: bytes, output: Callable[[Share], None]) -> None:
        """Calls output(Share) for shares 0..n-1 in order; like infectious,
        data shares are views of input and the parity buffer is reused
        between callbacks (callers DeepCopy, main.go:255-258)."""
        data = bytes(input)
        if len(data) % self.k != 0:
            raise RSError(RS_ELEN_NOT_MULTIPLE, "Encode")
        S = len(data) // self.k
        m = self.n - self.k
        parity = bytearray(m * S)
        if S and m:
            src = ctypes.c_char_p(data)
            dst = (ctypes.c_char * len(parity)).from_buffer(parity)
            _check(_lib().rs_encode(self._h, ctypes.cast(src, ctypes.c_void_p), len(data),
                                    ctypes.cast(dst, ctypes.c_void_p)), "Encode")
        view = memoryview(data)
        for i in range(self.k):
            output(Share(i, view[i * S:(i + 1) * S]))
        pv = memoryview(parity)
        for i in range(m):
            output(Share(self.k + i, pv[i * S:(i + 1) * S]))

    def encode_parity(self, input: bytes) -> bytes:
        """Parity shares k..n-1 concatenated (rs_encode)."""
        out: List[bytes] = []
        self.Encode(input, lambda s: out.append(bytes(s.Data)) if s.Number >= self.k else None)
        return b"".join(out)

    # -- (*FEC).Decode (main.go:77) -------------------------------------------
    def Decode(self, dst: Optional[bytearray], shares: List[Share]) -> bytes:
        """Returns the k*S-byte original.  Sorts `shares` in place by Number,
        as infectious does to the caller's slice."""
        cnt = len(shares)
        S = len(shares[0].Data) if cnt else 0
        for s in shares:
            if len(s.Data) != S:
                raise RSError(RS_ESHARE_LEN, "Decode")
        nums = (ctypes.c_int * max(cnt, 1))(*[s.Number for s in shares])
        keep = [bytes(s.Data) for s in shares]
        ptrs = (ctypes.c_void_p * max(cnt, 1))(
            *[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value for b in keep])
        out = bytearray(self.k * S)
        outp = (ctypes.c_char * max(len(out), 1)).from_buffer(out) if out else None
        code = _lib().rs_decode(self._h, nums, ptrs, cnt, S,
                                ctypes.cast(outp, ctypes.c_void_p) if outp is not None else None)
        _check(code, "Decode")
        # mirror the in-place sort
        order = sorted(range(cnt), key=lambda i: (shares[i].Number, i))
        shares[:] = [shares[i] for i in order]
        if dst is not None and len(dst) >= len(out):
            dst[:len(out)] = out
            return bytes(dst[:len(out)])
        return bytes(out)

    def DecodeBatch(self, messages: List[List[Share]]):
        """rs_decode_batch: decode many messages in one GPU pass.  Returns
        (outputs, statuses); outputs[b] is None where statuses[b] != 0."""
        B = len(messages)
        S = len(messages[0][0].Data) if B and messages[0] else 0
        counts = (ctypes.c_int * max(B, 1))(*[len(msg) for msg in messages])
        flat = [s for msg in messages for s in msg]
        for s in flat:
            if len(s.Data) != S:
                raise RSError(RS_ESHARE_LEN, "DecodeBatch")
        nums = (ctypes.c_int * max(len(flat), 1))(*[s.Number for s in flat])
        keep = [bytes(s.Data) for s in flat]
        ptrs = (ctypes.c_void_p * max(len(flat), 1))(
            *[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value for b in keep])
        outs = [bytearray(max(self.k * S, 1)) for _ in range(B)]
        outp = (ctypes.c_void_p * max(B, 1))(
            *[ctypes.addressof((ctypes.c_char * max(len(o), 1)).from_buffer(o)) for o in outs])
        st = (ctypes.c_int * max(B, 1))()
        _lib().rs_decode_batch(self._h, B, counts, nums, ptrs, S, outp, st)
        return ([bytes(o[:self.k * S]) if st[b] == RS_OK else None for b, o in enumerate(outs)],
                [st[b] for b in range(B)])

    def EncodeBatch(self, inputs: List[bytes]):
        """rs_encode_batch: the parity of many equal-length messages in one
        GPU pass (send-side batching).  Returns (parities, statuses);
        parities[b] is the m*S parity bytes (rs_encode's layout) or None where
        statuses[b] != 0."""
        B = len(inputs)
        L = len(inputs[0]) if B else 0
        for x in inputs:
            if len(x) != L:
                raise RSError(RS_EINVAL, "EncodeBatch: messages of unequal length")
        m = self.n - self.k
        P = (L // self.k) * m if L % self.k == 0 else 0
        keep = [bytes(x) for x in inputs]
        ins = (ctypes.c_void_p * max(B, 1))(
            *[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value for b in keep])
        outs = [bytearray(max(P, 1)) for _ in range(B)]
        outp = (ctypes.c_void_p * max(B, 1))(
            *[ctypes.addressof((ctypes.c_char * len(o)).from_buffer(o)) for o in outs])
        st = (ctypes.c_int * max(B, 1))()
        _lib().rs_encode_batch(self._h, B, ins, L, outp, st)
        return ([bytes(o[:P]) if st[b] == RS_OK else None for b, o in enumerate(outs)],
                [st[b] for b in range(B)])

    # -- device-resident batched API -------------------------------------------
    def encode_stripes(self, data_ptr: int, data_stride: int, parity_ptr: int,
                       parity_stride: int, pitch: int, shard_len: int, stripes: int,
                       stream: int = 0) -> None:
        _check(_lib().rs_encode_stripes(self._h, data_ptr, data_stride, parity_ptr,
                                        parity_stride, pitch, shard_len, stripes,
                                        stream or None), "rs_encode_stripes")

    def reconstruct_stripes(self, data_ptr: int, data_stride: int, parity_ptr: int,
                            parity_stride: int, pitch: int, shard_len: int, stripes: int,
                            erased: bytes, stream: int = 0) -> None:
        if len(erased) != stripes * self.n:
            raise RSError(RS_EINVAL, "erased must hold stripes*n flags")
        buf = ctypes.c_char_p(bytes(erased))
        _check(_lib().rs_reconstruct_stripes(self._h, data_ptr, data_stride, parity_ptr,
                                             parity_stride, pitch, shard_len, stripes,
                                             ctypes.cast(buf, ctypes.c_void_p), stream or None),
               "rs_reconstruct_stripes")

    def reconstruct_ptrs(self, shard_ptrs_dev: int, shard_len: int, stripes: int, erased: bytes,
                         stream: int = 0) -> None:
        """rs_reconstruct_ptrs: shard i of stripe s at the device address in
        the device array shard_ptrs_dev[s * n + i].  Every address must be
        16-byte aligned (the kernels move 16-byte vectors; rsmi.h), e.g. rows
        of a pool whose row pitch is a multiple of 16."""
        if len(erased) != stripes * self.n:
            raise RSError(RS_EINVAL, "erased must hold stripes*n flags")
        buf = ctypes.c_char_p(bytes(erased))
        _check(_lib().rs_reconstruct_ptrs(self._h, shard_ptrs_dev, shard_len, stripes,
                                          ctypes.cast(buf, ctypes.c_void_p), stream or None),
               "rs_reconstruct_ptrs")

    def pattern_count(self) -> int:
        return _lib().rs_pattern_count(self._h)

    (STAT_PATTERNS, STAT_EVICTIONS, STAT_BATCHES_IN_PLACE, STAT_BATCHES_STAGED, STAT_LEASES,
     STAT_ENCODES_IN_PLACE, STAT_DECODES_IN_PLACE, STAT_REC_STRIPES_TABLE, STAT_REC_STRIPES_SYNDROME,
     STAT_ENCODE_BATCHES, STAT_MAILBOX_CALLS, STAT_MAILBOX_RECOVERED) = range(12)

    def stat(self, which: int) -> int:
        return _lib().rs_stat(self._h, which)

    def pattern_evictions(self) -> int:
        return _lib().rs_pattern_evictions(self._h)

    def pattern_rows(self, erased: bytes):
        """(rows bytes m*k, count) the engine uses for this erasure pattern."""
        m = self.n - self.k
        buf = (ctypes.c_uint8 * max(m * self.k, 1))()
        cnt = ctypes.c_int()
        flags = ctypes.c_char_p(bytes(erased))
        _check(_lib().rs_pattern_rows(self._h, ctypes.cast(flags, ctypes.c_void_p),
                                      ctypes.cast(buf, ctypes.c_void_p), ctypes.byref(cnt)),
               "rs_pattern_rows")
        return bytes(buf)[:m * self.k], cnt.value

    def prepare_patterns(self, max_erasures: int, stream: int = 0) -> None:
        _check(_lib().rs_prepare_patterns(self._h, max_erasures, stream or None),
               "rs_prepare_patterns")

    def fill_splitmix(self, dev_ptr: int, nbytes: int, seed: int, stream: int = 0) -> None:
        _check(_lib().rs_fill_splitmix(self._h, dev_ptr, nbytes, seed & (2**64 - 1),
                                       stream or None), "rs_fill_splitmix")

    # -- signature hashing (blake2b policy, main.go:38-41, :219-223, :82-89) ----
    def blake2b_batch(self, messages: Sequence[bytes], digest_len: int = 32) -> List[bytes]:
        """BLAKE2b digests of many host messages in one GPU launch."""
        if not messages:
            return []
        keep, ptrs, lens = _message_table(messages)
        out = ctypes.create_string_buffer(len(messages) * digest_len)
        _check(_lib().rs_blake2b_batch(self._h, len(messages), ptrs, lens, digest_len,
                                       ctypes.cast(out, ctypes.c_void_p)), "rs_blake2b_batch")
        return _split(out.raw, len(messages), digest_len)

    def blake2b(self, messages: Sequence[bytes], digest_len: int = 32):
        """The hash policy (rs_blake2b): host CPU for one message or a batch
        whose longest chain dominates, the GPU kernel otherwise.  Returns
        (digests, where) with where 0 = host, 1 = GPU."""
        if not messages:
            return [], 0
        keep, ptrs, lens = _message_table(messages)
        out = ctypes.create_string_buffer(len(messages) * digest_len)
        where = ctypes.c_int(0)
        _check(_lib().rs_blake2b(self._h, len(messages), ptrs, lens, digest_len,
                                 ctypes.cast(out, ctypes.c_void_p), ctypes.byref(where)), "rs_blake2b")
        return _split(out.raw, len(messages), digest_len), where.value

    def blake2b_device(self, count: int, ptrs_dev: int, lens_dev: int, order_dev: int,
                       digest_len: int, out_dev: int, stream: int = 0) -> None:
        _check(_lib().rs_blake2b_device(self._h, count, ptrs_dev, lens_dev, order_dev or None,
                                        digest_len, out_dev, stream or None), "rs_blake2b_device")

    def sync(self, stream: int = 0) -> None:
        _check(_lib().rs_stream_sync(self._h, stream or None), "rs_stream_sync")


class Arena:
    """rs_arena: engine-pinned receive memory.  Shard bytes placed here (put,
    or the wire codec's rs_shard_unmarshal_arena) are read in place over
    PCIe by rs_decode_batch's kernel."""

    def __init__(self, nbytes: int):
        self._a = _lib().rs_arena_new(nbytes)
        if not self._a:
            raise RSError(RS_ENOMEM, "rs_arena_new")

    def put(self, data: bytes) -> int:
        """Copies data into a fresh 16-byte aligned slot (rs_arena_put:
        streaming stores, as rs_shard_unmarshal_arena); returns its address."""
        buf = bytes(data)
        p = _lib().rs_arena_put(self._a, buf, len(buf))
        if not p:
            raise RSError(RS_ENOMEM, "rs_arena_put")
        return p

    def used(self) -> int:
        return _lib().rs_arena_used(self._a)

    def reset(self) -> None:
        _lib().rs_arena_reset(self._a)

    def free(self) -> None:
        if getattr(self, "_a", None):
            _lib().rs_arena_free(self._a)
            self._a = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _message_table(messages: Sequence[bytes]):
    """(keep-alive, pointer array, length array) of host messages for the
    hash entry points: one pointer per message when there are few or large
    ones (no Python-side copy), pointers into one joined buffer otherwise."""
    import numpy as np
    cnt = len(messages)
    lens_np = np.fromiter((len(mm) for mm in messages), dtype=np.uint64, count=cnt)
    if cnt <= 1024 or int(lens_np.sum()) > (64 << 20):
        keep = [bytes(mm) for mm in messages]
        ptr_np = np.fromiter((ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value or 0 for b in keep),
                             dtype=np.uint64, count=cnt)
    else:
        keep = b"".join(bytes(mm) for mm in messages)
        base = ctypes.cast(ctypes.c_char_p(keep), ctypes.c_void_p).value or 0
        offs = np.zeros(cnt, dtype=np.uint64)
        np.cumsum(lens_np[:-1], out=offs[1:])
        ptr_np = (offs + np.uint64(base)).astype(np.uint64)
    keep = (keep, ptr_np, lens_np)
    return (keep, ptr_np.ctypes.data_as(ctypes.POINTER(ctypes.c_void_p)),
            lens_np.ctypes.data_as(ctypes.POINTER(ctypes.c_size_t)))


def _split(raw: bytes, cnt: int, digest_len: int) -> List[bytes]:
    return [raw[i * digest_len:(i + 1) * digest_len] for i in range(cnt)]


def blake2b_host(messages: Sequence[bytes], digest_len: int = 32, threads: int = 0) -> List[bytes]:
    """rs_blake2b_host: BLAKE2b on the host CPU (no context, no GPU)."""
    if not messages:
        return []
    keep, ptrs, lens = _message_table(messages)
    out = ctypes.create_string_buffer(len(messages) * digest_len)
    _check(_lib().rs_blake2b_host(len(messages), ptrs, lens, digest_len, ctypes.cast(out, ctypes.c_void_p),
                                  threads), "rs_blake2b_host")
    return _split(out.raw, len(messages), digest_len)


def NewFEC(k: int, n: int) -> FEC:
    """infectious.NewFEC(k, n) (main.go:73, :248)."""
    return FEC(k, n)


def strerror(code: int) -> str:
    return _lib().rs_strerror(code).decode()
