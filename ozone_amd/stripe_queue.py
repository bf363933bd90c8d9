"""Writer-side stripe batching over libozec's ozec_stripe_queue_*.

ECKeyOutputStream (ECKeyOutputStream.java:114, :304, :501-543) encodes each stripe synchronously as soon as
its data cells are full.  A StripeQueue lets the writer hand stripes over and keep filling the next ones:
stripes are encoded in batches by one fused GPU launch, with copies overlapped across three batches.
Pinned cell buffers (host_alloc) are DMA'd directly; pageable ones go through pinned staging.
"""
import collections
import ctypes

import numpy as np

from . import _lib as L
from .checksum import ChecksumType
from .rawcoder import IllegalArgumentException, _raise_for


class PinnedBuffer:
    """Pinned host memory from ozec_host_alloc(_on), viewed as a uint8 numpy array (`.array`).  Its pages live on
    the NUMA node of `device` (default: the current device)."""

    def __init__(self, nbytes, device=None):
        self._p = ctypes.c_void_p()
        if device is None:
            rc = L.lib().ozec_host_alloc(nbytes, ctypes.byref(self._p))
        else:
            rc = L.lib().ozec_host_alloc_on(nbytes, device, ctypes.byref(self._p))
        if rc != L.OZEC_OK:
            _raise_for(rc)
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(self._p.value)) if nbytes else \
            np.zeros(0, np.uint8)

    def free(self):
        if self._p is not None and self._p.value:
            self.array = None
            L.lib().ozec_host_free(self._p)
        self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


def host_alloc(nbytes, device=None):
    return PinnedBuffer(nbytes, device)


def device_numa_node(device):
    """Host NUMA node closest to `device` (-1: unknown)."""
    n = ctypes.c_int()
    rc = L.lib().ozec_device_numa_node(device, ctypes.byref(n))
    if rc != L.OZEC_OK:
        _raise_for(rc)
    return n.value


def page_node(addr):
    """NUMA node of the (touched) page at host address `addr`, -1 if unknown."""
    n = ctypes.c_int()
    rc = L.lib().ozec_host_page_node(addr, ctypes.byref(n))
    if rc != L.OZEC_OK:
        _raise_for(rc)
    return n.value


def host_register(addr, nbytes, device):
    """Pin [addr, addr+nbytes) for DMA, its pages placed on `device`'s NUMA node (device < 0: no placement)."""
    rc = L.lib().ozec_host_register(addr, nbytes, device)
    if rc != L.OZEC_OK:
        _raise_for(rc)


def host_unregister(addr):
    rc = L.lib().ozec_host_unregister(addr)
    if rc != L.OZEC_OK:
        _raise_for(rc)


class StripeQueue:
    """Batched, asynchronous stripe encoding for one RawErasureEncoder."""

    def __init__(self, encoder, cell_len, stripes_per_batch=64, checksum_type=ChecksumType.NONE,
                 bytes_per_checksum=16384, big_endian=False):
        self._enc = encoder  # keeps the coder alive
        self._k = encoder.get_num_data_units()
        self._p = encoder.get_num_parity_units()
        # CRCs cover the coded units: k data + p parity (XOR codes one parity row)
        self._units = self._k + (1 if encoder._config.get_codec() == "xor" else self._p)
        self._bpc = bytes_per_checksum if int(checksum_type) != int(ChecksumType.NONE) else 0
        self._h = ctypes.c_void_p()
        rc = L.lib().ozec_stripe_queue_create(encoder._handle, cell_len, stripes_per_batch, int(checksum_type),
                                              bytes_per_checksum, 1 if big_endian else 0, ctypes.byref(self._h))
        if rc != L.OZEC_OK:
            _raise_for(rc)
        self._held = collections.deque()  # (ticket, buffers) kept alive until their stripe completes

    def submit(self, data, parity, length=None, crcs=None):
        """data: k uint8 arrays, parity: p uint8 arrays (written when the stripe completes), crcs: optional
        uint32 array of (k+p) * windows.  Returns the stripe's ticket."""
        if len(data) != self._k or len(parity) != self._p:
            raise IllegalArgumentException("Invalid inputs/outputs length")
        n = length if length is not None else data[0].size
        # the library DMA's n contiguous bytes from / into each address and memcpy's units * windows uint32
        # values into crcs, so every buffer must be exactly what it claims to be
        for a in list(data) + list(parity):
            if not isinstance(a, np.ndarray) or a.dtype != np.uint8 or not a.flags.c_contiguous:
                raise IllegalArgumentException("Invalid buffer: C-contiguous uint8 arrays are required")
            if a.size < n:
                raise IllegalArgumentException(f"Invalid buffer, not of length {n}")
        for a in parity:
            if not a.flags.writeable:
                raise IllegalArgumentException("Invalid buffer: parity buffers must be writeable")
        if crcs is not None:
            need = self._units * (-(-n // self._bpc)) if self._bpc else 0
            if (not isinstance(crcs, np.ndarray) or crcs.dtype not in (np.uint32, np.int32)
                    or not crcs.flags.c_contiguous or not crcs.flags.writeable or crcs.size < need):
                raise IllegalArgumentException(
                    f"Invalid crcs buffer: a writeable C-contiguous uint32 array of >= {need} elements is required")
        t = ctypes.c_uint64()
        rc = L.lib().ozec_stripe_queue_submit(self._h, L.ptr_array([a.ctypes.data for a in data]),
                                              L.ptr_array([a.ctypes.data for a in parity]), n,
                                              None if crcs is None else crcs.ctypes.data, ctypes.byref(t))
        if rc != L.OZEC_OK:
            _raise_for(rc)
        self._held.append((t.value, (list(data), list(parity), crcs)))
        return t.value

    def state(self):
        """(batches in flight, first ticket of the oldest in-flight batch or None, stripes in filling batches)."""
        n, t, f = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.c_size_t()
        rc = L.lib().ozec_stripe_queue_state(self._h, ctypes.byref(n), ctypes.byref(t), ctypes.byref(f))
        if rc != L.OZEC_OK:
            _raise_for(rc)
        return n.value, (None if t.value == (1 << 64) - 1 else t.value), f.value

    def flush(self):
        rc = L.lib().ozec_stripe_queue_flush(self._h)
        if rc != L.OZEC_OK:
            _raise_for(rc)

    def wait(self, ticket):
        """Block until every stripe up to and including `ticket` is complete."""
        rc = L.lib().ozec_stripe_queue_wait(self._h, ticket)
        if rc != L.OZEC_OK:
            _raise_for(rc)
        while self._held and self._held[0][0] <= ticket:
            self._held.popleft()

    def close(self):
        if self._h is not None and self._h.value:
            rc = L.lib().ozec_stripe_queue_free(self._h)
            self._h = None
            self._held.clear()
            if rc != L.OZEC_OK:
                _raise_for(rc)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass
