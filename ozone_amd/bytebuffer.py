"""Minimal java.nio.ByteBuffer / ECChunk mirror for the host-side coder API.

The reference's buffer contract (RawErasureEncoder.java:66-97, ByteBufferEncodingState.java:36-109) is
defined in terms of position/limit/remaining, heap vs direct buffers and arrayOffset; the Python coder
classes follow it exactly, so the parity tests can be written like TestRawCoderBase/TestCoderBase.
Memory is host memory either way (numpy); "direct" only changes the isDirect() flag the validators check.
"""
import numpy as np


class ByteBuffer:
    __slots__ = ("_hb", "_off", "_cap", "_pos", "_lim", "_direct", "_readonly")

    def __init__(self, backing, offset, capacity, direct, position=0, limit=None, readonly=False):
        self._hb = backing
        self._off = offset
        self._cap = capacity
        self._pos = position
        self._lim = capacity if limit is None else limit
        self._direct = direct
        self._readonly = readonly

    # ---- factories ---------------------------------------------------------------------------
    @staticmethod
    def allocate(n):
        return ByteBuffer(np.zeros(n, np.uint8), 0, n, False)

    @staticmethod
    def allocate_direct(n):
        return ByteBuffer(np.zeros(n, np.uint8), 0, n, True)

    @staticmethod
    def wrap(array, offset=0, length=None):
        """ByteBuffer.wrap(byte[] array, int offset, int length): position=offset, limit=offset+length."""
        if isinstance(array, (bytes, bytearray, memoryview)):
            array = np.frombuffer(bytearray(array), np.uint8)
        array = np.asarray(array)
        # a Java byte[] is one contiguous run of bytes: the GPU path DMA's address() as such, so a strided view
        # or a wider dtype would read (and, as an output, write) the wrong memory
        if array.dtype != np.uint8 or array.ndim != 1 or not array.flags.c_contiguous:
            raise TypeError("ByteBuffer.wrap needs a 1-D C-contiguous uint8 array")
        n = array.size if length is None else length
        return ByteBuffer(array, 0, array.size, False, position=offset, limit=offset + n)

    # ---- java.nio.Buffer -----------------------------------------------------------------------
    def position(self, p=None):
        if p is None:
            return self._pos
        if p < 0 or p > self._lim:
            raise ValueError("newPosition > limit")
        self._pos = p
        return self

    def limit(self, lim=None):
        if lim is None:
            return self._lim
        if lim < 0 or lim > self._cap:
            raise ValueError("newLimit > capacity")
        self._lim = lim
        self._pos = min(self._pos, lim)
        return self

    def capacity(self):
        return self._cap

    def remaining(self):
        return max(0, self._lim - self._pos)

    def has_remaining(self):
        return self._pos < self._lim

    def is_direct(self):
        return self._direct

    def has_array(self):
        return not self._direct and not self._readonly

    def array(self):
        if self._direct:
            raise TypeError("UnsupportedOperationException: direct buffer has no array")
        return self._hb

    def array_offset(self):
        return self._off

    def flip(self):
        self._lim = self._pos
        self._pos = 0
        return self

    def clear(self):
        self._pos = 0
        self._lim = self._cap
        return self

    def rewind(self):
        self._pos = 0
        return self

    def slice(self):
        return ByteBuffer(self._hb, self._off + self._pos, self.remaining(), self._direct, readonly=self._readonly)

    def duplicate(self):
        return ByteBuffer(self._hb, self._off, self._cap, self._direct, self._pos, self._lim, self._readonly)

    def as_read_only_buffer(self):
        return ByteBuffer(self._hb, self._off, self._cap, self._direct, self._pos, self._lim, True)

    def is_read_only(self):
        return self._readonly

    # ---- data access ---------------------------------------------------------------------------
    def view(self):
        """numpy view of [position, limit) -- no copy."""
        return self._hb[self._off + self._pos:self._off + self._lim]

    def address(self):
        """host address of position() (array + arrayOffset + position for heap buffers)."""
        return self._hb.ctypes.data + self._off + self._pos

    def get(self, index=None):
        if index is None:
            v = int(self._hb[self._off + self._pos])
            self._pos += 1
            return v
        return int(self._hb[self._off + index])

    def put(self, data, index=None):
        if self._readonly:
            raise TypeError("ReadOnlyBufferException")
        if index is not None:
            self._hb[self._off + index] = data
            return self
        a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        if a.size > self.remaining():
            raise ValueError("BufferOverflowException")
        self._hb[self._off + self._pos:self._off + self._pos + a.size] = a
        self._pos += a.size
        return self


class ECChunk:
    """ECChunk (EC/ECChunk.java:25-113): a ByteBuffer plus the isAllZero flag."""

    def __init__(self, buffer, offset=None, length=None, all_zero=False):
        if isinstance(buffer, ByteBuffer):
            if offset is not None:  # ECChunk(ByteBuffer, int offset, int len): slice (ECChunk.java:41-49)
                tmp = buffer.duplicate()
                tmp.position(offset)
                tmp.limit(offset + length)
                buffer = tmp.slice()
        else:  # ECChunk(byte[] buffer[, offset, len])
            buffer = ByteBuffer.wrap(buffer, offset or 0, length)
        self.buffer = buffer
        self.all_zero = all_zero

    def get_buffer(self):
        return self.buffer

    def is_all_zero(self):
        return self.all_zero

    @staticmethod
    def to_buffers(chunks):
        """ECChunk.toBuffers / CoderUtil.toBuffers (CoderUtil.java:107-124): zero chunks flagged isAllZero."""
        out = []
        for c in chunks:
            if c is None:
                out.append(None)
                continue
            b = c.get_buffer()
            if c.is_all_zero():
                b.view()[:] = 0
            out.append(b)
        return out
