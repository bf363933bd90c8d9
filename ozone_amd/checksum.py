"""Chunk checksums on the GPU behind the reference's Checksum API.

Mirrors hadoop-hdds/common (CM/ = .../org/apache/hadoop/ozone/common/):
  Checksum.computeChecksum / verifyChecksum   CM/Checksum.java:106-297
  ChecksumData.verifyChecksumDataMatches      CM/ChecksumData.java:118-150
  ChecksumByteBuffer (update/getValue/reset)  CM/ChecksumByteBuffer.java:32-44
  ChecksumType {NONE=1, CRC32=2, CRC32C=3, SHA256=4, MD5=5}  DatanodeClientProtocol.proto:422-434
CRC32/CRC32C windows are computed by libozec.so on the GPU (one CRC per bytesPerChecksum window, last window
short, stored as the 4 big-endian bytes of (int)getValue() -- Checksum.int2ByteString, Checksum.java:59-70).
SHA256/MD5 are outside the GPU scope of this build (BASELINE.json north_star names CRC32/CRC32C); they are
delegated to hashlib exactly as the reference delegates them to MessageDigest (Checksum.java:42-57).
"""
import ctypes
import enum
import hashlib

import numpy as np

from . import _lib as L
from .bytebuffer import ByteBuffer
from .rawcoder import IOException, _dev_ptr, _stream_ptr


class ChecksumType(enum.IntEnum):
    NONE = 1
    CRC32 = 2
    CRC32C = 3
    SHA256 = 4
    MD5 = 5


class OzoneChecksumException(IOException):
    """OzoneChecksumException (CM/OzoneChecksumException.java)."""

    def __init__(self, msg_or_index):
        if isinstance(msg_or_index, int):
            super().__init__(f"Checksum mismatch at index {msg_or_index}")
            self.index = msg_or_index
        else:
            super().__init__(msg_or_index)
            self.index = None


def int2bytes(n):
    """Checksum.int2ByteString: Guava Ints.toByteArray -> 4 big-endian bytes."""
    return int(n & 0xFFFFFFFF).to_bytes(4, "big")


def _as_u8(data):
    if isinstance(data, ByteBuffer):
        return np.ascontiguousarray(data.view())
    if isinstance(data, (list, tuple)):  # List<ByteString>: ChunkBuffer over a buffer list (windows may span)
        parts = [np.frombuffer(bytes(x), np.uint8) for x in data]
        return np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1), np.uint8)
    return np.frombuffer(bytes(data), np.uint8)


def crc_windows(checksum_type, data, bytes_per_checksum):
    """uint32 array of (int)getValue() per window, computed on the GPU."""
    a = _as_u8(data)
    nwin = (a.size + bytes_per_checksum - 1) // bytes_per_checksum if bytes_per_checksum > 0 else 0
    out = np.zeros(max(1, nwin), np.uint32)
    rc = L.lib().ozec_checksum_windows(int(checksum_type), a.ctypes.data, a.size, bytes_per_checksum,
                                       out.ctypes.data, 0)
    if rc != L.OZEC_OK:
        raise OzoneChecksumException(L.last_error())
    return out[:nwin]


class ChecksumData:
    """ChecksumData (CM/ChecksumData.java:35-193)."""

    def __init__(self, checksum_type, bytes_per_checksum, checksums=None):
        self.type = ChecksumType(checksum_type)
        self.bytes_per_checksum = bytes_per_checksum
        self.checksums = list(checksums or [])

    def get_checksum_type(self):
        return self.type

    def get_bytes_per_checksum(self):
        return self.bytes_per_checksum

    def get_checksums(self):
        return self.checksums

    def verify_checksum_data_matches(self, that, start_index):
        if len(self.checksums) == 0:
            raise OzoneChecksumException("Original checksumData has no checksums")
        if len(that.checksums) == 0:
            raise OzoneChecksumException("Computed checksumData has no checksums")
        n = len(that.checksums)
        for i in range(n):
            if start_index + i >= len(self.checksums):
                raise OzoneChecksumException(
                    f"Computed checksum has {n} number of checksums. Original checksum has "
                    f"{len(self.checksums) - start_index} number of checksums starting from index {start_index}")
            if self.checksums[start_index + i] != that.checksums[i]:
                raise OzoneChecksumException(i)
        return True

    def __eq__(self, other):
        return (isinstance(other, ChecksumData) and self.type == other.type
                and self.bytes_per_checksum == other.bytes_per_checksum and self.checksums == other.checksums)

    def __repr__(self):
        return f"ChecksumData(type={self.type.name}, bpc={self.bytes_per_checksum}, n={len(self.checksums)})"


class Checksum:
    """Checksum (CM/Checksum.java:42-306). Not thread safe, like the reference (:40)."""

    def __init__(self, checksum_type, bytes_per_checksum):
        self.checksum_type = ChecksumType(checksum_type)
        self.bytes_per_checksum = bytes_per_checksum

    def compute_checksum(self, data, off=None, length=None):
        if self.checksum_type == ChecksumType.NONE:
            return ChecksumData(self.checksum_type, self.bytes_per_checksum)
        a = _as_u8(data)
        if off is not None:
            a = a[off:off + (a.size - off if length is None else length)]
        bpc = self.bytes_per_checksum
        if self.checksum_type in (ChecksumType.CRC32, ChecksumType.CRC32C):
            vals = crc_windows(self.checksum_type, a, bpc)
            return ChecksumData(self.checksum_type, bpc, [int2bytes(v) for v in vals])
        algo = "sha256" if self.checksum_type == ChecksumType.SHA256 else "md5"
        sums = [hashlib.new(algo, a[o:o + bpc].tobytes()).digest() for o in range(0, a.size, bpc)]
        return ChecksumData(self.checksum_type, bpc, sums)

    @staticmethod
    def verify_checksum(data, checksum_data, start_index=0):
        if checksum_data.get_checksum_type() == ChecksumType.NONE:
            return True
        computed = Checksum(checksum_data.get_checksum_type(),
                            checksum_data.get_bytes_per_checksum()).compute_checksum(data)
        return checksum_data.verify_checksum_data_matches(computed, start_index)


class ChecksumByteBuffer:
    """Streaming CRC (ChecksumByteBuffer, CM/ChecksumByteBuffer.java:32-44) backed by the GPU.

    update() sends the buffer to the GPU for its raw CRC and combines it with the running register on the
    host (x^(8n) mod P shift), so the value equals the sequential CrcIntTable / java.util.zip result.
    """

    def __init__(self, checksum_type):
        self.type = int(ChecksumType(checksum_type))
        self._state = ctypes.c_uint32(L.lib().ozec_crc_reset(self.type))

    def reset(self):
        self._state = ctypes.c_uint32(L.lib().ozec_crc_reset(self.type))

    def update(self, b, off=None, length=None):
        if isinstance(b, int):  # update(int b)
            a = np.array([b & 0xFF], np.uint8)
        elif isinstance(b, ByteBuffer):  # position moves to limit
            a = np.ascontiguousarray(b.view())
            b.position(b.limit())
        else:
            a = _as_u8(b)
            if off is not None:
                a = a[off:off + length]
        if a.size == 0:
            return
        rc = L.lib().ozec_crc_update(self.type, ctypes.byref(self._state), a.ctypes.data, a.size)
        if rc != L.OZEC_OK:
            raise OzoneChecksumException(L.last_error())

    def get_value(self):
        return int(L.lib().ozec_crc_value(self.type, self._state.value))


def crc32_impl():
    """ChecksumByteBufferFactory.crc32Impl (ChecksumByteBufferFactory.java:74-76)."""
    return ChecksumByteBuffer(ChecksumType.CRC32)


def crc32c_impl():
    """ChecksumByteBufferFactory.crc32CImpl (ChecksumByteBufferFactory.java:78-89)."""
    return ChecksumByteBuffer(ChecksumType.CRC32C)


def checksum_windows_batch(checksum_type, d_base, cell_stride, num_cells, length, bytes_per_checksum, d_out,
                           big_endian=False, stream=None):
    """Device-resident batch: cell c at d_base + c*cell_stride, CRCs to d_out[c][w] (uint32)."""
    rc = L.lib().ozec_checksum_windows_batch(int(checksum_type), _dev_ptr(d_base), cell_stride, num_cells, length,
                                             bytes_per_checksum, _dev_ptr(d_out), 1 if big_endian else 0,
                                             _stream_ptr(stream))
    if rc != L.OZEC_OK:
        raise OzoneChecksumException(L.last_error())


def checksum_verify_batch(checksum_type, d_base, cell_stride, num_cells, length, bytes_per_checksum, d_expected,
                          d_mismatch, expected_big_endian=False, stream=None):
    """Datanode-scanner style batch verify: d_mismatch[c] = -1 or first failing window."""
    rc = L.lib().ozec_checksum_verify_batch(int(checksum_type), _dev_ptr(d_base), cell_stride, num_cells, length,
                                            bytes_per_checksum, _dev_ptr(d_expected), 1 if expected_big_endian else 0,
                                            _dev_ptr(d_mismatch), _stream_ptr(stream))
    if rc != L.OZEC_OK:
        raise OzoneChecksumException(L.last_error())


def crc_combine(checksum_type, crc_a, crc_b, len_b):
    return int(L.lib().ozec_crc_combine(int(checksum_type), crc_a, crc_b, len_b))
