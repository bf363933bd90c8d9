"""COMPOSITE_CRC and stripe checksums over libozec.

Mirrors, with the reference's names and error behaviour:
  CrcUtil                         hadoop-ozone/common/.../client/checksum/CrcUtil.java
  CrcComposer                     hadoop-ozone/common/.../client/checksum/CrcComposer.java
  ReplicatedBlockChecksumComputer hadoop-ozone/client/.../client/checksum/ReplicatedBlockChecksumComputer.java
  ECBlockChecksumComputer         hadoop-ozone/client/.../client/checksum/ECBlockChecksumComputer.java
  stripe_checksum                 ECBlockOutputStreamEntry.calculateChecksum (OC/io/ECBlockOutputStreamEntry.java:390-414)
The CRC arithmetic (monomials, composition, the composer state machine and the batched device composition of
window CRCs) runs in libozec; the block computers are the reference's byte bookkeeping around it.
"""
import ctypes
import enum
import hashlib
from dataclasses import dataclass

from . import _lib as L
from .checksum import ChecksumData, ChecksumType
from .rawcoder import IllegalArgumentException, IOException, _dev_ptr, _stream_ptr

MULTIPLICATIVE_IDENTITY = 0x80000000  # CrcUtil.java:34
GZIP_POLYNOMIAL = 0xEDB88320
CASTAGNOLI_POLYNOMIAL = 0x82F63B78


class ChecksumCombineMode(enum.Enum):
    """OzoneClientConfig.ChecksumCombineMode."""
    MD5MD5CRC = "MD5MD5CRC"
    COMPOSITE_CRC = "COMPOSITE_CRC"


def _type_id(checksum_type):
    t = ChecksumType(checksum_type)
    if t not in (ChecksumType.CRC32, ChecksumType.CRC32C):
        raise IOException(f"No CRC polynomial could be associated with type: {t.name}")
    return int(t)


def _check(rc, exc=IllegalArgumentException):
    if rc == L.OZEC_OK:
        return
    msg = L.last_error()
    if rc == L.OZEC_EMISMATCH:
        raise IOException(msg)
    raise exc(msg)


def _s32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


class CrcUtil:
    """CrcUtil (CrcUtil.java:30-271). CRC values are Java ints (signed) or their unsigned 32-bit images."""

    @staticmethod
    def get_crc_polynomial_for_type(checksum_type):
        return GZIP_POLYNOMIAL if _type_id(checksum_type) == ChecksumType.CRC32 else CASTAGNOLI_POLYNOMIAL

    @staticmethod
    def get_monomial(length_bytes, checksum_type):
        out = ctypes.c_uint32()
        _check(L.lib().ozec_crc_monomial(_type_id(checksum_type), length_bytes, ctypes.byref(out)))
        return out.value

    @staticmethod
    def compose(crc_a, crc_b, length_b, checksum_type):
        out = ctypes.c_uint32()
        _check(L.lib().ozec_crc_compose(_type_id(checksum_type), crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, length_b,
                                        ctypes.byref(out)))
        return out.value

    @staticmethod
    def int_to_bytes(value):
        return (value & 0xFFFFFFFF).to_bytes(4, "big")

    @staticmethod
    def read_int(buf, offset=0):
        if offset + 4 > len(buf):
            raise IOException(f"readInt out of bounds: buf.length={len(buf)}, offset={offset}")
        return int.from_bytes(bytes(buf[offset:offset + 4]), "big")

    @staticmethod
    def to_single_crc_string(b):
        if len(b) != 4:
            raise IOException(f"Unexpected byte[] length '{len(b)}' for single CRC. Contents: {list(b)}")
        return "0x%08x" % CrcUtil.read_int(b)

    @staticmethod
    def to_multi_crc_string(b):
        if len(b) % 4 != 0:
            raise IOException(f"Unexpected byte[] length '{len(b)}' not divisible by 4. Contents: {list(b)}")
        return "[" + ", ".join("0x%08x" % CrcUtil.read_int(b, i) for i in range(0, len(b), 4)) + "]"


class CrcComposer:
    """CrcComposer (CrcComposer.java:44-215) backed by ozec_crc_composer."""

    def __init__(self, checksum_type, bytes_per_crc_hint, stripe_length=0):
        self._h = ctypes.c_void_p()
        _check(L.lib().ozec_crc_composer_create(_type_id(checksum_type), bytes_per_crc_hint, stripe_length,
                                                ctypes.byref(self._h)))

    @staticmethod
    def new_crc_composer(checksum_type, bytes_per_crc_hint):
        return CrcComposer(checksum_type, bytes_per_crc_hint)

    @staticmethod
    def new_striped_crc_composer(checksum_type, bytes_per_crc_hint, stripe_length):
        return CrcComposer(checksum_type, bytes_per_crc_hint, stripe_length)

    def update(self, crc_b, bytes_per_crc):
        """update(int crcB, long bytesPerCrc)."""
        _check(L.lib().ozec_crc_composer_update(self._h, crc_b & 0xFFFFFFFF, bytes_per_crc))

    def update_bytes(self, crc_buffer, offset, length, bytes_per_crc):
        """update(byte[] crcBuffer, int offset, int length, long bytesPerCrc)."""
        if length % 4 != 0:
            raise IOException(f"Trying to update CRC from byte array with length '{length}' at offset '{offset}' "
                              f"which is not a multiple of 4!")
        b = bytes(crc_buffer[offset:offset + length])
        _check(L.lib().ozec_crc_composer_update_bytes(self._h, b, len(b), bytes_per_crc))

    def digest(self):
        n = L.lib().ozec_crc_composer_pending(self._h)
        buf = ctypes.create_string_buffer(max(1, n))
        got = ctypes.c_size_t()
        _check(L.lib().ozec_crc_composer_digest(self._h, buf, n, ctypes.byref(got)))
        return buf.raw[:got.value]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.lib().ozec_crc_composer_free(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self._h = None


@dataclass
class ChunkInfo:
    """The ContainerProtos.ChunkInfo fields the block checksum computers read."""
    length: int
    checksum_data: ChecksumData
    stripe_checksum: bytes = None


class ReplicatedBlockChecksumComputer:
    """ReplicatedBlockChecksumComputer (ReplicatedBlockChecksumComputer.java:40-150)."""

    def __init__(self, chunk_infos):
        self._chunks = list(chunk_infos)
        self._out = None

    def compute(self, mode):
        if mode == ChecksumCombineMode.MD5MD5CRC:
            return self._md5_crc()
        if mode == ChecksumCombineMode.COMPOSITE_CRC:
            return self._composite_crc()
        raise IllegalArgumentException("unsupported combine mode")

    def get_out_bytes(self):
        return self._out

    def _md5_crc(self):  # :72-91, md5 over all chunk checksums concatenated
        self._out = hashlib.md5(b"".join(b for c in self._chunks for b in c.checksum_data.get_checksums())).digest()

    def _composite_crc(self):  # :94-148
        if not self._chunks:
            raise IllegalArgumentException("chunk list is empty")
        first = self._chunks[0]
        ctype = first.checksum_data.get_checksum_type()
        if ctype not in (ChecksumType.CRC32, ChecksumType.CRC32C):
            raise IllegalArgumentException(f"unsupported checksum type: {ChecksumType(ctype).name}")
        chunk_size = first.length
        bpc = first.checksum_data.get_bytes_per_checksum()
        block = CrcComposer.new_crc_composer(ctype, chunk_size)
        for ci in self._chunks:
            sums = ci.checksum_data.get_checksums()
            cc = CrcComposer.new_crc_composer(ctype, bpc)
            remaining = ci.length
            if remaining > len(sums) * chunk_size:
                raise IllegalArgumentException("chunk longer than its checksums cover")
            for s in sums:
                cc.update(CrcUtil.read_int(s), min(bpc, remaining))
                remaining -= bpc
            block.update(CrcUtil.read_int(cc.digest()), ci.length)
        self._out = block.digest()


class ECBlockChecksumComputer:
    """ECBlockChecksumComputer (ECBlockChecksumComputer.java:46-211). `chunk_infos` carry the stripe checksums
    (stripe_checksum: the concatenated 4-B window CRCs of every unit of the stripe, parity last)."""

    def __init__(self, chunk_infos, key_size, num_parity):
        self._chunks = list(chunk_infos)
        self._key_size = key_size
        self._parity = num_parity
        self._out = None

    def compute(self, mode):
        if mode == ChecksumCombineMode.MD5MD5CRC:
            return self._md5_crc()
        if mode == ChecksumCombineMode.COMPOSITE_CRC:
            return self._composite_crc()
        raise IllegalArgumentException("Unsupported combine mode")

    def get_out_bytes(self):
        return self._out

    def _parity_bytes(self, chunk_size, bpc):  # getParityBytes :202-209
        return -(-chunk_size // bpc) * 4 * self._parity

    def _md5_crc(self):  # :72-103
        first = self._chunks[0]
        bpc = first.checksum_data.get_bytes_per_checksum()
        parity_bytes = self._parity_bytes(first.length, bpc)
        md5 = hashlib.md5()
        for ci in self._chunks:
            sc = ci.stripe_checksum
            if sc is None or len(sc) % 4 != 0:
                raise IllegalArgumentException("Checksum Bytes size does not match")
            md5.update(sc[:len(sc) - parity_bytes])
        md5.digest()
        # the reference stores a second digest() of the already-reset digester (:96-97), i.e. MD5 of nothing
        self._out = hashlib.md5().digest()

    def _composite_crc(self):  # :105-195
        if not self._chunks:
            raise IllegalArgumentException("chunk list is empty")
        first = self._chunks[0]
        ctype = first.checksum_data.get_checksum_type()
        if ctype not in (ChecksumType.CRC32, ChecksumType.CRC32C):
            raise IllegalArgumentException(f"Unsupported checksum type: {ChecksumType(ctype).name}")
        bpc = first.checksum_data.get_bytes_per_checksum()
        chunk_size = first.length
        offset = chunk_size % bpc
        key_size = self._key_size
        parity_bytes = self._parity_bytes(chunk_size, bpc)
        per_chunk = -(-chunk_size // bpc)
        block = CrcComposer.new_crc_composer(ctype, bpc)
        for ci in self._chunks:
            sc = ci.stripe_checksum
            if sc is None or len(sc) % 4 != 0:
                raise IllegalArgumentException("Checksum Bytes size does not match")
            body = sc[:len(sc) - parity_bytes]
            idx = 1
            for off in range(0, len(body), 4):
                cur_off = offset if (idx % per_chunk == 0 and offset > 0) else (1 << 63) - 1
                size = min(min(key_size, bpc), cur_off)
                cc = CrcComposer.new_crc_composer(ctype, bpc)
                cc.update(CrcUtil.read_int(body, off), size)
                block.update(CrcUtil.read_int(cc.digest()), size)
                key_size -= min(bpc, cur_off)
                idx += 1
        self._out = block.digest()


def stripe_checksum(unit_checksums):
    """ECBlockOutputStreamEntry.calculateChecksum (:390-414): the stripe's chunk checksums of every unit that has
    the chunk, concatenated in unit order. `unit_checksums`: list of ChecksumData (None for a unit without it)."""
    return b"".join(b for cd in unit_checksums if cd is not None for b in cd.get_checksums())


def compose_windows_batch(checksum_type, d_crcs, crc_cell_stride, num_cells, num_windows, bytes_per_checksum,
                          last_len, d_out, crcs_big_endian=False, out_big_endian=False, stream=None):
    """Device: CrcComposer over each cell's window CRCs (ozec_crc_compose_windows_batch)."""
    rc = L.lib().ozec_crc_compose_windows_batch(_type_id(checksum_type), _dev_ptr(d_crcs), crc_cell_stride,
                                                num_cells, num_windows, bytes_per_checksum, last_len,
                                                1 if crcs_big_endian else 0, _dev_ptr(d_out),
                                                1 if out_big_endian else 0, _stream_ptr(stream))
    _check(rc)
