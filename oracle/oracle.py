"""ctypes binding of liboracle.so (TEST INFRASTRUCTURE ONLY -- see ozec_oracle.c header).

Every function mirrors one reference routine; citations are in ozec_oracle.c.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

CRC32 = 0
CRC32C = 1

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_ip = ctypes.POINTER(ctypes.c_int)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_gf_mul.restype = ctypes.c_uint8
        L.oracle_gf_inv.restype = ctypes.c_uint8
        L.oracle_crc_update.restype = ctypes.c_uint32
        L.oracle_crc_update.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc.restype = ctypes.c_uint32
        L.oracle_crc.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc_windows.restype = ctypes.c_size_t
        L.oracle_crc_windows.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_void_p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(arrs):
    out = (ctypes.c_void_p * len(arrs))()
    for i, a in enumerate(arrs):
        out[i] = None if a is None else a.ctypes.data
    return out


def gf_tables():
    base = np.zeros(256, np.uint8)
    logb = np.zeros(256, np.uint8)
    lib().oracle_gf_tables(_ptr(base), _ptr(logb))
    return base, logb


def gf_mul(a, b):
    return int(lib().oracle_gf_mul(ctypes.c_uint8(a), ctypes.c_uint8(b)))


def gf_inv(a):
    return int(lib().oracle_gf_inv(ctypes.c_uint8(a)))


def cauchy_matrix(k, p):
    m = np.zeros((k + p) * k, np.uint8)
    lib().oracle_gen_cauchy_matrix(_ptr(m), k + p, k)
    return m.reshape(k + p, k)


def invert_matrix(mat):
    n = mat.shape[0]
    a = np.ascontiguousarray(mat, dtype=np.uint8).copy()
    out = np.zeros((n, n), np.uint8)
    rc = lib().oracle_gf_invert_matrix(_ptr(a), _ptr(out), n)
    if rc != 0:
        raise RuntimeError("Not invertible")
    return out


def rs_encode(k, p, data):
    """data: list of k uint8 arrays of equal length -> list of p parity arrays."""
    n = len(data[0])
    data = [np.ascontiguousarray(d, dtype=np.uint8) for d in data]
    par = [np.zeros(n, np.uint8) for _ in range(p)]
    rc = lib().oracle_rs_encode(k, p, n, _ptr_array(data), _ptr_array(par))
    if rc != 0:
        raise ValueError("Invalid numDataUnits and numParityUnits")
    return par


def rs_decode_matrix(k, p, valid, erased):
    v = (ctypes.c_int * k)(*valid[:k])
    e = (ctypes.c_int * max(1, len(erased)))(*erased)
    out = np.zeros(max(1, len(erased)) * k, np.uint8)
    rc = lib().oracle_rs_decode_matrix(k, p, v, e, len(erased), _ptr(out))
    if rc != 0:
        raise RuntimeError("Not invertible")
    return out[: len(erased) * k].reshape(len(erased), k)


def rs_decode(k, p, inputs, erased):
    """inputs: k+p slots (None = erased/not read). Returns len(erased) recovered arrays."""
    n = next(len(x) for x in inputs if x is not None)
    ins = [None if x is None else np.ascontiguousarray(x, dtype=np.uint8) for x in inputs]
    outs = [np.zeros(n, np.uint8) for _ in erased]
    e = (ctypes.c_int * max(1, len(erased)))(*erased)
    rc = lib().oracle_rs_decode(k, p, n, _ptr_array(ins), e, len(erased), _ptr_array(outs))
    if rc == -1:
        raise RuntimeError("Not invertible")
    if rc == -2:
        raise ValueError("No enough valid inputs are provided, not recoverable")
    return outs


def xor_encode(data):
    n = len(data[0])
    data = [np.ascontiguousarray(d, dtype=np.uint8) for d in data]
    out = np.zeros(n, np.uint8)
    lib().oracle_xor_encode(len(data), n, _ptr_array(data), _ptr(out))
    return out


def xor_decode(inputs, erased0):
    n = next(len(x) for x in inputs if x is not None)
    ins = [None if x is None else np.ascontiguousarray(x, dtype=np.uint8) for x in inputs]
    out = np.zeros(n, np.uint8)
    rc = lib().oracle_xor_decode(len(ins), n, _ptr_array(ins), erased0, _ptr(out))
    if rc != 0:
        raise ValueError("null input")
    return out


def crc_table(ctype):
    t = np.zeros(0x800, np.uint32)
    lib().oracle_crc_table(ctype, _ptr(t))
    return t


def crc(ctype, data):
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             dtype=np.uint8)
    return int(lib().oracle_crc(ctype, _ptr(a), a.size))


def crc_windows(ctype, data, bpc):
    a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    nw = (a.size + bpc - 1) // bpc
    out = np.zeros(max(1, nw), np.uint32)
    lib().oracle_crc_windows(ctype, _ptr(a), a.size, bpc, _ptr(out))
    return out[:nw]


# ---------------------------------------------------------------- COMPOSITE_CRC (ozec_oracle.c) ---------------

def _composite_lib():
    L = lib()
    if not getattr(L, "_composite_ready", False):
        L.oracle_crc_poly.restype = ctypes.c_uint32
        L.oracle_gf32_multiply.restype = ctypes.c_uint32
        L.oracle_gf32_multiply.argtypes = [ctypes.c_uint32] * 3
        L.oracle_crc_monomial.argtypes = [ctypes.c_int64, ctypes.c_uint32, _u32p]
        L.oracle_crc_compose.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint32, _u32p]
        L.oracle_composer_new.restype = ctypes.c_void_p
        L.oracle_composer_new.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.oracle_composer_update.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64]
        L.oracle_composer_digest.restype = ctypes.c_size_t
        L.oracle_composer_digest.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_composer_free.argtypes = [ctypes.c_void_p]
        L.oracle_composer_pending.restype = ctypes.c_size_t
        L.oracle_composer_pending.argtypes = [ctypes.c_void_p]
        L._composite_ready = True
    return L


def crc_monomial(ctype, length):
    out = ctypes.c_uint32()
    L = _composite_lib()
    if L.oracle_crc_monomial(length, L.oracle_crc_poly(ctype), ctypes.byref(out)):
        raise ValueError(f"lengthBytes must be positive, got {length}")
    return out.value


def crc_compose(ctype, crc_a, crc_b, len_b):
    """CrcUtil.compose (OC/CrcUtil.java:124-127)."""
    out = ctypes.c_uint32()
    L = _composite_lib()
    if L.oracle_crc_compose(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b, L.oracle_crc_poly(ctype), ctypes.byref(out)):
        raise ValueError(f"lengthBytes must be positive, got {len_b}")
    return out.value


class Composer:
    """CrcComposer (OC/CrcComposer.java:44-215) through ozec_oracle.c."""

    def __init__(self, ctype, bytes_per_crc_hint, stripe_length=(1 << 63) - 1):
        self._L = _composite_lib()
        self._c = self._L.oracle_composer_new(ctype, bytes_per_crc_hint, stripe_length)

    def update(self, crc, bytes_per_crc):
        rc = self._L.oracle_composer_update(self._c, crc & 0xFFFFFFFF, bytes_per_crc)
        if rc == -1:
            raise ValueError(f"lengthBytes must be positive, got {bytes_per_crc}")
        if rc == -2:
            raise OSError("Current position in stripe exceeds stripeLength without stripe alignment.")

    def digest(self):
        buf = ctypes.create_string_buffer(max(4, self._L.oracle_composer_pending(self._c)))
        n = self._L.oracle_composer_digest(self._c, buf, len(buf))
        return buf.raw[:n]

    def __del__(self):
        if getattr(self, "_c", None):
            self._L.oracle_composer_free(self._c)
            self._c = None


def read_int(b, off=0):
    v = int.from_bytes(bytes(b[off:off + 4]), "big")
    return v


def replicated_block_composite_crc(ctype, chunks, bytes_per_crc):
    """ReplicatedBlockChecksumComputer.computeCompositeCrc (client/checksum/ReplicatedBlockChecksumComputer.java:
    94-148). chunks: list of (chunk_len, [window crc ints]); the first chunk's length is the block hint."""
    block = Composer(ctype, chunks[0][0])
    for chunk_len, crcs in chunks:
        cc = Composer(ctype, bytes_per_crc)
        remaining = chunk_len
        for c in crcs:
            cc.update(c, min(bytes_per_crc, remaining))
            remaining -= bytes_per_crc
        block.update(read_int(cc.digest()), chunk_len)
    return block.digest()


def ec_block_composite_crc(ctype, stripe_checksums, chunk_size, bytes_per_crc, key_size, num_parity):
    """ECBlockChecksumComputer.computeCompositeCrc (client/checksum/ECBlockChecksumComputer.java:105-195).
    stripe_checksums: list of bytes (the concatenated 4-B BE window CRCs of a stripe, parity units last)."""
    offset = chunk_size % bytes_per_crc
    parity_bytes = -(-chunk_size // bytes_per_crc) * 4 * num_parity
    per_chunk = -(-chunk_size // bytes_per_crc)
    block = Composer(ctype, bytes_per_crc)
    for sc in stripe_checksums:
        assert len(sc) % 4 == 0
        body = sc[:len(sc) - parity_bytes]
        idx = 1
        for off in range(0, len(body), 4):
            cur_off = offset if (idx % per_chunk == 0 and offset > 0) else (1 << 63) - 1
            crc = read_int(body, off)
            size = min(min(key_size, bytes_per_crc), cur_off)
            cc = Composer(ctype, bytes_per_crc)
            cc.update(crc, size)
            block.update(read_int(cc.digest()), size)
            key_size -= min(bytes_per_crc, cur_off)
            idx += 1
    return block.digest()
