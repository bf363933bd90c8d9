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
