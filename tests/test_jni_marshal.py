"""The JNI-free marshaling core of the Java drop-in (jni/ozec_marshal.c, ozone_amd/lib/libozec_marshal.so).

CPU tests: buffer resolution (positions, array offsets, null slots, bounds), the status -> Java exception map and
every argument check that runs before a device is needed.  GPU tests: encode / decode / CRC through the core
against the oracle, with direct-buffer positions and byte[] offsets as AbstractNativeRawEncoder.doEncode
(EC/rawcoder/AbstractNativeRawEncoder.java:49-73) and ByteArrayEncodingState hand them over.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from synth import SEED, cells

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ozone_amd", "lib", "libozec_marshal.so")

OZEC_EINVAL, OZEC_ENOTINVERTIBLE, OZEC_EDEVICE, OZEC_ECLOSED = -1, -2, -3, -4
OZEC_ENOMEM, OZEC_EUNSUPPORTED, OZEC_EMISMATCH = -5, -6, -7


class Buf(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("offset", ctypes.c_int64), ("capacity", ctypes.c_int64),
                ("present", ctypes.c_int)]


class Status(ctypes.Structure):
    _fields_ = [("code", ctypes.c_int), ("exception_class", ctypes.c_char * 64), ("message", ctypes.c_char * 256)]


@pytest.fixture(scope="module")
def M():
    if not os.path.exists(LIB):
        pytest.skip("libozec_marshal.so not built")
    L = ctypes.CDLL(LIB)
    L.ozm_exception_class.restype = ctypes.c_char_p
    L.ozm_exception_class.argtypes = [ctypes.c_int]
    L.ozm_resolve.argtypes = [ctypes.POINTER(Buf), ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(Status)]
    L.ozm_encode.argtypes = [ctypes.c_void_p, ctypes.POINTER(Buf), ctypes.c_int, ctypes.POINTER(Buf), ctypes.c_int,
                             ctypes.c_int64, ctypes.POINTER(Status)]
    L.ozm_decode.argtypes = [ctypes.c_void_p, ctypes.POINTER(Buf), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                             ctypes.c_int, ctypes.POINTER(Buf), ctypes.c_int, ctypes.c_int64, ctypes.POINTER(Status)]
    L.ozm_crc_update.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(Buf), ctypes.c_int64,
                                 ctypes.POINTER(Status)]
    L.ozm_checksum_windows.argtypes = [ctypes.c_int, ctypes.POINTER(Buf), ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(Status)]
    return L


def bufs(items):
    """items: (array, offset) for a buffer, None for a null slot -> ctypes Buf[]"""
    arr = (Buf * max(1, len(items)))()
    for i, it in enumerate(items):
        if it is None:
            arr[i] = Buf(None, 0, 0, 0)
        else:
            a, off = it
            arr[i] = Buf(a.ctypes.data if a is not None else None, off, a.size if a is not None else -1, 1)
    return arr


def test_exception_map(M):
    cls = {rc: M.ozm_exception_class(rc) for rc in (0, OZEC_EINVAL, OZEC_ENOTINVERTIBLE, OZEC_EDEVICE, OZEC_ECLOSED,
                                                     OZEC_ENOMEM, OZEC_EUNSUPPORTED, OZEC_EMISMATCH)}
    assert cls == {0: None,
                   OZEC_EINVAL: b"org/apache/hadoop/HadoopIllegalArgumentException",
                   OZEC_ENOTINVERTIBLE: b"java/lang/RuntimeException",
                   OZEC_EDEVICE: b"java/io/IOException",
                   OZEC_ECLOSED: b"java/io/IOException",
                   OZEC_ENOMEM: b"java/lang/OutOfMemoryError",
                   OZEC_EUNSUPPORTED: b"java/lang/UnsupportedOperationException",
                   OZEC_EMISMATCH: b"org/apache/hadoop/ozone/common/OzoneChecksumException"}


def test_resolve_positions_offsets_nulls_and_bounds(M):
    a = np.arange(100, dtype=np.uint8)
    b = np.arange(50, dtype=np.uint8)
    out = (ctypes.c_void_p * 3)()
    st = Status()
    assert M.ozm_resolve(bufs([(a, 11), None, (b, 0)]), 3, 1, 39, out, ctypes.byref(st)) == 0
    assert out[0] == a.ctypes.data + 11 and out[1] is None and out[2] == b.ctypes.data
    # a null slot is only allowed for decode inputs
    assert M.ozm_resolve(bufs([(a, 0), None]), 2, 0, 10, out, ctypes.byref(st)) == OZEC_EINVAL
    assert b"not allowing null" in st.message
    assert st.exception_class == b"org/apache/hadoop/HadoopIllegalArgumentException"
    # position + length past the capacity
    assert M.ozm_resolve(bufs([(a, 61)]), 1, 0, 40, out, ctypes.byref(st)) == OZEC_EINVAL
    assert b"exceeds capacity" in st.message
    assert M.ozm_resolve(bufs([(a, -1)]), 1, 0, 4, out, ctypes.byref(st)) == OZEC_EINVAL
    # a present object without an address: a heap ByteBuffer handed to the direct path
    assert M.ozm_resolve(bufs([(None, 0)]), 1, 0, 4, out, ctypes.byref(st)) == OZEC_EINVAL
    assert b"not a direct buffer" in st.message
    assert M.ozm_resolve(bufs([(a, 0)]), 1, 0, -5, out, ctypes.byref(st)) == OZEC_EINVAL


def test_closed_handle_and_argument_checks_before_the_device(M):
    st = Status()
    a = np.zeros(64, np.uint8)
    # the Java handle is 0 after release(): IOException, as TestRawCoderBase.java:118-134 expects
    assert M.ozm_encode(None, bufs([(a, 0)] * 6), 6, bufs([(a, 0)] * 3), 3, 64, ctypes.byref(st)) == OZEC_ECLOSED
    assert st.exception_class == b"java/io/IOException" and b"closed" in st.message
    er = (ctypes.c_int * 1)(0)
    assert M.ozm_decode(None, bufs([None] * 9), 9, er, 1, bufs([(a, 0)]), 1, 64, ctypes.byref(st)) == OZEC_ECLOSED
    state = ctypes.c_uint32(0xFFFFFFFF)
    assert M.ozm_crc_update(3, ctypes.byref(state), bufs([(a, 0)]), 0, ctypes.byref(st)) == 0  # empty update
    assert state.value == 0xFFFFFFFF
    out = np.zeros(16, np.uint8)
    w = ctypes.c_int64()
    assert M.ozm_checksum_windows(3, bufs([(a, 0)]), 64, 0, out.ctypes.data, 16, ctypes.byref(w),
                                  ctypes.byref(st)) == OZEC_EINVAL
    assert M.ozm_checksum_windows(3, bufs([(a, 0)]), 64, 8, out.ctypes.data, 16, ctypes.byref(w),
                                  ctypes.byref(st)) == OZEC_EINVAL  # 8 windows need 32 bytes
    assert b"too small" in st.message
    assert M.ozm_checksum_windows(3, bufs([(a, 0)]), 0, 8, out.ctypes.data, 16, ctypes.byref(w),
                                  ctypes.byref(st)) == 0 and w.value == 0  # empty data: no checksums


# ------------------------------------------------------------------------------------------ GPU

def _coder(decoder, codec, k, p):
    from ozone_amd import _lib
    h = ctypes.c_void_p()
    fn = _lib.lib().ozec_decoder_create if decoder else _lib.lib().ozec_encoder_create
    assert fn(codec, k, p, ctypes.byref(h)) == 0
    return h


@pytest.mark.gpu
@pytest.mark.parametrize("k,p,n", [(6, 3, 1 << 16), (3, 2, 1007), (10, 4, 4096)])
def test_encode_decode_through_the_core(M, k, p, n):
    from ozone_amd import _lib
    enc, dec = _coder(False, 0, k, p), _coder(True, 0, k, p)
    try:
        d = cells(SEED, 730000 + k, k, n)
        # direct buffers at position 11 inside larger allocations, as TestCoderBase's position-11 buffers
        wide = [np.zeros(n + 20, np.uint8) for _ in range(k)]
        for w, x in zip(wide, d):
            w[11:11 + n] = x
        outs = [np.full(n + 20, 0xA5, np.uint8) for _ in range(p)]
        st = Status()
        assert M.ozm_encode(enc, bufs([(w, 11) for w in wide]), k, bufs([(o, 11) for o in outs]), p, n,
                            ctypes.byref(st)) == 0, st.message
        ref = oracle.rs_encode(k, p, d)
        for o, r in zip(outs, ref):
            assert (o[11:11 + n] == r).all() and (o[:11] == 0xA5).all() and (o[11 + n:] == 0xA5).all()
        units = d + ref
        erased = [0, k] if p >= 2 else [0]
        ins = [None if u in erased else (units[u], 0) for u in range(k + p)]
        rec = [np.zeros(n, np.uint8) for _ in erased]
        er = (ctypes.c_int * len(erased))(*erased)
        assert M.ozm_decode(dec, bufs(ins), k + p, er, len(erased), bufs([(r, 0) for r in rec]), len(erased), n,
                            ctypes.byref(st)) == 0, st.message
        for r, e in zip(rec, erased):
            assert (r == units[e]).all()
        # errors carry the reference's exception class and text
        assert M.ozm_encode(enc, bufs([(w, 11) for w in wide[:-1]]), k - 1, bufs([(o, 11) for o in outs]), p, n,
                            ctypes.byref(st)) == OZEC_EINVAL
        assert st.message.startswith(b"Invalid inputs length")
        too_many = (ctypes.c_int * (p + 1))(*range(p + 1))
        assert M.ozm_decode(dec, bufs(ins), k + p, too_many, p + 1, bufs([(rec[0], 0)] * (p + 1)), p + 1, n,
                            ctypes.byref(st)) == OZEC_EINVAL
        assert b"Too many erased" in st.message
        _lib.lib().ozec_coder_release(enc)
        assert M.ozm_encode(enc, bufs([(w, 11) for w in wide]), k, bufs([(o, 11) for o in outs]), p, n,
                            ctypes.byref(st)) == OZEC_ECLOSED
        assert st.exception_class == b"java/io/IOException"
    finally:
        _lib.lib().ozec_coder_free(enc)
        _lib.lib().ozec_coder_free(dec)


@pytest.mark.gpu
def test_checksums_through_the_core(M):
    n, bpc = 100_000, 16384
    data = cells(SEED, 731000, 1, n + 7)[0]
    st = Status()
    for ctype, otype in ((3, oracle.CRC32C), (2, oracle.CRC32)):
        out = np.zeros(4 * 7, np.uint8)
        w = ctypes.c_int64()
        assert M.ozm_checksum_windows(ctype, bufs([(data, 7)]), n, bpc, out.ctypes.data, out.size, ctypes.byref(w),
                                      ctypes.byref(st)) == 0, st.message
        assert w.value == 28
        assert (out.view(">u4") == oracle.crc_windows(otype, data[7:7 + n], bpc)).all()
        state = ctypes.c_uint32(0xFFFFFFFF)
        assert M.ozm_crc_update(ctype, ctypes.byref(state), bufs([(data, 7)]), n, ctypes.byref(st)) == 0
        assert (~state.value) & 0xFFFFFFFF == oracle.crc_windows(otype, data[7:7 + n], n)[0]
