"""jni/ozec_jni.c itself, compiled against the JNI test double (tests/native/mockjni) and called the way the Java
classes (java/src/main/java/.../OzecNative.java) call it: direct ByteBuffers with positions, byte[] with offsets,
null decode inputs, int[] erasedIndexes.  Checks the results against the oracle (GPU), the Java exception each
failure raises, and that every pinned array is released and every local reference deleted (CPU and GPU)."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle
from synth import SEED, cells

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "ozone_amd", "lib")
P = "Java_org_apache_ozone_erasurecode_rawcoder_OzecNative_"
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64


@pytest.fixture(scope="module")
def J():
    if not os.path.exists(os.path.join(LIBDIR, "libozec.so")):
        pytest.skip("libozec.so not built")
    d = tempfile.mkdtemp(prefix="ozec_mockjni_")
    so = os.path.join(d, "libozec_jni_mock.so")
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "tests", "native", "mockjni"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "jni", "ozec_jni.c"), os.path.join(ROOT, "jni", "ozec_marshal.c"),
                    os.path.join(ROOT, "tests", "native", "mockjni", "mockjni.c"), "-L", LIBDIR, "-lozec",
                    # device-work entry points wrapped by the mock (pins outstanding at each call)
                    "-Wl,--wrap=ozec_encode,--wrap=ozec_decode,--wrap=ozec_crc_update,--wrap=ozec_checksum_windows,"
                    "--wrap=ozec_encode_cb,--wrap=ozec_decode_cb,"
                    "--wrap=ozec_host_alloc,--wrap=ozec_host_free",
                    f"-Wl,-rpath,{LIBDIR}", "-o", so], check=True, capture_output=True, timeout=120)
    L = ctypes.CDLL(so)
    for name, res, args in [
        ("mock_env", vp, []), ("mock_direct", vp, [vp, i64]), ("mock_heap_buffer", vp, [vp, i64]),
        ("mock_bytes", vp, [vp, i64]), ("mock_ints", vp, [vp, i64]), ("mock_objects", vp, [i64]),
        ("mock_set", None, [vp, i64, vp]), ("mock_data", vp, [vp]), ("mock_len", i64, [vp]), ("mock_free", None, [vp]),
        ("mock_pins", ctypes.c_int, []), ("mock_local_refs", ctypes.c_int, []),
        ("mock_pins_at_device_call", ctypes.c_int, []), ("mock_device_calls", ctypes.c_int, []),
        ("mock_reset_device_calls", None, []), ("mock_region_copies", ctypes.c_int, []),
        ("mock_set_missing_class", None, [ctypes.c_char_p]), ("mock_host_allocs", ctypes.c_int, []),
        ("mock_host_live", ctypes.c_int, []), ("mock_refuse_pin_after", None, [ctypes.c_int]),
        ("mock_calls_with_pending", ctypes.c_int, []), ("mock_pins_after_callback", ctypes.c_int, []),
        ("mock_take_exception", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
        ("ozec_jni_heap_mode", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_ulong),
                                              ctypes.POINTER(ctypes.c_ulong)]),
        (P + "deviceCount", i32, [vp, vp]),
        (P + "setDevices", None, [vp, vp, vp]), (P + "getDevices", vp, [vp, vp]),
        (P + "setDevicePolicy", None, [vp, vp, i32]), (P + "coderDevice", i32, [vp, vp, i64]),
        (P + "coderCreate", i64, [vp, vp, ctypes.c_uint8, i32, i32, i32]),
        (P + "coderRelease", None, [vp, vp, i64]),
        (P + "encodeDirect", None, [vp, vp, i64, vp, vp, i32, vp, vp]),
        (P + "encodeArrays", None, [vp, vp, i64, vp, vp, i32, vp, vp]),
        (P + "decodeDirect", None, [vp, vp, i64, vp, vp, i32, vp, vp, vp]),
        (P + "decodeArrays", None, [vp, vp, i64, vp, vp, i32, vp, vp, vp]),
        (P + "crcUpdateDirect", i32, [vp, vp, i32, i32, vp, i32, i32]),
        (P + "crcUpdateArray", i32, [vp, vp, i32, i32, vp, i32, i32]),
        (P + "checksumWindowsDirect", i32, [vp, vp, i32, vp, i32, i32, i32, vp]),
        (P + "checksumWindowsArray", i32, [vp, vp, i32, vp, i32, i32, i32, vp]),
        (P + "allocatePinned", vp, [vp, vp, i32]), (P + "freePinned", None, [vp, vp, vp]),
        (P + "queueCreate", i64, [vp, vp, i64, i32, i32, i32, i32]),
        (P + "queueSubmit", i64, [vp, vp, i64, vp, vp, vp, vp, i32, vp, i32]),
        (P + "queueWait", None, [vp, vp, i64, i64]), (P + "queueFree", None, [vp, vp, i64]),
        (P + "reconstructHostBatch", None, [vp, vp, i64, vp, i64, i64, vp, vp, vp, i32, i32, i32, i32, vp, vp, vp]),
        (P + "crcMonomial", i32, [vp, vp, i32, i64]), (P + "crcCompose", i32, [vp, vp, i32, i32, i32, i64]),
        (P + "composerCreate", i64, [vp, vp, i32, i64, i64]), (P + "composerUpdate", None, [vp, vp, i64, i32, i64]),
        (P + "composerUpdateBytes", None, [vp, vp, i64, vp, i32, i32, i64]),
        (P + "composerPending", i32, [vp, vp, i64]), (P + "composerDigest", i32, [vp, vp, i64, vp]),
        (P + "composerFree", None, [vp, vp, i64]),
        (P + "composeWindowsBatch", None, [vp, vp, i32, i64, i64, i64, i64, i64, i64, ctypes.c_uint8, i64,
                                           ctypes.c_uint8, i64])]:
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    L.env = L.mock_env()
    return L


class Java:
    """Builds fake Java objects over numpy memory (kept alive here) and reads the pending exception."""

    def __init__(self, J):
        self.J, self.keep, self.objs = J, [], []

    def _o(self, o):
        self.objs.append(o)
        return o

    def direct(self, a):
        self.keep.append(a)
        return self._o(self.J.mock_direct(a.ctypes.data, a.size))

    def heap(self, a):
        self.keep.append(a)
        return self._o(self.J.mock_heap_buffer(a.ctypes.data, a.size))

    def bytes(self, a):
        self.keep.append(a)
        return self._o(self.J.mock_bytes(a.ctypes.data, a.size))

    def ints(self, v):
        a = np.asarray(v, np.int32)
        self.keep.append(a)
        return self._o(self.J.mock_ints(a.ctypes.data, a.size))

    def array(self, elems):
        arr = self._o(self.J.mock_objects(len(elems)))
        for i, e in enumerate(elems):
            self.J.mock_set(arr, i, e)
        return arr

    def exception(self):
        c, m = ctypes.create_string_buffer(128), ctypes.create_string_buffer(512)
        return (c.value.decode(), m.value.decode()) if self.J.mock_take_exception(c, 128, m, 512) else None

    def close(self):
        for o in self.objs:
            self.J.mock_free(o)
        self.objs = []


@pytest.fixture
def java(J):
    j = Java(J)
    yield j
    assert J.mock_pins() == 0, "a pinned array was not released"
    assert J.mock_local_refs() == 0, "a local reference was not deleted"
    j.close()


def call(J, name, *args):
    return getattr(J, P + name)(J.env, None, *args)


def gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


# ------------------------------------------------------------------------------------------ CPU


def test_closed_handle_raises_ioexception_and_unpins(J, java):
    a = [np.zeros(64, np.uint8) for _ in range(9)]
    call(J, "encodeDirect", 0, java.array([java.direct(x) for x in a[:6]]), java.ints([0] * 6), 64,
         java.array([java.direct(x) for x in a[6:]]), java.ints([0] * 3))
    assert java.exception() == ("java/io/IOException", "coder is closed")
    call(J, "encodeArrays", 0, java.array([java.bytes(x) for x in a[:6]]), java.ints([0] * 6), 64,
         java.array([java.bytes(x) for x in a[6:]]), java.ints([0] * 3))
    assert java.exception()[0] == "java/io/IOException"
    call(J, "decodeArrays", 0, java.array([None] + [java.bytes(x) for x in a[1:9]]), java.ints([0] * 9), 64,
         java.ints([0]), java.array([java.bytes(a[0])]), java.ints([0]))
    assert java.exception()[0] == "java/io/IOException"


def test_argument_errors_before_the_device(J, java):
    data = np.zeros(100, np.uint8)
    out = np.zeros(64, np.uint8)
    assert call(J, "checksumWindowsDirect", 3, java.direct(data), 0, 100, 0, java.bytes(out)) == 0
    assert java.exception() == ("org/apache/hadoop/HadoopIllegalArgumentException", "bytesPerChecksum must be positive")
    # hadoop-common absent from the class path: the superclass is thrown instead
    J.mock_set_missing_class(b"org/apache/hadoop/HadoopIllegalArgumentException")
    try:
        call(J, "checksumWindowsArray", 3, java.bytes(data), 0, 100, 0, java.bytes(out))
        assert java.exception() == ("java/lang/IllegalArgumentException", "bytesPerChecksum must be positive")
    finally:
        J.mock_set_missing_class(None)
    assert call(J, "crcUpdateArray", 3, -1, java.bytes(data), 0, 0) == -1  # empty update: register unchanged
    assert java.exception() is None
    assert call(J, "crcUpdateArray", 3, -1, java.bytes(data), 90, 20) == -1  # offset + length past the array
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
    assert call(J, "allocatePinned", -1) is None
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
    assert call(J, "queueCreate", 0, 0, 4, 3, 16384) == 0
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"


def test_no_device_makes_the_factory_throw(J, java):
    """Without a GPU the coder constructor throws, so CodecUtil falls back to rs_java (CodecUtil.java:62-78)."""
    if gpu():
        pytest.skip("a GPU is visible")
    assert call(J, "deviceCount") == 0
    assert call(J, "coderCreate", 0, 0, 6, 3) == 0
    cls, msg = java.exception()
    assert cls == "java/io/IOException" and "no HIP device" in msg


def _s32(v):
    return v - (1 << 32) if v >= 1 << 31 else v


@pytest.mark.parametrize("ctype", [2, 3])
def test_crcutil_natives_vs_oracle(J, java, ctype):
    """HipCrcUtil's natives (CrcUtil.getMonomial / compose, OC/CrcUtil.java:74-127) vs the oracle; a negative length
    raises the reference's IllegalArgumentException, a non-CRC type its IOException."""
    ot = oracle.CRC32 if ctype == 2 else oracle.CRC32C
    r = np.random.default_rng(ctype)
    for n in (0, 1, 16, 4096, 16384, 1 << 20, (1 << 40) + 7):
        assert call(J, "crcMonomial", ctype, n) & 0xFFFFFFFF == oracle.crc_monomial(ot, n)
    for _ in range(100):
        a, b = (int(x) for x in r.integers(0, 1 << 32, 2, dtype=np.uint64))
        n = int(r.integers(0, 1 << 33))
        assert call(J, "crcCompose", ctype, _s32(a), _s32(b), n) & 0xFFFFFFFF == oracle.crc_compose(ot, a, b, n)
    assert java.exception() is None
    call(J, "crcMonomial", ctype, -1)
    assert java.exception() == ("java/lang/IllegalArgumentException", "lengthBytes must be positive, got -1")
    call(J, "crcCompose", ctype, 1, 2, -3)
    assert java.exception()[0] == "java/lang/IllegalArgumentException"
    call(J, "crcMonomial", 4, 16)  # SHA256
    assert java.exception() == ("java/io/IOException", "No CRC polynomial could be associated with type: 4")


@pytest.mark.parametrize("ctype", [2, 3])
@pytest.mark.parametrize("hint,stripe", [(4096, (1 << 63) - 1), (4096, 16384), (512, 1536)])
def test_crc_composer_natives_vs_oracle(J, java, ctype, hint, stripe):
    """HipCrcComposer's natives (CrcComposer, OC/CrcComposer.java:44-215): update(int, long) and update(byte[], ...)
    interleaved, digests of partial and whole stripes, vs the oracle's CrcComposer."""
    ot = oracle.CRC32 if ctype == 2 else oracle.CRC32C
    r = np.random.default_rng(hint + ctype)
    c = call(J, "composerCreate", ctype, hint, stripe)
    assert java.exception() is None and c
    ref = oracle.Composer(ot, hint, stripe)
    try:
        for step in range(120):
            crcs = r.integers(0, 1 << 32, int(r.integers(1, 5)), dtype=np.uint64)
            crcs[0] = 0 if step % 17 == 0 else crcs[0]  # the cur == 0 shortcut
            if step % 2:
                for v in crcs:
                    call(J, "composerUpdate", c, _s32(int(v)), hint)
            else:
                be = crcs.astype(">u4").view(np.uint8)
                buf = np.concatenate([np.zeros(3, np.uint8), be])
                call(J, "composerUpdateBytes", c, java.bytes(buf), 3, be.size, hint)
            for v in crcs:
                ref.update(int(v), hint)
            assert java.exception() is None
            if step % 25 == 0:
                out = np.zeros(call(J, "composerPending", c), np.uint8)
                assert call(J, "composerDigest", c, java.bytes(out)) == out.size
                assert out.tobytes() == ref.digest()
        out = np.zeros(call(J, "composerPending", c) + 8, np.uint8)
        n = call(J, "composerDigest", c, java.bytes(out))
        assert out[:n].tobytes() == ref.digest() and n > 0
        assert call(J, "composerPending", c) == 0
    finally:
        call(J, "composerFree", c)


def test_crc_composer_update_bytes_composes_up_to_a_failing_read(J, java):
    """CrcComposer.update(byte[], ...) reads one CRC at a time (CrcUtil.readInt), so the CRCs before a read past the
    array are composed when the IOException comes, as in the reference: the digest after the failure equals a fresh
    composer that saw only those CRCs."""
    crcs = np.array([0x11223344, 0x55667788, 0x99AABBCC], dtype=">u4").view(np.uint8)  # 12 bytes, big-endian
    c = call(J, "composerCreate", 3, 4, 0)
    ref = call(J, "composerCreate", 3, 4, 0)
    try:
        call(J, "composerUpdateBytes", c, java.bytes(crcs), 4, 12, 4)  # reads offsets 4, 8, then 12 fails
        assert java.exception() == ("java/io/IOException", "readInt out of bounds: buf.length=12, offset=12")
        call(J, "composerUpdateBytes", ref, java.bytes(crcs), 4, 8, 4)
        assert java.exception() is None
        a = np.zeros(8, np.uint8)
        b = np.zeros(8, np.uint8)
        na = call(J, "composerDigest", c, java.bytes(a))
        nb = call(J, "composerDigest", ref, java.bytes(b))
        assert na == nb == 4 and (a == b).all()
    finally:
        call(J, "composerFree", c)
        call(J, "composerFree", ref)


def test_crc_composer_natives_raise_the_reference_exceptions(J, java):
    c = call(J, "composerCreate", 3, 4, 10)
    try:
        call(J, "composerUpdate", c, 5, 4)
        call(J, "composerUpdate", c, 6, 4)
        assert java.exception() is None
        call(J, "composerUpdate", c, 7, 4)  # position 12 passes the 10-byte stripe
        ex = java.exception()
        assert ex[0] == "java/io/IOException" and "without stripe alignment" in ex[1]
        call(J, "composerUpdateBytes", c, java.bytes(np.zeros(8, np.uint8)), 0, 6, 4)
        ex = java.exception()
        assert ex == ("java/io/IOException", "Trying to update CRC from byte array with length '6' at offset '0' "
                                             "which is not a multiple of 4!")
        call(J, "composerUpdateBytes", c, java.bytes(np.zeros(8, np.uint8)), 6, 4, 4)
        assert java.exception() == ("java/io/IOException", "readInt out of bounds: buf.length=8, offset=6")
        call(J, "composerUpdateBytes", c, java.bytes(np.zeros(8, np.uint8)), -4, 8, 4)
        assert java.exception() == ("java/lang/ArrayIndexOutOfBoundsException", "Index -4 out of bounds for length 8")
        call(J, "composerUpdate", c, 1, -4)
        assert java.exception()[0] == "java/lang/IllegalArgumentException"
        call(J, "composerDigest", c, java.bytes(np.zeros(0, np.uint8)))  # pending bytes do not fit
        assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
    finally:
        call(J, "composerFree", c)
    assert call(J, "composerCreate", 5, 4, 0) == 0  # MD5
    assert java.exception()[0] == "java/io/IOException"
    assert call(J, "composerCreate", 3, -1, 0) == 0
    assert java.exception()[0] == "java/lang/IllegalArgumentException"
    call(J, "composerUpdate", 0, 1, 4)
    assert java.exception() == ("java/io/IOException", "CrcComposer closed")


# ------------------------------------------------------------------------------------------ GPU


@pytest.mark.gpu
@pytest.mark.parametrize("arrays", [False, True])
def test_encode_decode_vs_oracle(J, java, arrays):
    k, p, n, pos = 6, 3, 1 << 16, 11
    h = call(J, "coderCreate", 0, 0, k, p)
    hd = call(J, "coderCreate", 1, 0, k, p)
    assert java.exception() is None and h and hd
    try:
        wrap = java.bytes if arrays else java.direct
        enc_fn, dec_fn = ("encodeArrays", "decodeArrays") if arrays else ("encodeDirect", "decodeDirect")
        d = cells(SEED, 740000, k, n)
        ins = [np.zeros(n + 2 * pos, np.uint8) for _ in range(k)]
        for w, x in zip(ins, d):
            w[pos:pos + n] = x
        outs = [np.full(n + 2 * pos, 0xA5, np.uint8) for _ in range(p)]
        call(J, enc_fn, h, java.array([wrap(x) for x in ins]), java.ints([pos] * k), n,
             java.array([wrap(x) for x in outs]), java.ints([pos] * p))
        assert java.exception() is None
        ref = oracle.rs_encode(k, p, d)
        for o, r in zip(outs, ref):
            assert (o[pos:pos + n] == r).all() and (o[:pos] == 0xA5).all()
        units = d + ref
        erased = [1, 7]
        inputs = [None if u in erased else wrap(units[u]) for u in range(k + p)]
        rec = [np.zeros(n, np.uint8) for _ in erased]
        call(J, dec_fn, hd, java.array(inputs), java.ints([0] * (k + p)), n, java.ints(erased),
             java.array([wrap(r) for r in rec]), java.ints([0, 0]))
        assert java.exception() is None
        assert all((r == units[e]).all() for r, e in zip(rec, erased))
        # the reference's failures, with its exception classes
        call(J, enc_fn, h, java.array([wrap(x) for x in ins[:5]]), java.ints([pos] * 5), n,
             java.array([wrap(x) for x in outs]), java.ints([pos] * p))
        assert java.exception() == ("org/apache/hadoop/HadoopIllegalArgumentException", "Invalid inputs length 5 !=6")
        call(J, dec_fn, hd, java.array(inputs), java.ints([0] * (k + p)), n, java.ints([0, 1, 2, 3]),
             java.array([wrap(r) for r in rec] * 2), java.ints([0] * 4))
        assert java.exception()[1] == "Too many erased, not recoverable"
        if not arrays:  # a heap ByteBuffer in the direct path has no address
            call(J, "encodeDirect", h, java.array([java.heap(ins[0])] + [java.direct(x) for x in ins[1:]]),
                 java.ints([pos] * k), n, java.array([java.direct(x) for x in outs]), java.ints([pos] * p))
            assert "not a direct buffer" in java.exception()[1]
    finally:
        call(J, "coderRelease", h)
        call(J, "coderRelease", hd)


@pytest.mark.gpu
def test_checksums_and_streaming_update_vs_oracle(J, java):
    n, bpc = 70000, 16384
    data = cells(SEED, 741000, 1, n + 5)[0]
    out = np.zeros(4 * 5, np.uint8)
    assert call(J, "checksumWindowsArray", 3, java.bytes(data), 5, n, bpc, java.bytes(out)) == 20
    assert (out.view(">u4") == oracle.crc_windows(oracle.CRC32C, data[5:5 + n], bpc)).all()
    out[:] = 0
    assert call(J, "checksumWindowsDirect", 2, java.direct(data), 5, n, bpc, java.bytes(out)) == 20
    assert (out.view(">u4") == oracle.crc_windows(oracle.CRC32, data[5:5 + n], bpc)).all()
    state = -1  # reset(): 0xFFFFFFFF
    for lo, hi in ((0, 1), (1, 4000), (4000, 70005)):  # update(byte[]) then update(ByteBuffer) pieces
        fn = "crcUpdateArray" if lo == 0 else "crcUpdateDirect"
        state = call(J, fn, 3, state, java.bytes(data) if lo == 0 else java.direct(data), lo, hi - lo)
    assert java.exception() is None
    assert (~state) & 0xFFFFFFFF == oracle.crc_windows(oracle.CRC32C, data, n + 5)[0]


@pytest.mark.gpu
def test_device_list_natives(J, java):
    """OzecNative.setDevices / getDevices / setDevicePolicy / coderDevice (ozone.ec.hip.devices): a list of the one
    GPU twice, coders bound to it, a bad ordinal refused with the device exception, the default restored."""
    call(J, "setDevices", java.ints([0, 0]))
    assert java.exception() is None
    arr = call(J, "getDevices")
    assert J.mock_len(arr) == 2 and list(np.ctypeslib.as_array(ctypes.cast(J.mock_data(arr), ctypes.POINTER(
        ctypes.c_int32)), (2,))) == [0, 0]
    J.mock_free(arr)
    h = call(J, "coderCreate", 0, 0, 6, 3)
    assert call(J, "coderDevice", h) == 0
    call(J, "coderRelease", h)
    call(J, "setDevices", java.ints([99]))
    assert java.exception()[0] == "java/io/IOException"
    call(J, "setDevicePolicy", 9)
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
    call(J, "setDevices", java.ints([]))
    assert java.exception() is None
    call(J, "coderDevice", 0)
    assert java.exception()[0] == "java/io/IOException"


HEAP_AUTO, HEAP_CB, HEAP_ARENA = 0, 1, 2


def heap_forms(J):
    cb, ar = ctypes.c_ulong(), ctypes.c_ulong()
    J.ozec_jni_heap_mode(-1, ctypes.byref(cb), ctypes.byref(ar))
    return cb.value, ar.value


@pytest.fixture(params=[HEAP_CB, HEAP_ARENA], ids=["callback", "arena"])
def heap_form(J, request):
    """the two forms a heap-array coder call can take (jni/ozec_jni.c heap_code): libozec's staged pipeline with the
    glue's fill / drain callbacks, or a pinned arena around an in-place call"""
    prev = J.ozec_jni_heap_mode(request.param, None, None)
    before = heap_forms(J)
    yield request.param
    after = heap_forms(J)
    J.ozec_jni_heap_mode(prev, None, None)
    took = after[0] - before[0] if request.param == HEAP_CB else after[1] - before[1]
    assert took > 0 and sum(after) - sum(before) == took, "a call took the other form"


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1 << 16, (4 << 20) + 4096 + 3])  # one chunk; two chunks of the 4 MiB arena
def test_heap_arrays_never_pinned_across_device_work(J, java, heap_form, n):
    """byte[] inputs and outputs are copied into a pooled pinned arena (coder calls: the arrays held
    critical for the parallel copy only, ozec_host_copy; checksum calls: Get/SetByteArrayRegion), and no array is
    pinned while libozec works -- the mock records the array pins outstanding at every wrapped ozec_encode /
    ozec_decode / ozec_crc_update / ozec_checksum_windows call.  Results vs the oracle, calls longer than one arena
    chunk included, inputs untouched and outputs written only inside their regions."""
    k, p, pos = 3, 2, 7
    h = call(J, "coderCreate", 0, 0, k, p)
    hd = call(J, "coderCreate", 1, 0, k, p)
    try:
        J.mock_reset_device_calls()
        copies0 = J.mock_region_copies()
        d = cells(SEED, 742000 + n % 97, k, n)
        ins = [np.zeros(n + 2 * pos, np.uint8) for _ in range(k)]
        for w, x in zip(ins, d):
            w[pos:pos + n] = x
        keep = [w.copy() for w in ins]
        outs = [np.full(n + 2 * pos, 0xA5, np.uint8) for _ in range(p)]
        call(J, "encodeArrays", h, java.array([java.bytes(x) for x in ins]), java.ints([pos] * k), n,
             java.array([java.bytes(x) for x in outs]), java.ints([pos] * p))
        assert java.exception() is None
        ref = oracle.rs_encode(k, p, d)
        for o, r in zip(outs, ref):
            assert (o[pos:pos + n] == r).all() and (o[:pos] == 0xA5).all() and (o[pos + n:] == 0xA5).all()
        assert all((a == b).all() for a, b in zip(ins, keep))
        units = d + ref
        erased = [0, 4]
        inputs = [None if u in erased else java.bytes(units[u]) for u in range(k + p)]
        rec = [np.zeros(n, np.uint8) for _ in erased]
        call(J, "decodeArrays", hd, java.array(inputs), java.ints([0] * (k + p)), n, java.ints(erased),
             java.array([java.bytes(r) for r in rec]), java.ints([0, 0]))
        assert java.exception() is None
        assert all((r == units[e]).all() for r, e in zip(rec, erased))
        bpc = 16384
        nw = (n + bpc - 1) // bpc
        out = np.zeros(4 * nw, np.uint8)
        assert call(J, "checksumWindowsArray", 3, java.bytes(ins[0]), pos, n, bpc, java.bytes(out)) == 4 * nw
        assert (out.view(">u4") == oracle.crc_windows(oracle.CRC32C, d[0], bpc)).all()
        out[:] = 0
        assert call(J, "checksumWindowsDirect", 2, java.direct(ins[1]), pos, n, bpc, java.bytes(out)) == 4 * nw
        assert (out.view(">u4") == oracle.crc_windows(oracle.CRC32, d[1], bpc)).all()
        state = call(J, "crcUpdateArray", 3, -1, java.bytes(ins[2]), pos, n)
        assert java.exception() is None
        assert (~state) & 0xFFFFFFFF == oracle.crc_windows(oracle.CRC32C, d[2], n)[0]
        assert J.mock_device_calls() >= 5
        assert J.mock_pins_at_device_call() == 0, "an array was pinned while libozec did device work"
        assert J.mock_pins_after_callback() == 0, "a fill / drain callback returned to libozec with an array pinned"
        assert J.mock_region_copies() > copies0
        assert J.mock_pins() == 0
    finally:
        call(J, "coderRelease", h)
        call(J, "coderRelease", hd)


@pytest.mark.gpu
@pytest.mark.parametrize("refuse_after", [0, 2, 3])  # the first input pin, the last one, the first output pin
def test_refused_array_pin_leaves_its_exception_and_no_further_jni_call(J, java, heap_form, refuse_after):
    """a JVM that cannot pin an array (GetPrimitiveArrayCritical -> NULL, OutOfMemoryError pending) ends the
    copy: the arrays already pinned are released without write-back, the exception stays the pending one (no JNI call
    but ExceptionCheck / Release / DeleteLocalRef runs while it is pending), outputs stay untouched, and the next call
    works."""
    k, p, n = 3, 2, 1 << 16
    h = call(J, "coderCreate", 0, 0, k, p)
    try:
        d = cells(SEED, 743000 + refuse_after, k, n)
        outs = [np.full(n, 0xA5, np.uint8) for _ in range(p)]
        pending0 = J.mock_calls_with_pending()
        J.mock_refuse_pin_after(refuse_after)
        call(J, "encodeArrays", h, java.array([java.bytes(x) for x in d]), java.ints([0] * k), n,
             java.array([java.bytes(x) for x in outs]), java.ints([0] * p))
        assert java.exception() == ("java/lang/OutOfMemoryError", "could not pin the array")
        assert J.mock_calls_with_pending() == pending0, "a JNI call ran with the exception pending"
        assert J.mock_pins() == 0
        assert all((o == 0xA5).all() for o in outs)
        call(J, "encodeArrays", h, java.array([java.bytes(x) for x in d]), java.ints([0] * k), n,
             java.array([java.bytes(x) for x in outs]), java.ints([0] * p))
        assert java.exception() is None
        assert all((o == r).all() for o, r in zip(outs, oracle.rs_encode(k, p, d)))
    finally:
        J.mock_refuse_pin_after(-1)
        call(J, "coderRelease", h)


@pytest.mark.gpu
def test_heap_arenas_are_pooled_across_threads(J, java):
    """The pinned arenas heap-array checksum calls copy through come from a bounded pool, not one per Java thread: 24
    threads calling one after another reuse one arena (no new pinned allocation after the first); coder calls copy
    into libozec's own staging (ozec_encode_cb) and allocate no arena at all; the results stay exact."""
    import threading
    k, p, n, bpc = 6, 3, 50_000, 4096
    h = call(J, "coderCreate", 0, 0, k, p)
    try:
        d = cells(SEED, 748000, k, n)
        ref = oracle.rs_encode(k, p, d)
        nw = (n + bpc - 1) // bpc
        crc_ref = oracle.crc_windows(oracle.CRC32C, d[0], bpc)

        def one():
            outs = [np.zeros(n, np.uint8) for _ in range(p)]
            call(J, "encodeArrays", h, java.array([java.bytes(x) for x in d]), java.ints([0] * k), n,
                 java.array([java.bytes(x) for x in outs]), java.ints([0] * p))
            assert java.exception() is None
            assert all((o == r).all() for o, r in zip(outs, ref))
            c = np.zeros(4 * nw, np.uint8)
            assert call(J, "checksumWindowsArray", 3, java.bytes(d[0]), 0, n, bpc, java.bytes(c)) == 4 * nw
            assert (c.view(">u4") == crc_ref).all()

        one()  # the first call sizes an arena
        allocs0, live0 = J.mock_host_allocs(), J.mock_host_live()
        for _ in range(24):
            t = threading.Thread(target=one)
            t.start()
            t.join()
        assert J.mock_host_allocs() == allocs0, "a thread got a pinned arena of its own"
        assert J.mock_host_live() == live0
    finally:
        call(J, "coderRelease", h)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [300_000, 65536 - 3])  # copy path beside other calls; zero copy (host_zc_shared_max)
def test_concurrent_heap_calls_take_either_form_exactly(J, java, n):
    """Default (auto) form choice: a call alone takes the callback form, a call made while another coder call is in
    flight takes the arena form (whose libozec call codes the arena in place: by DMA for large cells, zero copy for cells
    up to host_zc_shared_max).  Eight threads encoding and decoding at once: every call exact, every call counted under
    one of the two forms, and a call alone afterwards takes the callback form."""
    import threading
    k, p = 6, 3
    prev = J.ozec_jni_heap_mode(HEAP_AUTO, None, None)
    h = call(J, "coderCreate", 0, 0, k, p)
    hd = call(J, "coderCreate", 1, 0, k, p)
    errors = []
    try:
        d = cells(SEED, 749000, k, n)
        ref = oracle.rs_encode(k, p, d)
        units = d + ref
        # erasure patterns, some listing a parity unit before a data unit: those decode with the reference's ordering
        # quirk (oracle/ozec_oracle.c oracle_rs_decode_matrix), so the expected outputs are the oracle's
        patterns = [[t % (k + p), (t + 4) % (k + p)] for t in range(8)]
        want = [oracle.rs_decode(k, p, [None if u in e else units[u] for u in range(k + p)], e) for e in patterns]
        before = heap_forms(J)

        def worker(t):
            try:
                for i in range(6):
                    outs = [np.zeros(n, np.uint8) for _ in range(p)]
                    call(J, "encodeArrays", h, java.array([java.bytes(x) for x in d]), java.ints([0] * k), n,
                         java.array([java.bytes(x) for x in outs]), java.ints([0] * p))
                    assert all((o == r).all() for o, r in zip(outs, ref)), f"encode {t}/{i}"
                    erased = patterns[t]
                    rec = [np.zeros(n, np.uint8) for _ in erased]
                    call(J, "decodeArrays", hd, java.array([None if u in erased else java.bytes(units[u])
                                                            for u in range(k + p)]),
                         java.ints([0] * (k + p)), n, java.ints(erased), java.array([java.bytes(r) for r in rec]),
                         java.ints([0, 0]))
                    assert all((r == w).all() for r, w in zip(rec, want[t])), f"decode {t}/{i}"
            except Exception as e:  # noqa: BLE001 - reported below
                errors.append(e)

        ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors
        mid = heap_forms(J)
        assert sum(mid) - sum(before) == 8 * 6 * 2
        outs = [np.zeros(n, np.uint8) for _ in range(p)]
        call(J, "encodeArrays", h, java.array([java.bytes(x) for x in d]), java.ints([0] * k), n,
             java.array([java.bytes(x) for x in outs]), java.ints([0] * p))
        assert all((o == r).all() for o, r in zip(outs, ref))
        after = heap_forms(J)
        assert after[0] == mid[0] + 1 and after[1] == mid[1], "a call alone did not take the callback form"
    finally:
        J.ozec_jni_heap_mode(prev, None, None)
        call(J, "coderRelease", h)
        call(J, "coderRelease", hd)


@pytest.mark.gpu
def test_compose_windows_batch_through_jni(J, java):
    """composeWindowsBatch on device pointers (a GPU pipeline's window CRCs): the composite CRC of every cell equals
    the CRC of the whole cell."""
    import torch
    from devcopy import to_dev, to_host
    n, bpc, C = 100_000, 4096, 5
    nwin = (n + bpc - 1) // bpc
    data = np.stack(cells(SEED, 747000, C, n))
    win = np.stack([oracle.crc_windows(oracle.CRC32C, data[c], bpc) for c in range(C)]).astype(np.uint32)
    d_win = to_dev(win.view(np.int32))
    d_out = torch.zeros(C, dtype=torch.int32, device="cuda")
    call(J, "composeWindowsBatch", 3, d_win.data_ptr(), nwin, C, nwin, bpc, n - (nwin - 1) * bpc, 0, d_out.data_ptr(),
         0, 0)
    assert java.exception() is None
    torch.cuda.synchronize()
    got = to_host(d_out).view(np.uint32)
    assert [int(v) for v in got] == [oracle.crc_windows(oracle.CRC32C, data[c], n)[0] for c in range(C)]
    call(J, "composeWindowsBatch", 3, d_win.data_ptr(), nwin, -1, nwin, bpc, 1, 0, d_out.data_ptr(), 0, 0)
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"


@pytest.mark.gpu
def test_pinned_buffers_and_stripe_queue_through_jni(J, java):
    k, p, n, bpc = 6, 3, 1 << 15, 8192
    h = call(J, "coderCreate", 0, 0, k, p)
    q = call(J, "queueCreate", h, n, 2, 3, bpc)
    assert java.exception() is None and q
    slabs, jobs = [], []
    try:
        for s in range(5):
            pb = call(J, "allocatePinned", (k + p) * n)
            assert java.exception() is None and pb
            slabs.append(pb)
            view = np.ctypeslib.as_array((ctypes.c_uint8 * ((k + p) * n)).from_address(J.mock_data(pb)))
            for j, x in enumerate(cells(SEED, 742000 + 10 * s, k, n)):
                view[j * n:(j + 1) * n] = x
            crcs = np.zeros((k + p) * (n // bpc), np.uint32)
            cells_d = java.array([pb] * k)
            cells_p = java.array([pb] * p)
            t = call(J, "queueSubmit", q, cells_d, java.ints([j * n for j in range(k)]), cells_p,
                     java.ints([(k + r) * n for r in range(p)]), n, java.direct(crcs.view(np.uint8)), 0)
            assert java.exception() is None
            jobs.append((t, view, crcs))
        call(J, "queueWait", q, jobs[-1][0])
        assert java.exception() is None
        for t, view, crcs in jobs:
            d = [view[j * n:(j + 1) * n].copy() for j in range(k)]
            ref = oracle.rs_encode(k, p, d)
            assert all((view[(k + r) * n:(k + r + 1) * n] == ref[r]).all() for r in range(p)), t
            exp = np.concatenate([oracle.crc_windows(oracle.CRC32C, u, bpc) for u in d + ref])
            assert (crcs.byteswap() == exp).all(), t
    finally:
        call(J, "queueFree", q)
        for pb in slabs:
            call(J, "freePinned", pb)
            J.mock_free(pb)
        call(J, "coderRelease", h)
    assert java.exception() is None


@pytest.mark.gpu
def test_stripe_queue_submit_checks_and_encoder_lifetime(J, java):
    """queueSubmit checks the cell counts against the queue and the CRC buffer's room from its position (the
    native side writes (k + p) * windows ints there); a queue keeps its encoder's native handle alive, so releasing
    the encoder first makes submits fail with the reference's "closed" IOException and queueFree stays safe
    (HipStripeQueue.java:32 / ozec_jni.c:372)."""
    k, p, n, bpc = 6, 3, 1 << 14, 4096
    nwin = n // bpc
    cells_ = [np.asarray(x) for x in cells(SEED, 746000, k, n)]
    par = [np.zeros(n, np.uint8) for _ in range(p)]
    h = call(J, "coderCreate", 0, 0, k, p)
    q = call(J, "queueCreate", h, n, 4, 3, bpc)
    assert java.exception() is None and q

    def submit(nd=k, np_=p, crc=None, crc_off=0, length=n):
        return call(J, "queueSubmit", q, java.array([java.direct(x) for x in cells_[:nd]]), java.ints([0] * nd),
                    java.array([java.direct(x) for x in par[:np_]] + [java.direct(par[0])] * (np_ - p)),
                    java.ints([0] * np_), length, None if crc is None else java.direct(crc), crc_off)
    try:
        submit(nd=5)
        ex = java.exception()
        assert ex[0] == "org/apache/hadoop/HadoopIllegalArgumentException" and "Invalid inputs/outputs length" in ex[1]
        submit(np_=4)
        assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
        small = np.zeros((k + p) * nwin * 4 - 4, np.uint8)          # one CRC short
        submit(crc=small)
        ex = java.exception()
        assert ex[0] == "org/apache/hadoop/HadoopIllegalArgumentException" and "too small" in ex[1]
        roomy = np.zeros((k + p) * nwin * 4 + 64, np.uint8)
        submit(crc=roomy, crc_off=68)                                # the position leaves 60 bytes short
        assert "too small" in java.exception()[1]
        submit(length=n + 1)
        assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"
        t = submit(crc=roomy, crc_off=64)
        assert java.exception() is None
        call(J, "queueWait", q, t)
        assert java.exception() is None
        crcs = roomy[64:].view(">u4")
        ref = oracle.rs_encode(k, p, cells_)
        assert all((par[r] == ref[r]).all() for r in range(p))
        exp = np.concatenate([oracle.crc_windows(oracle.CRC32C, u, bpc) for u in cells_ + ref])
        assert (crcs == exp).all() and not roomy[:64].any()
        call(J, "coderRelease", h)                                   # encoder released while the queue lives
        h = 0
        submit(crc=roomy, crc_off=64)
        ex = java.exception()
        assert ex[0] == "java/io/IOException" and "closed" in ex[1]
    finally:
        call(J, "queueFree", q)
        if h:
            call(J, "coderRelease", h)
    assert java.exception() is None


def test_reconstruct_batch_argument_errors(J, java):
    """reconstructHostBatch: heap buffers and a closed handle raise the reference's exceptions before anything runs
    (size checks against a live decoder: test_reconstruct_batch_through_jni)."""
    k, p, n, S, bpc = 6, 3, 4096, 2, 4096
    stripes = np.zeros(S * (k + p) * n, np.uint8)
    out, crc = np.zeros(S * n, np.uint8), np.zeros(S * 4, np.uint8)
    present, erased = list(range(1, 9)), [0]
    call(J, "reconstructHostBatch", 0, java.heap(stripes), (k + p) * n, n, java.ints(present), java.ints(erased),
         java.direct(out), S, n, 3, bpc, None, java.direct(crc), None)
    assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"  # not a direct buffer
    call(J, "reconstructHostBatch", 0, java.direct(stripes), (k + p) * n, n, java.ints(present), java.ints(erased),
         java.direct(out), S, n, 3, bpc, None, java.direct(crc), None)
    ex = java.exception()
    assert ex and ex[0] == "java/io/IOException" and "closed" in ex[1]


@pytest.mark.gpu
def test_reconstruct_batch_through_jni(J, java):
    """reconstructHostBatch over pinned direct buffers vs the oracle: rebuilt units, their big-endian CRCs and the
    per-stripe verdicts (one stripe corrupted)."""
    k, p, n, S, bpc = 10, 4, 1 << 15, 5, 4096
    nwin = n // bpc
    h = call(J, "coderCreate", 1, 0, k, p)
    pbs = []
    try:
        def pinned(nbytes):
            pb = call(J, "allocatePinned", nbytes)
            assert java.exception() is None and pb
            pbs.append(pb)
            return pb, np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(J.mock_data(pb)))
        sb, sv = pinned(S * (k + p) * n)
        eb, ev = pinned(S * (k + p) * nwin * 4)
        ob, ov = pinned(S * 4 * n)
        cb, cv = pinned(S * 4 * nwin * 4)
        mb, mv = pinned(S * 4)
        stripes = sv.reshape(S, k + p, n)
        for s in range(S):
            d = cells(SEED, 745000 + s * k, k, n)
            for u, x in enumerate(d + oracle.rs_encode(k, p, d)):
                stripes[s, u] = x
        orig = stripes.copy()
        ev.view(np.uint32)[:] = np.concatenate([oracle.crc_windows(oracle.CRC32C, orig[s, u], bpc)
                                                for s in range(S) for u in range(k + p)]).byteswap()
        erased = [1, 4, 10, 13]
        present = [u for u in range(k + p) if u not in erased]
        small = java.direct(np.zeros(n, np.uint8))
        call(J, "reconstructHostBatch", h, sb, (k + p) * n, n, java.ints(present), java.ints(erased), small, S, n, 3,
             bpc, eb, cb, mb)
        ex = java.exception()
        assert ex[0] == "org/apache/hadoop/HadoopIllegalArgumentException" and "too small" in ex[1]
        call(J, "reconstructHostBatch", h, sb, (k + p) * n, n, java.ints(present[:9]), java.ints(erased + [0]), ob, S,
             n, 3, bpc, eb, cb, mb)
        assert java.exception()[0] == "org/apache/hadoop/HadoopIllegalArgumentException"  # 5 erased of 4 parity
        for stride in (1 << 62, (1 << 63) - 1):  # strides whose layout size wraps int64: rejected, nothing read
            call(J, "reconstructHostBatch", h, sb, stride, n, java.ints(present), java.ints(erased), ob, S, n, 3, bpc,
                 eb, cb, mb)
            ex = java.exception()
            assert ex[0] == "org/apache/hadoop/HadoopIllegalArgumentException" and "overflows" in ex[1], stride
        call(J, "reconstructHostBatch", h, sb, (k + p) * n, 1 << 61, java.ints(present), java.ints(erased), ob, S, n,
             3, bpc, eb, cb, mb)
        assert "overflows" in java.exception()[1]
        stripes[:, erased] = 0
        stripes[3, 12, 5] ^= 0x80                 # stripe 3: the last unit read is corrupted in window 0
        call(J, "reconstructHostBatch", h, sb, (k + p) * n, n, java.ints(present), java.ints(erased), ob, S, n, 3, bpc,
             eb, cb, mb)
        assert java.exception() is None
        got, crcs, mism = ov.reshape(S, 4, n), cv.view(np.uint32).reshape(S, 4, nwin), mv.view(np.int32)
        assert list(mism) == [-1, -1, -1, 12 * nwin + 0, -1]
        for s in (0, 1, 2, 4):
            for i, u in enumerate(erased):
                assert (got[s, i] == orig[s, u]).all(), (s, u)
                assert (crcs[s, i].byteswap() == oracle.crc_windows(oracle.CRC32C, orig[s, u], bpc)).all(), (s, u)
    finally:
        for pb in pbs:
            call(J, "freePinned", pb)
            J.mock_free(pb)
        call(J, "coderRelease", h)
    assert java.exception() is None

