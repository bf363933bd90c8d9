"""ozec_encode_cb / ozec_decode_cb (round 6): host coding with the caller moving the bytes (GPU).

libozec's staged pipeline asks `fill(off, len, dst)` for bytes [off, off + len) of every input unit (decode: k + p slots
by unit, null for the units it does not read) and hands `drain(off, len, src)` the outputs, column chunk by column
chunk -- what the JNI glue does for Java heap arrays (jni/ozec_jni.c heap_code).  Checked here through ctypes callbacks
against the oracle: RS and XOR (XOR with p > 1: outputs past the first drained as zeros, XORRawEncoder.java:67-85;
XOR decode: outputs past erasedIndexes[0] zero, XORRawDecoder.java:45-61), lengths across the zero-copy chunking and
the copy path, chunk offsets that tile the call exactly once, which slots a decode fill is handed, and a failing fill /
drain ending the call with its status while the next call still works."""
import ctypes

import numpy as np
import pytest

import oracle
from synth import SEED, cells

pytestmark = pytest.mark.gpu

from ozone_amd import _lib as L  # noqa: E402


def _coder(decoder, codec, k, p):
    h = ctypes.c_void_p()
    make = L.lib().ozec_decoder_create if decoder else L.lib().ozec_encoder_create
    assert make(codec, k, p, ctypes.byref(h)) == 0, L.last_error()
    return h


def _free(h):
    L.lib().ozec_coder_release(h)
    L.lib().ozec_coder_free(h)


class Mover:
    """fill / drain callbacks over numpy units, recording every (off, len) they are handed"""

    def __init__(self, inputs, outputs, fail_fill_at=None, fail_drain_at=None):
        self.inputs, self.outputs = inputs, outputs
        self.fills, self.drains, self.fill_slots = [], [], []
        self.fail_fill_at, self.fail_drain_at = fail_fill_at, fail_drain_at
        self.errors = []  # exceptions inside a callback (ctypes would only print them): reported by check()
        self.fill = L.FILL_FN(lambda *a: self._guard(self._fill, *a))
        self.drain = L.DRAIN_FN(lambda *a: self._guard(self._drain, *a))

    def _guard(self, fn, *args):
        try:
            return fn(*args)
        except Exception as e:  # noqa: BLE001 - surfaced by check()
            self.errors.append(e)
            return -99

    def check(self):
        assert not self.errors, self.errors

    def _fill(self, user, off, n, dst):
        if self.fail_fill_at is not None and len(self.fills) == self.fail_fill_at:
            return -77
        self.fills.append((off, n))
        slots = []
        for j, x in enumerate(self.inputs):
            if not dst[j]:
                slots.append(False)
                continue
            slots.append(True)
            assert x is not None, f"fill handed a slot for unit {j}, which the caller does not hold"
            ctypes.memmove(dst[j], x[off:off + n].ctypes.data, n)
        self.fill_slots.append(slots)
        return 0

    def _drain(self, user, off, n, src):
        if self.fail_drain_at is not None and len(self.drains) == self.fail_drain_at:
            return -78
        self.drains.append((off, n))
        for r, o in enumerate(self.outputs):
            assert src[r], f"drain handed a null output {r}"
            ctypes.memmove(o[off:off + n].ctypes.data, src[r], n)
        return 0


def _tiles(calls, n):
    """the (off, len) pieces cover [0, n) exactly once, in order"""
    pos = 0
    for off, ln in calls:
        assert off == pos and ln > 0, calls
        pos += ln
    assert pos == n, calls


@pytest.mark.parametrize("codec,k,p,n", [("rs", 6, 3, 1 << 20), ("rs", 6, 3, (3 << 20) + 17), ("rs", 10, 4, 65536 + 5),
                                         ("rs", 3, 2, 1), ("xor", 2, 1, 700_001), ("xor", 3, 2, 300_000)])
@pytest.mark.parametrize("zc", [48, 0])
def test_encode_cb_vs_oracle(codec, k, p, n, zc):
    lib = L.lib()
    assert lib.ozec_set_tuning(b"host_zero_copy", zc) == 0
    h = _coder(False, L.OZEC_CODEC_RS if codec == "rs" else L.OZEC_CODEC_XOR, k, p)
    try:
        data = cells(SEED, 752000 + n % 89 + k, k, n)
        ref = oracle.rs_encode(k, p, data) if codec == "rs" else [oracle.xor_encode(data)] + \
            [np.zeros(n, np.uint8)] * (p - 1)
        outs = [np.full(n, 0xA5, np.uint8) for _ in range(p)]
        m = Mover(data, outs)
        assert lib.ozec_encode_cb(h, n, m.fill, m.drain, None) == 0, (L.last_error(), m.errors)
        m.check()
        assert all((o == r).all() for o, r in zip(outs, ref)), (codec, k, p, n, zc)
        _tiles(m.fills, n)
        _tiles(m.drains, n)
    finally:
        lib.ozec_set_tuning(b"host_zero_copy", 48)
        _free(h)


@pytest.mark.parametrize("codec,k,p,n,erased,absent", [
    ("rs", 6, 3, 1 << 20, [0, 7], [0, 7]),
    ("rs", 6, 3, 400_003, [2], [2, 8]),           # unit 8 also absent: the first k valid are read
    ("rs", 10, 4, 65536, [1, 4, 10, 13], [1, 4, 10, 13]),
    ("rs", 6, 3, 200_000, [7, 2], [2, 7]),        # parity listed first: the reference's ordering quirk
    ("xor", 3, 2, 100_000, [1, 3], [1]),          # XOR: only erasedIndexes[0] is rebuilt, the rest is zero
])
def test_decode_cb_vs_oracle(codec, k, p, n, erased, absent):
    lib = L.lib()
    h = _coder(True, L.OZEC_CODEC_RS if codec == "rs" else L.OZEC_CODEC_XOR, k, p)
    try:
        data = cells(SEED, 753000 + n % 83 + k, k, n)
        par = oracle.rs_encode(k, p, data) if codec == "rs" else [oracle.xor_encode(data)] + \
            [np.zeros(n, np.uint8)] * (p - 1)
        units = list(data) + list(par)
        inputs = [None if u in absent else units[u] for u in range(k + p)]
        if codec == "rs":
            want = oracle.rs_decode(k, p, inputs, erased)
        else:
            want = [oracle.xor_decode([None if u == erased[0] else units[u] for u in range(k + p)], erased[0])] + \
                [np.zeros(n, np.uint8)] * (len(erased) - 1)
        outs = [np.full(n, 0x5A, np.uint8) for _ in erased]
        m = Mover(inputs, outs)
        present = (ctypes.c_uint8 * (k + p))(*[x is not None for x in inputs])
        er = (ctypes.c_int * len(erased))(*erased)
        assert lib.ozec_decode_cb(h, present, er, len(erased), n, m.fill, m.drain, None) == 0, (L.last_error(), m.errors)
        m.check()
        assert all((o == w).all() for o, w in zip(outs, want)), (codec, k, p, erased)
        _tiles(m.fills, n)
        _tiles(m.drains, n)
        # the slots a fill is handed: the first k present units for RS, every unit but erasedIndexes[0] for XOR
        read = [u for u in range(k + p) if inputs[u] is not None][:k] if codec == "rs" else \
            [u for u in range(k + p) if u != erased[0]]
        assert all(s == [u in read for u in range(k + p)] for s in m.fill_slots), m.fill_slots[0]
    finally:
        _free(h)


@pytest.mark.parametrize("where", ["fill0", "fill1", "drain0", "drain1"])
def test_callback_failure_ends_the_call_and_the_next_works(where):
    """a nonzero fill / drain status ends the call with that status (no further callback), the slot's stream is
    drained, and the next call on the same coder is exact"""
    lib = L.lib()
    k, p, n = 6, 3, 2 << 20  # two column chunks when zero copy splits a lone call
    h = _coder(False, L.OZEC_CODEC_RS, k, p)
    try:
        data = cells(SEED, 754000, k, n)
        ref = oracle.rs_encode(k, p, data)
        outs = [np.zeros(n, np.uint8) for _ in range(p)]
        kind, at = where[:-1], int(where[-1])
        m = Mover(data, outs, fail_fill_at=at if kind == "fill" else None,
                  fail_drain_at=at if kind == "drain" else None)
        rc = lib.ozec_encode_cb(h, n, m.fill, m.drain, None)
        m.check()
        assert rc == (-77 if kind == "fill" else -78), (rc, m.fills, m.drains)
        assert len(m.fills if kind == "fill" else m.drains) == at
        outs2 = [np.zeros(n, np.uint8) for _ in range(p)]
        m2 = Mover(data, outs2)
        assert lib.ozec_encode_cb(h, n, m2.fill, m2.drain, None) == 0, (L.last_error(), m2.errors)
        m2.check()
        assert all((o == r).all() for o, r in zip(outs2, ref))
    finally:
        _free(h)


def test_callback_argument_errors():
    lib = L.lib()
    h = _coder(False, L.OZEC_CODEC_RS, 6, 3)
    hd = _coder(True, L.OZEC_CODEC_RS, 6, 3)
    try:
        m = Mover([], [])
        assert lib.ozec_encode_cb(hd, 16, m.fill, m.drain, None) != 0  # not an encoder
        assert lib.ozec_encode_cb(h, 0, m.fill, m.drain, None) == 0 and not m.fills  # len 0: nothing to move
        present = (ctypes.c_uint8 * 9)(*([0] * 9))
        er = (ctypes.c_int * 1)(0)
        assert lib.ozec_decode_cb(hd, present, er, 1, 16, m.fill, m.drain, None) != 0  # all inputs absent
        assert "all being null" in L.last_error()
        present = (ctypes.c_uint8 * 9)(*([1] * 5 + [0] * 4))
        assert lib.ozec_decode_cb(hd, present, er, 1, 16, m.fill, m.drain, None) != 0  # fewer than k valid
        assert "No enough valid inputs" in L.last_error()
    finally:
        _free(h)
        _free(hd)
