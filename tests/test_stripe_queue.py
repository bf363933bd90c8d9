"""writer-side stripe batching (ozec_stripe_queue_*) against the oracle, bit-exact."""
import numpy as np
import pytest

import oracle
from synth import SEED, cells

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from ozone_amd import rawcoder as rc  # noqa: E402
from ozone_amd.checksum import ChecksumType  # noqa: E402
from ozone_amd.stripe_queue import StripeQueue, host_alloc  # noqa: E402


def _stripe(first, k, n, pinned, keep):
    d = cells(SEED, first, k, n)
    if not pinned:
        return d
    out = []
    for x in d:
        pb = host_alloc(n)
        pb.array[:] = x
        keep.append(pb)
        out.append(pb.array)
    return out


def _parity(p, n, pinned, keep):
    if not pinned:
        return [np.full(n, 0xA5, np.uint8) for _ in range(p)]
    out = []
    for _ in range(p):
        pb = host_alloc(n)
        pb.array[:] = 0xA5
        keep.append(pb)
        out.append(pb.array)
    return out


@pytest.mark.parametrize("codec,k,p", [("rs", 6, 3), ("rs", 3, 2), ("rs", 10, 4), ("xor", 2, 1), ("xor", 3, 2)])
@pytest.mark.parametrize("ctype,otype", [(ChecksumType.NONE, None), (ChecksumType.CRC32C, oracle.CRC32C)])
def test_queue_matches_oracle(codec, k, p, ctype, otype):
    n, bpc, S = 65536, 16384, 4
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec))
    keep, jobs = [], []
    with StripeQueue(enc, n, S, ctype, bpc, big_endian=True) as q:
        for s in range(11):  # two full batches + a partial one, pinned and pageable buffers mixed
            pinned = s % 3 == 1
            d = _stripe(90000 + 100 * s, k, n, pinned, keep)
            par = _parity(p, n, pinned and s % 2 == 1, keep)
            crcs = np.zeros((k + p) * (n // bpc), np.uint32) if otype is not None else None
            jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs))
        q.wait(jobs[-1][0])
    for t, d, par, crcs in jobs:
        ref = oracle.rs_encode(k, p, d) if codec == "rs" else [oracle.xor_encode(d)] + [np.zeros(n, np.uint8)] * (p - 1)
        assert all((a == b).all() for a, b in zip(par, ref)), t
        if otype is not None:
            exp = np.concatenate([oracle.crc_windows(otype, u, bpc) for u in list(d) + ref[:1 if codec == "xor" else p]])
            got = crcs.byteswap()[:exp.size]
            assert (got == exp).all(), t


def test_queue_mixed_lengths_and_wait_order():
    k, p, cell = 6, 3, 1 << 16
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    q = StripeQueue(enc, cell, 8, ChecksumType.CRC32, 4096)
    jobs = []
    for s, n in enumerate([cell, cell, 1000, 4096 + 16, cell, 17, cell]):
        d = cells(SEED, 91000 + 100 * s, k, n)
        par = [np.zeros(n, np.uint8) for _ in range(p)]
        crcs = np.zeros((k + p) * ((n + 4095) // 4096), np.uint32)
        jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs, n))
    q.wait(jobs[3][0])  # stripes 0..3 are complete now, whatever batch they were in
    for t, d, par, crcs, n in jobs[:4]:
        ref = oracle.rs_encode(k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), t
    q.flush()
    q.wait(jobs[-1][0])
    for t, d, par, crcs, n in jobs:
        ref = oracle.rs_encode(k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), t
        exp = np.concatenate([oracle.crc_windows(oracle.CRC32, u, 4096) for u in list(d) + ref])
        assert (crcs == exp).all(), t
    q.close()


def test_queue_many_batches_rotate():
    k, p, n = 6, 3, 4096
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    jobs = []
    with StripeQueue(enc, n, 5) as q:
        for s in range(203):
            d = cells(SEED, 92000 + 10 * s, k, n)
            par = [np.zeros(n, np.uint8) for _ in range(p)]
            jobs.append((q.submit(d, par), d, par))
            if s % 50 == 49:
                q.wait(jobs[s - 7][0])
        q.wait(jobs[-1][0])
    for t, d, par in jobs:
        ref = oracle.rs_encode(k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), t


def test_queue_errors():
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(6, 3))
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(6, 3))
    with pytest.raises(Exception):
        StripeQueue(dec, 4096)
    q = StripeQueue(enc, 4096)
    with pytest.raises(Exception):
        q.submit(cells(SEED, 1, 6, 8192), [np.zeros(8192, np.uint8)] * 3)  # longer than cell_len
    with pytest.raises(Exception):
        q.wait(5)  # no such ticket yet
    with pytest.raises(rc.IllegalArgumentException):
        q.submit(cells(SEED, 1, 5, 4096), [np.zeros(4096, np.uint8)] * 3)
    q.close()


@pytest.mark.parametrize("n", [1 << 16, 5000])
def test_queue_contiguous_pinned_stripe(n):
    """Cells back to back in one pinned buffer (one H2D and one D2H copy per stripe when len == cell_len)."""
    k, p, cell = 6, 3, 1 << 16
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    slabs, jobs = [], []
    with StripeQueue(enc, cell, 3, ChecksumType.CRC32C, 4096) as q:
        for s in range(7):
            sl = host_alloc((k + p) * n)
            slabs.append(sl)
            d = [sl.array[j * n:(j + 1) * n] for j in range(k)]
            for j, x in enumerate(cells(SEED, 93000 + 10 * s, k, n)):
                d[j][:] = x
            par = [sl.array[(k + r) * n:(k + r + 1) * n] for r in range(p)]
            crcs = np.zeros((k + p) * ((n + 4095) // 4096), np.uint32)
            jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs))
        q.wait(jobs[-1][0])
        for t, d, par, crcs in jobs:
            ref = oracle.rs_encode(k, p, [np.array(x) for x in d])
            assert all((a == b).all() for a, b in zip(par, ref)), t
            exp = np.concatenate([oracle.crc_windows(oracle.CRC32C, u, 4096) for u in [np.array(x) for x in d] + ref])
            assert (crcs == exp).all(), t


@pytest.mark.parametrize("batches", [2, 5])
def test_queue_ring_depth_and_ordered_h2d(batches):
    """Every H2D copy runs on one queue-wide stream and each batch's kernel waits on its event: parity stays
    bit-exact for any ring depth while the submitting thread keeps refilling the oldest batch."""
    from ozone_amd import _lib
    k, p, n = 6, 3, 1 << 15
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    assert _lib.lib().ozec_set_tuning(b"queue_batches", batches) == 0
    try:
        keep, jobs = [], []
        with StripeQueue(enc, n, 3, ChecksumType.CRC32C, 8192) as q:
            for s in range(3 * batches * 3 + 2):
                pinned = s % 2 == 0
                d = _stripe(93000 + 10 * s, k, n, pinned, keep)
                par = _parity(p, n, pinned, keep)
                crcs = np.zeros((k + p) * (n // 8192), np.uint32)
                jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs))
            q.wait(jobs[-1][0])
    finally:
        _lib.lib().ozec_set_tuning(b"queue_batches", 0)
    for t, d, par, crcs in jobs:
        ref = oracle.rs_encode(k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), t
        exp = np.concatenate([oracle.crc_windows(oracle.CRC32C, u, 8192) for u in list(d) + ref])
        assert (crcs == exp).all(), t


def test_queue_close_with_unlaunched_batch_drains():
    """Closing a queue whose current batch was submitted but never launched waits for its H2D copies."""
    k, p, n = 6, 3, 1 << 16
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    keep = []
    q = StripeQueue(enc, n, 8)
    for s in range(3):
        q.submit(_stripe(94000 + 10 * s, k, n, True, keep), _parity(p, n, True, keep))
    q.close()
    with StripeQueue(enc, n, 8) as q2:  # the device is still usable
        d = cells(SEED, 94100, k, n)
        par = [np.zeros(n, np.uint8) for _ in range(p)]
        q2.wait(q2.submit(d, par))
    assert all((a == b).all() for a, b in zip(par, oracle.rs_encode(k, p, d)))


@pytest.mark.parametrize("batches", [2, 3])
def test_queue_completes_oldest_on_wrap(batches):
    """When the ring wraps, submit() completes the OLDEST in-flight batch and refills it; every other batch stays
    in flight (the rotation used to skip the oldest batch and complete the next one)."""
    from ozone_amd import _lib
    k, p, n, S = 6, 3, 1 << 14, 2
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    assert _lib.lib().ozec_set_tuning(b"queue_batches", batches) == 0
    try:
        jobs = []
        with StripeQueue(enc, n, S) as q:
            for s in range(S * batches):  # fill every batch of the ring: all in flight
                d = cells(SEED, 95000 + 10 * s, k, n)
                par = [np.zeros(n, np.uint8) for _ in range(p)]
                jobs.append((q.submit(d, par), d, par))
            assert q.state() == (batches, 0, 0)
            for wrap in range(2 * batches):  # each wrap completes exactly the oldest batch
                s = S * batches + wrap * S
                d = cells(SEED, 95000 + 10 * s, k, n)
                par = [np.zeros(n, np.uint8) for _ in range(p)]
                jobs.append((q.submit(d, par), d, par))
                n_in, oldest, filling = q.state()
                assert (n_in, oldest, filling) == (batches - 1, S * (wrap + 1), 1), (wrap, q.state())
                # the completed batch's callers already hold their parity
                for t, dd, pp in jobs[S * wrap:S * (wrap + 1)]:
                    ref = oracle.rs_encode(k, p, dd)
                    assert all((a == b).all() for a, b in zip(pp, ref)), t
                for _ in range(S - 1):  # fill the rest of the refilled batch: it launches
                    s = len(jobs)
                    d = cells(SEED, 95000 + 10 * s, k, n)
                    par = [np.zeros(n, np.uint8) for _ in range(p)]
                    jobs.append((q.submit(d, par), d, par))
                assert q.state()[0] == batches
            q.wait(jobs[-1][0])
    finally:
        _lib.lib().ozec_set_tuning(b"queue_batches", 0)
    for t, d, par in jobs:
        assert all((a == b).all() for a, b in zip(par, oracle.rs_encode(k, p, d))), t


def test_queue_close_completes_pending_stripes():
    """Stripes submitted but never waited for get their parity and CRCs when the queue is closed (ozec.h)."""
    k, p, n, bpc = 6, 3, 1 << 15, 8192
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    keep, jobs = [], []
    q = StripeQueue(enc, n, 4, ChecksumType.CRC32C, bpc)
    for s in range(10):  # two launched batches + a filling one
        d = _stripe(96000 + 10 * s, k, n, s % 2 == 0, keep)
        par = _parity(p, n, s % 3 == 0, keep)
        crcs = np.zeros((k + p) * (n // bpc), np.uint32)
        jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs))
    q.close()
    for t, d, par, crcs in jobs:
        ref = oracle.rs_encode(k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), t
        exp = np.concatenate([oracle.crc_windows(oracle.CRC32C, u, bpc) for u in list(d) + ref])
        assert (crcs == exp).all(), t


def test_queue_rejects_buffers_it_cannot_dma():
    """crcs / data / parity are checked for dtype, contiguity and size before native code sees them."""
    k, p, n, bpc = 6, 3, 1 << 14, 4096
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    d = cells(SEED, 97000, k, n)
    par = [np.zeros(n, np.uint8) for _ in range(p)]
    with StripeQueue(enc, n, 2, ChecksumType.CRC32C, bpc) as q:
        with pytest.raises(rc.IllegalArgumentException):  # too few CRC slots
            q.submit(d, par, crcs=np.zeros((k + p) * (n // bpc) - 1, np.uint32))
        with pytest.raises(rc.IllegalArgumentException):  # wrong dtype
            q.submit(d, par, crcs=np.zeros((k + p) * (n // bpc), np.uint8))
        with pytest.raises(rc.IllegalArgumentException):  # strided data cell
            q.submit([np.zeros(2 * n, np.uint8)[::2]] + d[1:], par)
        with pytest.raises(rc.IllegalArgumentException):  # read-only parity
            ro = np.zeros(n, np.uint8)
            ro.flags.writeable = False
            q.submit(d, [ro] + par[1:])
        crcs = np.zeros((k + p) * (n // bpc), np.uint32)
        q.wait(q.submit(d, par, crcs=crcs))
    ref = oracle.rs_encode(k, p, d)
    assert all((a == b).all() for a, b in zip(par, ref))


def test_queue_outlives_its_encoder_handle():
    """The C ABI queue co-owns its encoder (ozec_coder_retain; ADVICE r2: the Java HipStripeQueue kept a raw handle
    that AbstractHipRawEncoder.release() freed): with the encoder released and freed by its creator, a submit fails
    with OZEC_ECLOSED and freeing the queue -- pending stripes included -- touches no freed memory."""
    import ctypes
    from ozone_amd import _lib as L
    lib = L.lib()
    k, p, n = 6, 3, 8192
    h = ctypes.c_void_p()
    assert lib.ozec_encoder_create(0, k, p, ctypes.byref(h)) == 0
    q = ctypes.c_void_p()
    assert lib.ozec_stripe_queue_create(h, n, 4, 3, 4096, 0, ctypes.byref(q)) == 0
    kk, pp, rows, ct = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    cl, bpc = ctypes.c_size_t(), ctypes.c_size_t()
    assert lib.ozec_stripe_queue_info(q, ctypes.byref(kk), ctypes.byref(pp), ctypes.byref(rows), ctypes.byref(cl),
                                      ctypes.byref(ct), ctypes.byref(bpc)) == 0
    assert (kk.value, pp.value, rows.value, cl.value, ct.value, bpc.value) == (k, p, p, n, 3, 4096)
    d = cells(SEED, 93000, k, n)
    par = [np.zeros(n, np.uint8) for _ in range(p)]
    crcs = np.zeros((k + p) * 2, np.uint32)
    dp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in d])
    pq = (ctypes.c_void_p * p)(*[x.ctypes.data for x in par])
    t = ctypes.c_uint64()
    assert lib.ozec_stripe_queue_submit(q, dp, pq, n, crcs.ctypes.data, ctypes.byref(t)) == 0  # pending in the queue
    assert lib.ozec_coder_release(h) == 0
    lib.ozec_coder_free(h)  # the creator's reference: the queue's keeps the memory
    assert lib.ozec_stripe_queue_submit(q, dp, pq, n, crcs.ctypes.data, ctypes.byref(t)) == L.OZEC_ECLOSED
    assert "closed" in L.last_error()
    rc_ = lib.ozec_stripe_queue_free(q)  # drains: the pending batch cannot launch on a closed coder
    assert rc_ in (0, L.OZEC_ECLOSED, L.OZEC_EDEVICE)
