"""Seeded random sweep of the HIP path against the oracle, bit-exact (GPU).

The fixed-shape tests pin the configurations BASELINE names and the reference's own test shapes; this sweep draws
shapes, lengths, alignments, erasure patterns, CRC types and window sizes at random (recorded seed per case) so the
dispatch between kernels -- fused vs unfused, full vs short last windows, aligned vs misaligned cells, nibble vs
per-window vs XOR kernels, first-k-valid decode -- is crossed in combinations no hand-written case lists.
Reference semantics followed: RSRawEncoder / RSRawDecoder (EC/rawcoder/RSRawDecoder.java:79-176, first k valid
inputs), XORRawEncoder / XORRawDecoder (XORRawEncoder.java:39-85), Checksum.computeChecksum window split
(CM/Checksum.java:157-200, short last window), ECReconstructionCoordinator's verify + decode + re-checksum.
"""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
from devcopy import to_dev, to_host  # noqa: E402
pytestmark = pytest.mark.gpu

from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

DEV = "cuda:0"
N_CASES = int(os.environ.get("OZEC_RANDOM_CASES", "48"))  # draws per entry family (a wider sweep: e.g. 480)


def _rng(tag, i):
    return np.random.default_rng([0x5EED, tag, i])


def _codec(r):
    """(codec, k, p): RS over the reference's schemas and odd ones, XOR with 1-3 parity slots."""
    if r.random() < 0.2:
        return "xor", int(r.integers(1, 9)), int(r.integers(1, 4))
    k = int(r.choice([1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16]))
    p = int(r.choice([1, 2, 3, 4])) if k < 16 else int(r.choice([2, 4]))
    return "rs", k, p


def _parity(codec, k, p, data):
    return oracle.rs_encode(k, p, data) if codec == "rs" else [oracle.xor_encode(data)] + \
        [np.zeros(len(data[0]), np.uint8) for _ in range(p - 1)]


def _erasure(r, codec, k, p):
    """(erased indexes in the reference's order, inputs present)."""
    if codec == "xor":  # XORRawDecoder XORs every other slot (XORRawDecoder.java:40-86): all of them present
        e = int(r.integers(0, k + p))
        return [e], [u for u in range(k + p) if u != e]
    ne = int(r.integers(1, p + 1))
    erased = sorted(int(x) for x in r.choice(k + p, size=ne, replace=False))
    present = [u for u in range(k + p) if u not in erased]
    return erased, present


def _cells(r, k, n):
    return [r.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_host_encode_decode(i):
    """Host-buffer entry points (the JNI drop-in's per-call path): cells at random offsets inside larger buffers,
    outputs pre-filled with garbage, decode from the reference's input-slot convention."""
    r = _rng(1, i)
    codec, k, p = _codec(r)
    n = int(r.integers(1, 300_000))
    data = _cells(r, k, n)
    pad = int(r.integers(0, 64))
    bufs = [np.zeros(n + 2 * pad + 1, np.uint8) for _ in range(k)]
    ins = [b[pad:pad + n] for b in bufs]
    for a, d in zip(ins, data):
        a[:] = d
    outs = [np.full(n, 0xA5, np.uint8) for _ in range(p)]
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec)).encode(ins, outs)
    ref = _parity(codec, k, p, data)
    assert all((o == x).all() for o, x in zip(outs, ref)), (codec, k, p, n)
    units = data + ref  # XOR p > 1: the extra parity slots hold the zeros the encoder wrote
    erased, present = _erasure(r, codec, k, p)
    slots = [units[u] if u in present else None for u in range(k + p)]
    got = [np.full(n, 0x5A, np.uint8) for _ in erased]
    rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec)).decode(slots, erased, got)
    assert all((g == units[e]).all() for g, e in zip(got, erased)), (codec, k, p, n, erased)


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_device_encode_decode(i):
    """Device-pointer entry points at random 0-15-byte misalignments, against the oracle."""
    r = _rng(2, i)
    codec, k, p = _codec(r)
    n = int(r.integers(1, 200_000))
    data = _cells(r, k, n)
    off = [int(x) for x in r.integers(0, 16, k + p + 8)]
    raw = [torch.zeros(n + 32, dtype=torch.uint8, device=DEV) for _ in range(k)]
    for j in range(k):
        raw[j][off[j]:off[j] + n] = to_dev(data[j])
    out = [torch.full((n + 32,), 0xA5, dtype=torch.uint8, device=DEV) for _ in range(p)]
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec)).encode_device(
        [raw[j][off[j]:] for j in range(k)], [out[q][off[k + q]:] for q in range(p)], n)
    torch.cuda.synchronize()
    ref = _parity(codec, k, p, data)
    for q in range(p if codec == "rs" else 1):
        o = to_host(out[q])
        assert (o[off[k + q]:off[k + q] + n] == ref[q]).all(), (codec, k, p, n, q)
        assert (o[:off[k + q]] == 0xA5).all() and (o[off[k + q] + n:] == 0xA5).all()  # nothing outside the cell
    units = data + ref
    erased, present = _erasure(r, codec, k, p)
    d_in = [to_dev(units[u]) if u in present else None for u in range(k + p)]
    d_out = [torch.zeros(n, dtype=torch.uint8, device=DEV) for _ in erased]
    rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec)).decode_device(d_in, erased, d_out, n)
    torch.cuda.synchronize()
    assert all((to_host(x) == units[e]).all() for x, e in zip(d_out, erased)), (codec, k, p, n, erased)


FUSED = [("rs", 6, 3), ("rs", 6, 2), ("rs", 6, 1), ("rs", 3, 2), ("rs", 3, 1), ("rs", 10, 4), ("rs", 10, 3),
         ("rs", 10, 2), ("rs", 10, 1), ("xor", 2, 1), ("xor", 3, 1), ("rs", 5, 2), ("rs", 4, 4)]


def _fused_case(r):
    codec, k, p = FUSED[int(r.integers(0, len(FUSED)))]
    bpc = int(r.choice([512, 1000, 4096, 8192, 16384, 65536]))
    n = int(r.choice([bpc * int(r.integers(1, 5)), int(r.integers(1, 4 * bpc))]))  # full or short last windows
    S = int(r.integers(1, 7))
    ctype = (ck.ChecksumType.CRC32, ck.ChecksumType.CRC32C)[int(r.integers(0, 2))]
    return codec, k, p, bpc, n, S, ctype


def _otype(ctype):
    return oracle.CRC32 if ctype == ck.ChecksumType.CRC32 else oracle.CRC32C


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_fused_encode_crc(i):
    """encode + window CRCs of every unit in one call, stripe-major batch, vs oracle parity and CRCs."""
    r = _rng(3, i)
    codec, k, p, bpc, n, S, ctype = _fused_case(r)
    rows = p if codec == "rs" else 1
    data = np.stack([np.stack(_cells(r, k, n)) for _ in range(S)])              # [S][k][n]
    units = torch.full((S, k + p, n), 0xA5, dtype=torch.uint8, device=DEV)
    units[:, :k] = to_dev(data)
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + rows, nwin), dtype=torch.int32, device=DEV)
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec)).encode_crc_batch(
        units, (k + p) * n, n, units[:, k:], (k + p) * n, n, S, n, ctype, bpc, crcs)
    torch.cuda.synchronize()
    got, c = to_host(units), to_host(crcs).view(np.uint32)
    for s in range(S):
        ref = _parity(codec, k, p, list(data[s]))
        for q in range(p):
            assert (got[s, k + q] == ref[q]).all(), (codec, k, p, n, bpc, s, q)
        for u, cell in enumerate(list(data[s]) + ref[:rows]):
            assert (c[s, u] == oracle.crc_windows(_otype(ctype), cell, bpc)).all(), (codec, k, p, n, bpc, s, u)


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_fused_reconstruction(i):
    """Verify stored CRCs of the units read + decode + CRC of the rebuilt units, with a silent corruption planted
    in a random stripe: that stripe reports the first failing (unit, window), the others rebuild exactly."""
    r = _rng(4, i)
    codec, k, p, bpc, n, S, ctype = _fused_case(r)
    S = max(S, 2)
    data = [list(_cells(r, k, n)) for _ in range(S)]
    units = np.stack([np.stack(d + _parity(codec, k, p, d)) for d in data])      # [S][k+p][n]
    nwin = -(-n // bpc)
    ot = _otype(ctype)
    stored = np.stack([np.stack([oracle.crc_windows(ot, units[s, u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)
    erased, present = _erasure(r, codec, k, p)
    read = present[:k]
    bad_s, bad_u = int(r.integers(0, S)), int(r.choice(read))
    bad_w = int(r.integers(0, nwin))
    pos = min(n - 1, bad_w * bpc + int(r.integers(0, bpc)))
    corrupted = units.copy()
    corrupted[:, erased] = 0xEE
    corrupted[bad_s, bad_u, pos] ^= 0x41
    d_out = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    d_crc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec))
    dec.reconstruct_crc_batch(to_dev(corrupted), (k + p) * n, n, present, erased, d_out,
                              len(erased) * n, n, S, n, ctype, bpc, d_crc,
                              d_expected=to_dev(stored.view(np.int32)), d_mismatch=mism)
    torch.cuda.synchronize()
    out, crcs, m = to_host(d_out), to_host(d_crc).view(np.uint32), to_host(mism)
    for s in range(S):
        if s == bad_s:
            assert m[s] == bad_u * nwin + pos // bpc, (codec, k, p, n, bpc, erased, bad_u, pos)
            for q in range(len(erased)):  # rebuilt CRCs describe what was written
                assert (crcs[s, q] == oracle.crc_windows(ot, out[s, q], bpc)).all()
            continue
        assert m[s] == -1, (codec, k, p, n, bpc, s)
        for q, e in enumerate(erased):
            assert (out[s, q] == units[s, e]).all(), (codec, k, p, n, bpc, s, e)
            assert (crcs[s, q] == stored[s, e]).all(), (codec, k, p, n, bpc, s, e)


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_checksum_windows(i):
    """Checksum.computeChecksum over random lengths, window sizes and offsets, host and device, both CRC types."""
    r = _rng(5, i)
    bpc = int(r.choice([1, 7, 16, 512, 1000, 4096, 16384, 65536, 1 << 20]))
    n = int(r.integers(1, 400_000 if bpc >= 16 else 20_000))
    ctype = (ck.ChecksumType.CRC32, ck.ChecksumType.CRC32C)[int(r.integers(0, 2))]
    off = int(r.integers(0, 32))
    buf = r.integers(0, 256, n + off, dtype=np.uint8)
    want = [int(x) for x in oracle.crc_windows(_otype(ctype), buf[off:], bpc)]
    cd = ck.Checksum(ctype, bpc).compute_checksum(buf[off:])
    assert [int.from_bytes(b, "big") for b in cd.get_checksums()] == want, (n, bpc, off)


@pytest.fixture
def device_list():
    """ozec_set_devices for one test, the default list restored afterwards."""
    yield rc.set_devices
    rc.set_devices(None)


@pytest.mark.parametrize("i", range(N_CASES // 2))
def test_random_host_batches(device_list, i):
    """C5's host-batch entry points (ozec_encode_crc_host_batch / ozec_reconstruct_crc_host_batch) over random
    shapes, batch sizes, pipeline chunks, unit gaps, pinned or pageable batches and device lists ([0, 0, 0] stands
    for three GPUs on the one-GPU box: the batch is cut into that many stripe ranges, each on its own pipeline)."""
    from ozone_amd.stripe_queue import host_alloc
    r = _rng(6, i)
    codec, k, p, bpc, n, S, ctype = _fused_case(r)
    S = int(r.integers(1, 40))
    chunk = int(r.integers(0, 9))
    gap = int(r.choice([0, 0, 16, 4096]))
    devs = [0] * int(r.integers(1, 4))
    pinned = bool(r.integers(0, 2))
    device_list(devs)
    rows = p if codec == "rs" else 1
    us = n + gap
    nwin = -(-n // bpc)
    data = [_cells(r, k, n) for _ in range(S)]
    units = [d + _parity(codec, k, p, d) for d in data]
    keep = []

    def host(nbytes, dtype=np.uint8):
        if not pinned:
            return np.zeros(nbytes // np.dtype(dtype).itemsize, dtype)
        b = host_alloc(nbytes)
        keep.append(b)
        return b.array.view(dtype)

    buf = host(S * (k + p) * us)
    v = buf.reshape(S, k + p, us)
    v[:] = 0xA5
    for s in range(S):
        for j in range(k):
            v[s, j, :n] = data[s][j]
    crcs = host(S * (k + rows) * nwin * 4, np.uint32)
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec))
    enc.encode_crc_host_batch(buf.ctypes.data, (k + p) * us, us, buf.ctypes.data + k * us, (k + p) * us, us, S, n,
                              ctype, bpc, crcs, False, chunk)
    ot = _otype(ctype)
    c = crcs.reshape(S, k + rows, nwin)
    for s in range(S):
        for q in range(p):
            assert (v[s, k + q, :n] == units[s][k + q]).all(), (codec, k, p, n, S, chunk, devs, s, q)
        for u in range(k + rows):
            assert (c[s, u] == oracle.crc_windows(ot, units[s][u], bpc)).all(), (codec, k, p, n, S, s, u)
    # the same stripes rebuilt from host memory, one planted corruption
    erased, present = _erasure(r, codec, k, p)
    for s in range(S):
        for q in range(p):
            v[s, k + q, :n] = units[s][k + q]
    stored = np.stack([np.stack([oracle.crc_windows(ot, units[s][u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)
    bad_s, bad_u = int(r.integers(0, S)), int(present[int(r.integers(0, k))])
    pos = int(r.integers(0, n))
    v[bad_s, bad_u, pos] ^= 0x08
    e = len(erased)
    out = host(S * e * n)
    ocrc = host(S * e * nwin * 4, np.uint32)
    mism = np.zeros(S, np.int32)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec))
    dec.reconstruct_crc_host_batch(buf, (k + p) * us, us, present, erased, out, e * n, n, S, n, ctype, bpc, ocrc,
                                   h_expected=stored.reshape(-1), h_mismatch=mism, stripes_per_chunk=chunk)
    got, oc = out.reshape(S, e, n), ocrc.reshape(S, e, nwin)
    for s in range(S):
        if s == bad_s:
            assert mism[s] == bad_u * nwin + pos // bpc, (codec, k, p, n, S, erased, bad_u, pos)
            continue
        assert mism[s] == -1, (codec, k, p, n, S, chunk, devs, s)
        for q, u in enumerate(erased):
            assert (got[s, q] == units[s][u]).all() and (oc[s, q] == stored[s, u]).all(), (codec, k, p, s, u)


@pytest.mark.parametrize("i", range(N_CASES // 2))
def test_random_stripe_queue(i):
    """The writer-side stripe queue (ozec_stripe_queue_*): random codec, cell length, batch size,
    stripe lengths up to the cell, CRC type (or none) and wait pattern; every stripe's parity and CRCs vs the oracle."""
    from ozone_amd.stripe_queue import StripeQueue
    r = _rng(7, i)
    codec, k, p = _codec(r)
    cell = int(r.choice([4096, 65536, 200_000, 1 << 20]))
    batch = int(r.integers(1, 9))
    with_crc = bool(r.integers(0, 2))
    ctype = (ck.ChecksumType.CRC32, ck.ChecksumType.CRC32C)[int(r.integers(0, 2))] if with_crc \
        else ck.ChecksumType.NONE
    bpc = int(r.choice([512, 4096, 16384]))
    rows = p if codec == "rs" else 1
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec))
    jobs = []
    with StripeQueue(enc, cell, batch, ctype, bpc) as q:
        for s in range(int(r.integers(1, 3 * batch + 3))):
            n = int(r.choice([cell, int(r.integers(1, cell + 1))]))
            d = _cells(r, k, n)
            par = [np.full(n, 0xA5, np.uint8) for _ in range(p)]
            crcs = np.zeros((k + rows) * -(-n // bpc), np.uint32) if with_crc else None
            jobs.append((q.submit(d, par, crcs=crcs), d, par, crcs, n))
            if r.random() < 0.2:
                q.wait(jobs[int(r.integers(0, len(jobs)))][0])
        q.wait(jobs[-1][0])
    for t, d, par, crcs, n in jobs:
        ref = _parity(codec, k, p, d)
        assert all((a == b).all() for a, b in zip(par, ref)), (codec, k, p, cell, batch, t, n)
        if with_crc:
            got = crcs.reshape(k + rows, -1)
            for u, x in enumerate(d + ref[:rows]):
                assert (got[u] == oracle.crc_windows(_otype(ctype), x, bpc)).all(), (codec, k, p, t, n, u)


@pytest.mark.parametrize("i", range(N_CASES // 2))
def test_random_host_zero_copy_and_callbacks(i):
    """Round 6's host paths under random knobs: zero copy on / off / at a tiny grid (host_zero_copy), 1-3 column chunks
    (host_zc_chunks), cells pinned in one pool at a stride (the JNI arena's layout) or pageable, and the
    caller-moves-the-bytes entry points (ozec_encode_cb / ozec_decode_cb, the JNI heap-array form) -- encode and a
    decode of the drawn erasure pattern vs the oracle."""
    import ctypes
    from ozone_amd import _lib as L
    from ozone_amd.stripe_queue import host_alloc
    lib = L.lib()
    r = _rng(9, i)
    codec, k, p = _codec(r)
    n = int(r.integers(1, 2_600_000))
    zc, zch = int(r.choice([0, 5, 48])), int(r.integers(1, 4))
    pinned = bool(r.random() < 0.5)
    data = _cells(r, k, n)
    ref = _parity(codec, k, p, data)
    units = data + ref
    erased, present = _erasure(r, codec, k, p)
    assert lib.ozec_set_tuning(b"host_zero_copy", zc) == 0 and lib.ozec_set_tuning(b"host_zc_chunks", zch) == 0
    pool = None
    try:
        # the ozone_amd API, pinned or pageable cells
        if pinned:
            pool = host_alloc((k + p + len(erased)) * n + 64)
            cell = [pool.array[u * n:(u + 1) * n] for u in range(k + p + len(erased))]
            ins, outs = cell[:k], cell[k:k + p]
            for a, d in zip(ins, data):
                a[:] = d
            for o in outs:
                o[:] = 0xA5
        else:
            ins, outs = [d.copy() for d in data], [np.full(n, 0xA5, np.uint8) for _ in range(p)]
        rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec)).encode(ins, outs)
        assert all((o == x).all() for o, x in zip(outs, ref)), (codec, k, p, n, zc, zch, pinned)
        slots = [(cell[u] if pinned else units[u].copy()) if u in present else None for u in range(k + p)]
        if pinned:
            for u in range(k, k + p):
                cell[u][:] = units[u]
        got = cell[k + p:] if pinned else [np.zeros(n, np.uint8) for _ in erased]
        for g in got:
            g[:] = 0x5A
        rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec)).decode(slots, erased, got)
        assert all((g == units[e]).all() for g, e in zip(got, erased)), (codec, k, p, n, erased, zc, zch, pinned)
        if pinned:
            del cell, ins, outs, slots, got
        # the callback entry points
        errors = []

        def fill_from(src_units):
            def fill(user, off, ln, dst):
                try:
                    for j, x in enumerate(src_units):
                        if dst[j]:
                            ctypes.memmove(dst[j], x[off:off + ln].ctypes.data, ln)
                    return 0
                except Exception as e:  # noqa: BLE001
                    errors.append(e)
                    return -99
            return L.FILL_FN(fill)

        def drain_to(dst_units):
            def drain(user, off, ln, src):
                try:
                    for q, o in enumerate(dst_units):
                        ctypes.memmove(o[off:off + ln].ctypes.data, src[q], ln)
                    return 0
                except Exception as e:  # noqa: BLE001
                    errors.append(e)
                    return -99
            return L.DRAIN_FN(drain)

        cid = L.OZEC_CODEC_RS if codec == "rs" else L.OZEC_CODEC_XOR
        he, hd = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.ozec_encoder_create(cid, k, p, ctypes.byref(he)) == 0
        assert lib.ozec_decoder_create(cid, k, p, ctypes.byref(hd)) == 0
        try:
            cb_out = [np.full(n, 0xA5, np.uint8) for _ in range(p)]
            f, d = fill_from(data), drain_to(cb_out)
            assert lib.ozec_encode_cb(he, n, f, d, None) == 0, (L.last_error(), errors)
            assert not errors and all((o == x).all() for o, x in zip(cb_out, ref)), (codec, k, p, n, zc, zch)
            cb_got = [np.zeros(n, np.uint8) for _ in erased]
            have = [units[u] if u in present else None for u in range(k + p)]
            f, d = fill_from(have), drain_to(cb_got)
            pres = (ctypes.c_uint8 * (k + p))(*[u in present for u in range(k + p)])
            er = (ctypes.c_int * len(erased))(*erased)
            assert lib.ozec_decode_cb(hd, pres, er, len(erased), n, f, d, None) == 0, (L.last_error(), errors)
            assert not errors and all((g == units[e]).all() for g, e in zip(cb_got, erased)), \
                (codec, k, p, n, erased, zc, zch)
        finally:
            for h in (he, hd):
                lib.ozec_coder_release(h)
                lib.ozec_coder_free(h)
    finally:
        lib.ozec_set_tuning(b"host_zero_copy", 48)
        lib.ozec_set_tuning(b"host_zc_chunks", 2)
        if pool is not None:
            pool.free()
