"""Byte-granular cells on the fused encode + CRC path (round 5, fused_nb.hpp nb_tail) vs the oracle (GPU).

Every key's last stripe has cells of any length (parityCellSize = dataBuffers[0].position(),
ECKeyOutputStream.java:276), and a packed device batch of such stripes puts its units at odd byte offsets.  These
cells now run on the nibble kernel: the whole 16-B blocks in the window loop, the last 1-15 bytes of each unit in
nb_tail (bytewise CRC register update, GF products from the s_gf nibble products), with unaligned 16-B buffer
accesses for the blocks.  Checked bit-exact against oracle.rs_encode / oracle.crc_windows (Checksum.java:157-200,
RSRawEncoder), with guard bytes around the batch that must stay untouched.
"""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
from devcopy import to_dev, to_host  # noqa: E402
pytestmark = pytest.mark.gpu

from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

DEV = "cuda:0"
PRODUCTION_ROUTING = os.environ.get("OZEC_TEST_PRODUCTION_ROUTING") == "1"
GUARD = 64


def _otype(ctype):
    return oracle.CRC32 if ctype == ck.ChecksumType.CRC32 else oracle.CRC32C


def _packed_case(k, p, n, S, bpc, ctype, shift, seed):
    """S stripes of k + p units of n bytes back to back (unit stride n, stripe stride (k + p) n) starting `shift`
    bytes into a device buffer with GUARD bytes of 0xA5 on both sides; parity written in place."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    flat = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    body = flat[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    body[:, :k] = data
    d = to_dev(flat)
    base = d[GUARD + shift:]
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p)).encode_crc_batch(
        base, (k + p) * n, n, base[k * n:], (k + p) * n, n, S, n, ctype, bpc, crcs)
    torch.cuda.synchronize()
    got = to_host(d)
    c = to_host(crcs).view(np.uint32)
    assert (got[:GUARD + shift] == 0xA5).all() and (got[GUARD + shift + S * (k + p) * n:] == 0xA5).all()
    units = got[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    ot = _otype(ctype)
    for s in range(S):
        ref = oracle.rs_encode(k, p, list(data[s]))
        for q in range(p):
            assert (units[s, k + q] == ref[q]).all(), (k, p, n, s, q)
        for u, cell in enumerate(list(data[s]) + ref):
            assert (c[s, u] == oracle.crc_windows(ot, cell, bpc)).all(), (k, p, n, bpc, s, u)


@pytest.mark.parametrize("k,p", [(6, 3), (10, 4), (3, 2), (6, 1), (10, 2), (3, 1)])
@pytest.mark.parametrize("n", [1, 5, 15, 17, 1007, 2 * 4096 + 5, 16384 + 3, 50001, 3 * 16384 + 15])
def test_encode_crc_packed_odd_cells(k, p, n):
    """Cells of 1 B up to several windows + 15 B, packed at odd strides, CRC32C per 16 KiB (4 KiB for the short)."""
    bpc = 4096 if n < 16384 else 16384
    _packed_case(k, p, n, 5, bpc, ck.ChecksumType.CRC32C, 0, [k, p, n])


@pytest.mark.parametrize("ctype", [ck.ChecksumType.CRC32, ck.ChecksumType.CRC32C])
@pytest.mark.parametrize("shift", [1, 3, 8])
def test_encode_crc_unaligned_base(ctype, shift):
    """A batch whose base pointer is 1 / 3 / 8 bytes past 16-B alignment, cells a multiple of 16 B (every unit
    offset unaligned, no byte tail) and not (both)."""
    for n in (65536, 65536 + 9):
        _packed_case(6, 3, n, 4, 16384, ctype, shift, [shift, n])


@pytest.mark.parametrize("variant", [0, 170, 171, 172, 173, 174, 177, 62, 87, 49, 56])
def test_encode_crc_odd_cells_any_variant(variant):
    """Byte-granular cells run on the TAIL instantiations of the nibble kernel (fused_nb.hpp launch_nb_tail_kr:
    170-174, 177 as pinned); any other pinned variant (62 / 87 nibble, 49 per-window, 56 streamed-input) falls back to
    the default one."""
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", variant) == 0
    try:
        _packed_case(10, 4, 2 * 16384 + 4099, 3, 16384, ck.ChecksumType.CRC32C, 0, [variant])
        _packed_case(6, 3, 16384 + 1, 3, 16384, ck.ChecksumType.CRC32C, 5, [variant, 1])
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)


def test_encode_crc_odd_cells_c5_shape():
    """rs-6-3 cells of 700,001 B (the odd-tail row of bench.py --workload tail) packed, 24 stripes: every stripe
    against the oracle."""
    _packed_case(6, 3, 700_001, 24, 16384, ck.ChecksumType.CRC32C, 0, [700_001])


@pytest.mark.parametrize("k,p,n", [(6, 3, 1 << 20), (10, 4, 700_001), (3, 2, 1007)])
def test_fused_min_units_routes_small_batches_unfused(k, p, n):
    """Batches of 16-B cells below fused_min_units (stripe x window units) take the unfused kernels, byte-granular
    ones stay fused: same bytes and CRCs either way."""
    import ctypes
    lib = L.lib()
    prev = ctypes.c_int64()
    assert lib.ozec_get_tuning(b"fused_min_units", ctypes.byref(prev)) == 0
    try:
        for m in (0, 1024, 1 << 40):  # fused everywhere, libozec's default routing, unfused everywhere
            assert lib.ozec_set_tuning(b"fused_min_units", m) == 0
            _packed_case(k, p, n, 2, 16384, ck.ChecksumType.CRC32C, 0, [k, n])
    finally:
        lib.ozec_set_tuning(b"fused_min_units", prev.value)


@pytest.mark.parametrize("k,p,n", [(6, 3, 700_001), (10, 4, 16384 + 3), (3, 2, 1007), (6, 2, 50_001)])
def test_packed_odd_cells_coding_and_checksum_entry_points(k, p, n):
    """The coding-only and checksum-only device entry points on the same packed odd-offset stripes (ozec_encode_batch:
    gf_code_vec through buffer descriptors at any byte offset; ozec_checksum_windows_batch: crc_windows_g26 with
    align-1 loads), vs the oracle, guard bytes untouched."""
    S, bpc = 3, 16384
    rng = np.random.default_rng([k, p, n, 7])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    shift = 5
    flat = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    body = flat[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    body[:, :k] = data
    d = to_dev(flat)
    base = d[GUARD + shift:]
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p)).encode_batch(base, (k + p) * n, n, base[k * n:], (k + p) * n,
                                                                     n, S, n)
    nwin = -(-n // bpc)
    crcs = torch.zeros((S * (k + p), nwin), dtype=torch.int32, device=DEV)
    ck.checksum_windows_batch(ck.ChecksumType.CRC32C, base, n, S * (k + p), n, bpc, crcs)
    torch.cuda.synchronize()
    got = to_host(d)
    c = to_host(crcs).view(np.uint32).reshape(S, k + p, nwin)
    assert (got[:GUARD + shift] == 0xA5).all() and (got[GUARD + shift + S * (k + p) * n:] == 0xA5).all()
    units = got[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    for s in range(S):
        ref = oracle.rs_encode(k, p, list(data[s]))
        for q in range(p):
            assert (units[s, k + q] == ref[q]).all(), (k, p, n, s, q)
        for u, cell in enumerate(list(data[s]) + ref):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, cell, bpc)).all(), (k, p, n, s, u)


@pytest.mark.parametrize("codec,k,p", [("xor", 2, 1), ("xor", 3, 1), ("xor", 5, 1), ("rs", 4, 2), ("rs", 5, 6)])
@pytest.mark.parametrize("n", [16, 1007, 16384 + 3, 700_001])
def test_packed_odd_cells_xor_and_generic_shapes(codec, k, p, n):
    """The shapes without a gf_code_vec instantiation -- XOR-k-1 (xor_vec) and RS schemas outside 3/6/10 data units
    (gf_code_vec_generic; rs-5-6 in two row groups) -- on packed stripes at odd byte offsets run the BUF (raw buffer)
    instantiations: encode + CRC32C and a decode of the last data unit, vs oracle.xor_* / rs_* and crc_windows,
    guard bytes untouched."""
    S, bpc, shift = 3, 16384, 3
    rng = np.random.default_rng([k, p, n, 11])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    flat = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    flat[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)[:, :k] = data
    d = to_dev(flat)
    base = d[GUARD + shift:]
    conf = rc.ECReplicationConfig(k, p, codec)
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    rc.RawErasureEncoder(conf).encode_crc_batch(base, (k + p) * n, n, base[k * n:], (k + p) * n, n, S, n,
                                                ck.ChecksumType.CRC32C, bpc, crcs)
    erased = [k - 1]
    out = torch.zeros((S, 1, n), dtype=torch.uint8, device=DEV)
    rc.RawErasureDecoder(conf).decode_batch(base, (k + p) * n, n, [u for u in range(k + p) if u != k - 1][:k], erased,
                                            out, n, n, S, n)
    torch.cuda.synchronize()
    got = to_host(d)
    c = to_host(crcs).view(np.uint32)
    o = to_host(out)
    assert (got[:GUARD + shift] == 0xA5).all() and (got[GUARD + shift + S * (k + p) * n:] == 0xA5).all()
    units = got[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    for s in range(S):
        ref = [oracle.xor_encode(list(data[s]))] if codec == "xor" else oracle.rs_encode(k, p, list(data[s]))
        for q in range(p):
            assert (units[s, k + q] == ref[q]).all(), (codec, k, p, n, s, q)
        for u, cell in enumerate(list(data[s]) + list(ref)):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, cell, bpc)).all(), (codec, k, p, n, s, u)
        assert (o[s, 0] == data[s, k - 1]).all(), (codec, k, p, n, s)


def _routes():
    import ctypes
    f, u = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.lib().ozec_fused_routes(ctypes.byref(f), ctypes.byref(u)) == 0
    return f.value, u.value


@pytest.mark.parametrize("k", [2, 3, 6, 10])
@pytest.mark.parametrize("n", [1, 15, 1007, 16384 + 3, 50001, 3 * 16384 + 15])
@pytest.mark.parametrize("shift", [0, 3])
def test_xor_fused_any_length_and_offset(k, n, shift):
    """the XOR codec's fused kernel (encode_crc_g26 TAIL) takes cells of any length at any byte
    offset -- packed stripes of xor-k-1 (unit stride n) -- in ONE launch for encode + CRC32C and for the fused
    reconstruction (verify + decode + CRC), where round 5 ran coding and CRC as two kernels.  Parity, window CRCs,
    the rebuilt unit, its CRCs and the first failing (unit, window) of a planted corruption vs the oracle
    (XORRawEncoder.java:39-85, XORRawDecoder.java:45-61, Checksum.java:157-200); guard bytes untouched; both calls
    counted on the fused route."""
    p, S, bpc = 1, 3, 16384
    rng = np.random.default_rng([k, n, shift, 13])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    flat = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    flat[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)[:, :k] = data
    d = to_dev(flat)
    base = d[GUARD + shift:]
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    conf = rc.ECReplicationConfig(k, p, "xor")
    f0, u0 = _routes()
    rc.RawErasureEncoder(conf).encode_crc_batch(base, (k + p) * n, n, base[k * n:], (k + p) * n, n, S, n,
                                                ck.ChecksumType.CRC32C, bpc, crcs)
    f1, u1 = _routes()
    assert PRODUCTION_ROUTING or (f1 - f0, u1 - u0) == (1, 0), "the encode did not take the fused kernel"
    got, c = to_host(d), to_host(crcs).view(np.uint32)
    assert (got[:GUARD + shift] == 0xA5).all() and (got[GUARD + shift + S * (k + p) * n:] == 0xA5).all()
    units = got[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n).copy()
    for s in range(S):
        ref = oracle.xor_encode(list(data[s]))
        assert (units[s, k] == ref).all(), (k, n, shift, s)
        for u in range(k + 1):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, units[s, u], bpc)).all(), (k, n, shift, s, u)
    # reconstruction of data unit 1 from the other k units, stored CRCs checked; stripe 1 has one corrupted byte in
    # the last unit read
    erased = [1]
    present = [u for u in range(k + 1) if u not in erased]
    stored = c.copy()
    bad = units.copy()
    bad[:, 1] = 0xEE
    pos = n // 2
    bad[1, present[-1], pos] ^= 0x10
    flat2 = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    flat2[GUARD + shift:GUARD + shift + S * (k + p) * n] = bad.reshape(-1)
    d2 = to_dev(flat2)
    out = torch.zeros((S, 1, n + 5), dtype=torch.uint8, device=DEV)
    ocrc = torch.zeros((S, 1, nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    ob = out.view(-1)[shift:]  # outputs at odd offsets too
    f0, u0 = _routes()
    rc.RawErasureDecoder(conf).reconstruct_crc_batch(
        d2[GUARD + shift:], (k + p) * n, n, present, erased, ob, n + 5, n, S, n, ck.ChecksumType.CRC32C, bpc, ocrc,
        d_expected=to_dev(stored.view(np.int32)), d_mismatch=mism)
    f1, u1 = _routes()
    assert PRODUCTION_ROUTING or (f1 - f0, u1 - u0) == (1, 0), "the reconstruction did not take the fused kernel"
    o = to_host(out).reshape(-1)[shift:shift + S * (n + 5)]
    oc, m = to_host(ocrc).view(np.uint32), to_host(mism)
    for s in range(S):
        rebuilt = o[s * (n + 5):s * (n + 5) + n]
        if s != 1:
            assert (rebuilt == data[s, 1]).all(), (k, n, shift, s)
            assert m[s] == -1
        assert (oc[s, 0] == oracle.crc_windows(oracle.CRC32C, rebuilt, bpc)).all(), (k, n, shift, s)
    assert m[1] == present[-1] * nwin + pos // bpc


@pytest.mark.parametrize("k,n", [(6, (1 << 20) + 5), (2, 700_001)])
def test_xor_fused_tail_at_bench_cell_size(k, n):
    """The XOR TAIL fused form at the A/B's cell sizes (profiles/r06/fused_ab/): 48 packed stripes of xor-k-1 whose
    cells are not a multiple of 16 B (every unit at an odd offset), at an odd base: one fused launch (past the
    small-batch threshold under libozec's own routing too), parity and every unit's CRC32C windows vs the oracle."""
    p, S, bpc, shift = 1, 48, 16384, 3
    rng = np.random.default_rng([k, n, 48])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    flat = np.full(GUARD + shift + S * (k + p) * n + GUARD, 0xA5, np.uint8)
    flat[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)[:, :k] = data
    d = to_dev(flat)
    base = d[GUARD + shift:]
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    f0, u0 = _routes()
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, "xor")).encode_crc_batch(
        base, (k + p) * n, n, base[k * n:], (k + p) * n, n, S, n, ck.ChecksumType.CRC32C, bpc, crcs)
    f1, u1 = _routes()
    assert (f1 - f0, u1 - u0) == (1, 0), "the encode did not take the fused kernel"
    got, c = to_host(d), to_host(crcs).view(np.uint32)
    assert (got[:GUARD + shift] == 0xA5).all() and (got[GUARD + shift + S * (k + p) * n:] == 0xA5).all()
    units = got[GUARD + shift:GUARD + shift + S * (k + p) * n].reshape(S, k + p, n)
    for s in range(S):
        ref = oracle.xor_encode(list(data[s]))
        assert (units[s, k] == ref).all(), (k, n, s)
        for u in range(k + 1):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, units[s, u], bpc)).all(), (k, n, s, u)
