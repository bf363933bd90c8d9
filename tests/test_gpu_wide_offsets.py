"""Batches whose unit offsets span more than 2 GiB (GPU).

The vector kernels address a stripe through 32-bit buffer offsets after rebase32 (device.hpp); a layout whose units
lie further apart -- a caller's stripes scattered over a large HBM pool, unit stride 768 MiB here -- must take the
64-bit paths (one buffer descriptor per unit: gf_code_vec WIDE, and since round 6 the fused kernels' WIDE forms, in
ONE launch for the fused shapes; typed-pointer / byte kernels for the other schemas) and still produce the oracle's
parity, decoded units and CRCs (RSUtil.encodeData, XORRawEncoder, Checksum.computeChecksum) and a clean verified
reconstruction (ChecksumData.java:118-150), aligned and at odd byte offsets, with the bytes after the units untouched.
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
PRODUCTION_ROUTING = os.environ.get("OZEC_TEST_PRODUCTION_ROUTING") == "1"
US = 768 << 20  # unit stride: 768 MiB


def _routes():
    import ctypes
    from ozone_amd import _lib as L
    f, u = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.lib().ozec_fused_routes(ctypes.byref(f), ctypes.byref(u)) == 0
    return f.value, u.value


@pytest.mark.parametrize("codec,k,p", [("rs", 6, 3), ("xor", 2, 1), ("rs", 4, 2), ("rs", 10, 4)])
@pytest.mark.parametrize("shift,n", [(0, 65536), (3, 65536 + 5)])
def test_units_more_than_2gib_apart(codec, k, p, shift, n):
    S, bpc = 2, 16384
    ss = n + 4096 + shift  # stripe stride: stripes side by side inside each unit slot
    span = (k + p - 1) * US + (S - 1) * ss + n
    buf = torch.empty(shift + span + 64, dtype=torch.uint8, device=DEV)
    base = buf[shift:]
    rng = np.random.default_rng([k, p, n, shift])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)

    def at(s, u):
        off = s * ss + u * US
        return base[off:off + n]
    for s in range(S):
        for u in range(k):
            at(s, u).copy_(to_dev(data[s, u]))
        for u in range(k, k + p):
            at(s, u).fill_(0x3C)
    guard_after = [base[s * ss + u * US + n:s * ss + u * US + n + 16].clone() for s in range(S) for u in range(k + p)]
    conf = rc.ECReplicationConfig(k, p, codec)
    nwin = -(-n // bpc)
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    fused_shape = (codec, k, p) in (("rs", 6, 3), ("xor", 2, 1), ("rs", 10, 4))
    r0 = _routes()
    rc.RawErasureEncoder(conf).encode_crc_batch(base, ss, US, base[k * US:], ss, US, S, n, ck.ChecksumType.CRC32C,
                                                bpc, crcs)
    r1 = _routes()
    # round 6: the fused shapes take ONE fused launch (one buffer descriptor per unit, WIDE), any length and offset
    if not PRODUCTION_ROUTING:  # (libozec's own routing sends batches this small to the unfused kernels)
        assert (r1[0] - r0[0], r1[1] - r0[1]) == ((1, 0) if fused_shape else (0, 1)), (codec, k, p, r0, r1)
    erased = [0] if codec == "xor" else [0, k]
    present = [u for u in range(k + p) if u not in erased][:k]
    out = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    rc.RawErasureDecoder(conf).decode_batch(base, ss, US, present, erased, out, len(erased) * n, n, S, n)
    rout = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    rcrc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    r0 = _routes()
    rc.RawErasureDecoder(conf).reconstruct_crc_batch(base, ss, US, present, erased, rout, len(erased) * n, n, S, n,
                                                     ck.ChecksumType.CRC32C, bpc, rcrc, d_expected=crcs,
                                                     d_mismatch=mism)
    r1 = _routes()
    rec_fused = (codec, k, p) in (("rs", 6, 3), ("xor", 2, 1), ("rs", 10, 4))  # rs-6-3 erasing 2: shape (6, 2)
    if not PRODUCTION_ROUTING:
        assert (r1[0] - r0[0], r1[1] - r0[1]) == ((1, 0) if rec_fused else (0, 1)), (codec, k, p, r0, r1)
    wcrc = torch.zeros((k + p, nwin), dtype=torch.int32, device=DEV)  # every unit of stripe 1, cell stride US
    ck.checksum_windows_batch(ck.ChecksumType.CRC32, base[ss:], US, k + p, n, bpc, wcrc)
    torch.cuda.synchronize()
    c, o, w = to_host(crcs).view(np.uint32), to_host(out), to_host(wcrc).view(np.uint32)
    ro, rcc, m = to_host(rout), to_host(rcrc).view(np.uint32), to_host(mism)
    for s in range(S):
        ref = [oracle.xor_encode(list(data[s]))] if codec == "xor" else oracle.rs_encode(k, p, list(data[s]))
        units = list(data[s]) + list(ref)
        for q in range(p):
            assert (to_host(at(s, k + q)) == ref[q]).all(), (codec, k, p, shift, n, s, q)
        for u in range(k + p):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, units[u], bpc)).all(), (codec, s, u)
        for i, e in enumerate(erased):
            assert (o[s, i] == units[e]).all(), (codec, s, e)
            assert (ro[s, i] == units[e]).all() and (rcc[s, i] == c[s, e]).all(), (codec, s, e)
        assert m[s] == -1, (codec, s, m)
        if s == 1:
            for u in range(k + p):
                assert (w[u] == oracle.crc_windows(oracle.CRC32, units[u], bpc)).all(), (codec, u)
    i = 0
    for s in range(S):
        for u in range(k + p):
            assert torch.equal(base[s * ss + u * US + n:s * ss + u * US + n + 16], guard_after[i]), (codec, s, u)
            i += 1


@pytest.mark.parametrize("codec,k,p", [("rs", 6, 3), ("xor", 2, 1)])
def test_wide_fused_at_bench_cell_size(codec, k, p):
    """The WIDE fused forms at the bench's cell size (profiles/r06/fused_ab/): 24 stripes of 1 MiB cells, units 768 MiB
    apart, at an odd base -- one fused launch (past the small-batch threshold under libozec's own routing too), every
    stripe's parity and all units' CRC32C windows vs the oracle, and a fused reconstruction of two units (one) whose
    rebuilt units and CRCs match and whose verification of the stored CRCs passes."""
    S, n, bpc, shift = 24, 1 << 20, 16384, 3
    ss = n
    buf = torch.empty(shift + (k + p - 1) * US + S * ss + 64, dtype=torch.uint8, device=DEV)
    base = buf[shift:]
    rng = np.random.default_rng([k, p, 24])
    data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
    for u in range(k):
        base[u * US:u * US + S * ss].copy_(to_dev(data[:, u].reshape(-1)))
    conf = rc.ECReplicationConfig(k, p, codec)
    nwin = n // bpc
    crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    r0 = _routes()
    rc.RawErasureEncoder(conf).encode_crc_batch(base, ss, US, base[k * US:], ss, US, S, n, ck.ChecksumType.CRC32C,
                                                bpc, crcs)
    r1 = _routes()
    assert (r1[0] - r0[0], r1[1] - r0[1]) == (1, 0), (r0, r1)
    erased = [0] if codec == "xor" else [1, k + 1]
    present = [u for u in range(k + p) if u not in erased][:k]
    rout = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    rcrc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    rc.RawErasureDecoder(conf).reconstruct_crc_batch(base, ss, US, present, erased, rout, len(erased) * n, n, S, n,
                                                     ck.ChecksumType.CRC32C, bpc, rcrc, d_expected=crcs,
                                                     d_mismatch=mism)
    torch.cuda.synchronize()
    c = to_host(crcs).view(np.uint32)
    par = [to_host(base[(k + q) * US:(k + q) * US + S * ss]).reshape(S, n) for q in range(p)]
    ro, rcc, m = to_host(rout), to_host(rcrc).view(np.uint32), to_host(mism)
    for s in range(S):
        ref = [oracle.xor_encode(list(data[s]))] if codec == "xor" else oracle.rs_encode(k, p, list(data[s]))
        units = list(data[s]) + list(ref)
        for q in range(p):
            assert (par[q][s] == ref[q]).all(), (codec, s, q)
        for u in range(k + p):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, units[u], bpc)).all(), (codec, s, u)
        for i, e in enumerate(erased):
            assert (ro[s, i] == units[e]).all() and (rcc[s, i] == c[s, e]).all(), (codec, s, e)
        assert m[s] == -1, (codec, s, m)
    del buf, base
