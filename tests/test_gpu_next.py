"""SURVEY.md §8(f) rows 1-2 on the GPU vs the oracle: batched checksum verify (datanode scanner) and the fused
reconstruction pass (verify read units' CRCs + decode + CRC of rebuilt units)."""
import numpy as np
import pytest

import oracle
from synth import SEED, cells
import variants

torch = pytest.importorskip("torch")
from devcopy import to_dev, to_host  # noqa: E402
pytestmark = pytest.mark.gpu

from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

DEV = "cuda:0"


def t(a):
    return to_dev(a)  # pinned staging, never a pageable DMA (devcopy.py)


def h(x):
    return to_host(x)


@pytest.mark.parametrize("ctype,otype", [(ck.ChecksumType.CRC32C, oracle.CRC32C), (ck.ChecksumType.CRC32, oracle.CRC32)])
@pytest.mark.parametrize("bpc,big_endian", [(16384, False), (16384, True), (4096, False), (1000, False)])
def test_checksum_verify_batch(ctype, otype, bpc, big_endian):
    C, n = 6, 100_000
    data = np.stack(cells(SEED, 60000, C, n))
    nwin = (n + bpc - 1) // bpc
    exp = np.stack([oracle.crc_windows(otype, data[c], bpc) for c in range(C)]).astype(np.uint32)
    if big_endian:
        exp = exp.byteswap()
    bad = data.copy()
    bad[2, 5 * bpc + 7] ^= 0x40          # window 5 of cell 2
    bad[4, n - 1] ^= 1                   # last window of cell 4
    d_exp = t(exp.view(np.int32))
    mism = torch.zeros(C, dtype=torch.int32, device=DEV)
    ck.checksum_verify_batch(ctype, t(bad), n, C, n, bpc, d_exp, mism, expected_big_endian=big_endian)
    got = h(mism)
    assert got.tolist() == [-1, -1, 5, -1, nwin - 1, -1]
    ck.checksum_verify_batch(ctype, t(data), n, C, n, bpc, d_exp, mism, expected_big_endian=big_endian)
    assert h(mism).tolist() == [-1] * C


def _stripe_units(codec, k, p, n, S, first):
    out = []
    for s in range(S):
        d = cells(SEED, first + s * k, k, n)
        par = oracle.rs_encode(k, p, d) if codec == "rs" else [oracle.xor_encode(d)]
        out.append(np.stack(d + par))
    return np.stack(out)  # [S][k+p][n]


@pytest.mark.parametrize("codec,k,p,erased,n,bpc", [
    ("rs", 6, 3, [0, 2, 7], 1 << 18, 16384),      # fused shape (6,3)
    ("rs", 6, 3, [1], 1 << 18, 16384),            # fused shape (6,1)
    ("rs", 10, 4, [0, 1, 2, 3], 1 << 17, 16384),  # fused shape (10,4)
    ("rs", 10, 4, [1, 4, 10, 13], 1 << 17, 16384),
    ("rs", 3, 2, [0, 4], 1 << 16, 4096),
    ("xor", 2, 1, [1], 1 << 16, 16384),           # fused shape (2,1)
    ("rs", 5, 2, [0, 6], 1 << 16, 16384),         # unfused fallback (shape not instantiated)
    ("rs", 6, 3, [0, 2, 7], 50000, 1000),         # unfused fallback (bpc not a multiple of 16)
    ("rs", 10, 4, [1, 4, 10, 13], 8 * 16384 + 2048, 16384),  # nibble kernel, short last window (2 KiB)
    ("rs", 3, 2, [0, 4], 1524 * 1024, 16384),     # rs-3-2-1524k: a 4 KiB last window
    ("rs", 3, 2, [4], 1 << 16, 16384),            # fused shape (3,1): single-unit reconstruction
    ("rs", 6, 3, [2], 4 * 16384 + 3008, 16384),   # nibble kernel, a 3008-B last window (virtual zero blocks in front)
    ("rs", 10, 4, [0, 5, 11], 3 * 16384 + 16, 16384),  # ... and a one-block last window
    # byte-granular cells at odd unit strides (round 5, nb_tail): blocks + a 3-B tail, a 7-B last window with no
    # whole block (the planted corruption sits in it), 50,001 B (an 849-B last window: 53 blocks + 1 B)
    ("rs", 6, 3, [0, 2, 7], 4 * 16384 + 3011, 16384),
    ("rs", 10, 4, [1, 4, 10, 13], 3 * 16384 + 7, 16384),
    ("rs", 3, 2, [0, 4], 50001, 16384),
])
@pytest.mark.parametrize("variant", [0] + variants.RS_FUSED + [4, 5])
def test_reconstruct_crc_batch(codec, k, p, erased, n, bpc, variant):
    """Fused reconstruction (verify + decode + CRC) vs the oracle for the default and every fused alternate the library
    holds (49 per-window, 56 / 59 streamed-input, 62-177 nibble-table; 4 / 5 the XOR codec's XO forms)."""
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", variant) == 0
    try:
        _reconstruct_case(codec, k, p, erased, n, bpc)
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)


def _reconstruct_case(codec, k, p, erased, n, bpc):
    S = 4
    units = _stripe_units(codec, k, p, n, S, 70000)
    ctype, otype = ck.ChecksumType.CRC32C, oracle.CRC32C
    nwin = (n + bpc - 1) // bpc
    stored = np.stack([np.stack([oracle.crc_windows(otype, units[s, u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)                     # [S][k+p][nwin]
    present = [u for u in range(k + p) if u not in erased]
    read = present[:k]
    corrupted = units.copy()
    corrupted[:, [e for e in erased]] = 0xEE                                     # erased units are garbage
    corrupted[1, read[-1], 3 * bpc + 1] ^= 0x10                                  # stripe 1: silent corruption
    d_in = t(corrupted)
    d_out = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    d_crc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec))
    dec.reconstruct_crc_batch(d_in, (k + p) * n, n, present, erased, d_out, len(erased) * n, n, S, n, ctype, bpc,
                              d_crc, d_expected=t(stored.view(np.int32)), d_mismatch=mism)
    out, crcs, m = h(d_out), h(d_crc).view(np.uint32), h(mism)
    assert m[0] == -1 and m[2] == -1 and m[3] == -1
    assert m[1] == read[-1] * nwin + 3
    for s in (0, 2, 3):  # clean stripes rebuild exactly, and their CRCs equal the stored ones
        for i, e in enumerate(erased):
            assert (out[s, i] == units[s, e]).all(), (s, e)
            assert (crcs[s, i] == stored[s, e]).all(), (s, e)
    for i in range(len(erased)):  # the corrupted stripe's rebuilt CRCs still describe what was written
        assert (crcs[1, i] == oracle.crc_windows(otype, out[1, i], bpc)).all()


# ------------------------------------------------------------------ §8(f) row 4: COMPOSITE_CRC


@pytest.mark.parametrize("ctype,otype", [(ck.ChecksumType.CRC32C, oracle.CRC32C), (ck.ChecksumType.CRC32, oracle.CRC32)])
@pytest.mark.parametrize("n,bpc,big_endian", [(1 << 20, 16384, False), (1 << 20, 16384, True), (100_000, 4096, False),
                                              (5000, 16384, False), (64 * 512, 512, False), (65 * 512 + 7, 512, True),
                                              (1000 * 100, 100, False)])
def test_compose_windows_batch_is_cell_crc(ctype, otype, n, bpc, big_endian):
    """GPU window CRCs -> GPU CrcComposer per cell == CRC of the whole cell (oracle)."""
    from ozone_amd import composite as cc
    C = 5
    data = np.stack(cells(SEED, 81000, C, n))
    nwin = (n + bpc - 1) // bpc
    d_crc = torch.zeros((C, nwin), dtype=torch.int32, device=DEV)
    ck.checksum_windows_batch(ctype, t(data), n, C, n, bpc, d_crc, big_endian=big_endian)
    d_out = torch.zeros(C, dtype=torch.int32, device=DEV)
    cc.compose_windows_batch(ctype, d_crc, nwin, C, nwin, bpc, n - (nwin - 1) * bpc, d_out,
                             crcs_big_endian=big_endian, out_big_endian=big_endian)
    got = h(d_out).view(np.uint32)
    if big_endian:
        got = got.byteswap()
    assert got.tolist() == [oracle.crc(otype, data[c]) for c in range(C)]


def test_ec_file_composite_crc_from_fused_kernel():
    """Writer side end to end: fused rs-6-3 encode + CRC32C windows on the GPU, stripe checksums as
    ECBlockOutputStreamEntry.calculateChecksum builds them, ECBlockChecksumComputer COMPOSITE_CRC == CRC32C of
    the key bytes (whole stripes) and == the oracle restatement of the computer."""
    from ozone_amd import composite as cc
    k, p, n, S, bpc = 6, 3, 1 << 18, 3, 16384
    key = cells(SEED, 82000, 1, S * k * n)[0]
    data = key.reshape(S, k, n)
    nwin = n // bpc
    d_out = torch.zeros((S, p, n), dtype=torch.uint8, device=DEV)
    d_crc = torch.zeros((S, k + p, nwin), dtype=torch.int32, device=DEV)
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    e.encode_crc_batch(t(data), k * n, n, d_out, p * n, n, S, n, ck.ChecksumType.CRC32C, bpc, d_crc, big_endian=True)
    crc_bytes = h(d_crc).view(np.uint8).reshape(S, k + p, nwin * 4)
    infos = []
    for s in range(S):
        cds = [ck.ChecksumData(ck.ChecksumType.CRC32C, bpc, [crc_bytes[s, u, 4 * w:4 * w + 4].tobytes()
                                                              for w in range(nwin)]) for u in range(k + p)]
        infos.append(cc.ChunkInfo(n, cds[0], cc.stripe_checksum(cds)))
    comp = cc.ECBlockChecksumComputer(infos, key.size, p)
    comp.compute(cc.ChecksumCombineMode.COMPOSITE_CRC)
    assert int.from_bytes(comp.get_out_bytes(), "big") == oracle.crc(oracle.CRC32C, key)
    assert comp.get_out_bytes() == oracle.ec_block_composite_crc(oracle.CRC32C, [i.stripe_checksum for i in infos],
                                                                 n, bpc, key.size, p)
    # per-cell composites on the GPU agree with the host computer's view of each data cell
    d_cell = torch.zeros((S, k + p), dtype=torch.int32, device=DEV)
    cc.compose_windows_batch(ck.ChecksumType.CRC32C, d_crc, nwin, S * (k + p), nwin, bpc, bpc, d_cell,
                             crcs_big_endian=True)
    cell = h(d_cell).view(np.uint32)
    assert all(cell[s, u] == oracle.crc(oracle.CRC32C, data[s, u]) for s in range(S) for u in range(k))
