"""Combined input verification (fused_nb.hpp CV variants 231 / 234, round 5) vs the oracle (GPU).

A reconstruction that checks the stored CRCs of the units it reads keeps one register for all of them, weighted per
input (kernels.hpp kCv*), and re-verifies a failing stripe unit by unit (fused.hip nb_reverify).  The report must be
the reference's first failing (unit, window) (ChecksumData.java:118-150) whatever the corruption: one unit, two units
with the same error pattern at the same offsets (the pair the weights separate, tests/test_cv_weights.py), several
windows and units, every stripe of a batch; the rebuilt units and their CRCs bit-exact either way.
"""
import numpy as np
import pytest

import oracle
from synth import SEED, cells

torch = pytest.importorskip("torch")
from devcopy import to_dev, to_host  # noqa: E402
pytestmark = pytest.mark.gpu

from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

DEV = "cuda:0"


def _units(k, p, n, S, first):
    out = []
    for s in range(S):
        d = cells(SEED, first + s * k, k, n)
        out.append(np.stack(d + oracle.rs_encode(k, p, d)))
    return np.stack(out)


def _first_failure(units, corrupted, read, nwin, bpc, otype):
    """the reference's report: min over the read units u and windows w of u * nwin + w whose CRC changed"""
    for u in sorted(read):
        a = oracle.crc_windows(otype, units[u], bpc)
        b = oracle.crc_windows(otype, corrupted[u], bpc)
        diff = np.nonzero(np.asarray(a) != np.asarray(b))[0]
        if len(diff):
            return u * nwin + int(diff[0])
    return -1


CASES = {
    "none": [],
    "one unit": [(2, 3 * 16384 + 5, 0x01)],
    "two units, same pattern": [(1, 7 * 16384 + 100, 0x80), (4, 7 * 16384 + 100, 0x80)],
    "two units, same zeroed range": "zero",
    "several windows and units": [(9, 2 * 16384, 0x10), (3, 60 * 16384 + 7, 0xff), (3, 5, 0x02)],
}


@pytest.mark.parametrize("variant", [231, 234, 0])
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("ctype,otype", [(ck.ChecksumType.CRC32C, oracle.CRC32C), (ck.ChecksumType.CRC32, oracle.CRC32)])
def test_combined_verify_reports_the_first_failure(variant, case, ctype, otype):
    k, p, n, bpc, S = 10, 4, 1 << 20, 16384, 3
    erased = [1, 4, 10, 13]
    present = [u for u in range(k + p) if u not in erased]
    read = present[:k]
    nwin = n // bpc
    units = _units(k, p, n, S, 91000)
    stored = np.stack([np.stack([oracle.crc_windows(otype, units[s, u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)
    corrupted = units.copy()
    corrupted[:, erased] = 0x5A
    bad = 1  # the corrupted stripe; 0 and 2 stay clean
    spec = CASES[case]
    if spec == "zero":  # both units' bytes of one range replaced by the same values (a shared stuck pattern)
        corrupted[bad, read[2], 9000:9100] = 0
        corrupted[bad, read[6], 9000:9100] = 0
        corrupted[bad, read[2], 9000] ^= 0x40  # ensure the two ranges really changed
        corrupted[bad, read[6], 9000] ^= 0x40
    else:
        for ui, pos, mask in spec:
            corrupted[bad, read[ui], pos] ^= mask
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", variant) == 0
    try:
        d_out = torch.zeros((S, 4, n), dtype=torch.uint8, device=DEV)
        d_crc = torch.zeros((S, 4, nwin), dtype=torch.int32, device=DEV)
        mism = torch.zeros(S, dtype=torch.int32, device=DEV)
        rc.RawErasureDecoder(rc.ECReplicationConfig(k, p)).reconstruct_crc_batch(
            to_dev(corrupted), (k + p) * n, n, present, erased, d_out, 4 * n, n, S, n, ctype, bpc,
            d_crc, d_expected=to_dev(stored.view(np.int32)), d_mismatch=mism)
        torch.cuda.synchronize()
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    m, out, oc = to_host(mism), to_host(d_out), to_host(d_crc).view(np.uint32)
    want = _first_failure(units[bad], corrupted[bad], read, nwin, bpc, otype)
    assert m[0] == -1 and m[2] == -1, (case, m)
    assert m[1] == want, (case, variant, m[1], want)
    for s in (0, 2):
        for i, e in enumerate(erased):
            assert (out[s, i] == units[s, e]).all() and (oc[s, i] == stored[s, e]).all(), (case, s, e)
    for i in range(4):  # the corrupted stripe's rebuilt CRCs describe what was written
        assert (oc[bad, i] == oracle.crc_windows(otype, out[bad, i], bpc)).all()


@pytest.mark.parametrize("variant", [231, 234])
def test_combined_variants_without_expected_crcs_and_for_encode(variant):
    """Without stored CRCs (decode + CRC of the rebuilt units only) and for encodes, the CV ids run their non-CV
    geometry: same bytes and CRCs as the oracle."""
    k, p, n, bpc, S = 6, 3, 1 << 18, 16384, 4
    units = _units(k, p, n, S, 93000)
    erased = [0, 5, 7]
    present = [u for u in range(k + p) if u not in erased]
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", variant) == 0
    try:
        d_out = torch.zeros((S, 3, n), dtype=torch.uint8, device=DEV)
        d_crc = torch.zeros((S, 3, n // bpc), dtype=torch.int32, device=DEV)
        rc.RawErasureDecoder(rc.ECReplicationConfig(k, p)).reconstruct_crc_batch(
            to_dev(units), (k + p) * n, n, present, erased, d_out, 3 * n, n, S, n,
            ck.ChecksumType.CRC32C, bpc, d_crc)
        enc_units = to_dev(units)
        enc_units[:, k:] = 0
        crcs = torch.zeros((S, k + p, n // bpc), dtype=torch.int32, device=DEV)
        rc.RawErasureEncoder(rc.ECReplicationConfig(k, p)).encode_crc_batch(
            enc_units, (k + p) * n, n, enc_units[:, k:], (k + p) * n, n, S, n, ck.ChecksumType.CRC32C, bpc, crcs)
        torch.cuda.synchronize()
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    out, oc = to_host(d_out), to_host(d_crc).view(np.uint32)
    eu, c = to_host(enc_units), to_host(crcs).view(np.uint32)
    for s in range(S):
        for i, e in enumerate(erased):
            assert (out[s, i] == units[s, e]).all()
            assert (oc[s, i] == oracle.crc_windows(oracle.CRC32C, units[s, e], bpc)).all()
        assert (eu[s] == units[s]).all()
        for u in range(k + p):
            assert (c[s, u] == oracle.crc_windows(oracle.CRC32C, units[s, u], bpc)).all()


@pytest.mark.parametrize("variant", [0, 24])
@pytest.mark.parametrize("bpc", [4096, 16384])
@pytest.mark.parametrize("ctype,otype", [(ck.ChecksumType.CRC32C, oracle.CRC32C), (ck.ChecksumType.CRC32, oracle.CRC32)])
def test_verify_run_check_reports_the_first_failing_window(variant, bpc, ctype, otype):
    """ozec_checksum_verify_batch (the datanode scanner) checks a run of windows as one message (crc_windows_g26s VR,
    the default) and re-checks a failing run window by window (24: always window by window).  Corruptions: one byte;
    the same pattern in two windows of one run (the pair the run weights separate); in two cells whose windows share a
    run; in a cell's last full window; none -- the per-cell first failing window vs the oracle."""
    C, n = 24, 1 << 20  # 24 cells of 64 (bpc 16 KiB) or 256 windows
    nwin = n // bpc
    data = np.stack(cells(SEED, 95000, C, n))
    exp = np.stack([oracle.crc_windows(otype, data[c], bpc) for c in range(C)]).astype(np.uint32)
    bad = data.copy()
    bad[1, 3 * bpc + 17] ^= 0x04                                   # one byte
    bad[5, 2 * bpc + 100] ^= 0x81                                  # same pattern, two windows of one run
    bad[5, 9 * bpc + 100] ^= 0x81
    bad[7, n - 1] ^= 0x10                                          # the cell's last (full) window
    bad[8, 0] ^= 0x01                                              # first window of a cell ...
    bad[9, 5] ^= 0x01                                              # ... and of the next one (often one run)
    want = np.full(C, -1)
    for c in range(C):
        diff = np.nonzero(np.asarray(oracle.crc_windows(otype, bad[c], bpc), np.uint32) != exp[c])[0]
        if len(diff):
            want[c] = int(diff[0])
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", variant) == 0
    try:
        mism = torch.zeros(C, dtype=torch.int32, device=DEV)
        ck.checksum_verify_batch(ctype, to_dev(bad), n, C, n, bpc,
                                 to_dev(exp.view(np.int32)), mism)
        torch.cuda.synchronize()
        got = to_host(mism)
        ck.checksum_verify_batch(ctype, to_dev(data), n, C, n, bpc,
                                 to_dev(exp.view(np.int32)), mism)
        torch.cuda.synchronize()
        clean = to_host(mism)
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    assert got.tolist() == want.tolist(), (variant, bpc)
    assert clean.tolist() == [-1] * C


@pytest.mark.parametrize("k,p,erased", [(10, 4, [0, 1, 2, 3]), (6, 3, [2, 7])])
def test_combined_verify_every_stripe_failing(k, p, erased):
    """Every stripe of the batch fails its combined check (a whole corrupted replica): each is re-verified window by
    window (nb_reverify, one wave per (input, window)) and reports its own first failing (unit, window), including a
    corruption in a cell's short last window and one in a virtual-padded first step; the rebuilt units stay exact."""
    n, bpc, S = 3 * 16384 + 4096, 16384, 6  # a short last window of 4 KiB
    nwin = -(-n // bpc)
    units = _units(k, p, n, S, 97000)
    stored = np.stack([np.stack([oracle.crc_windows(oracle.CRC32C, units[s, u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)
    present = [u for u in range(k + p) if u not in erased]
    read = present[:k]
    corrupted = units.copy()
    corrupted[:, erased] = 0x11
    rng = np.random.default_rng([k, p, 5])
    for s in range(S):
        for _ in range(1 + s % 3):
            corrupted[s, read[int(rng.integers(0, k))], int(rng.integers(0, n))] ^= int(rng.integers(1, 256))
    corrupted[S - 1, read[k - 1], n - 1] ^= 0x80  # the short last window of the last read unit
    lib = L.lib()
    d_out = torch.zeros((S, len(erased), n), dtype=torch.uint8, device=DEV)
    d_crc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device=DEV)
    mism = torch.zeros(S, dtype=torch.int32, device=DEV)
    assert lib.ozec_set_tuning(b"crc_variant", 231) == 0
    try:
        rc.RawErasureDecoder(rc.ECReplicationConfig(k, p)).reconstruct_crc_batch(
            to_dev(corrupted), (k + p) * n, n, present, erased, d_out, len(erased) * n, n, S, n,
            ck.ChecksumType.CRC32C, bpc, d_crc, d_expected=to_dev(stored.view(np.int32)),
            d_mismatch=mism)
        torch.cuda.synchronize()
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    m = to_host(mism)
    for s in range(S):
        assert m[s] == _first_failure(units[s], corrupted[s], read, nwin, bpc, oracle.CRC32C), (s, m)
