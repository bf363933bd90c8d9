"""Every recoverable erasure set, on the GPU (TestECBlockReconstructedStripeInputStream.java:94-213 reconstructs every
recoverable index set of rs-3-2; TestRSRawCoderBase.java:33-115 lists rs-6-3 / rs-10-4 patterns).

For rs-3-2, rs-6-3 and rs-10-4 every erasure set of 1..p units (data indexes first, ascending: the order
RSRawDecoder expects, TestCoderBase.java:172-187) is decoded from the first k valid units by ozec_decode_batch and,
for rs-3-2 / rs-6-3, rebuilt with CRC verification by ozec_reconstruct_crc_batch -- each against the original units
and their oracle CRCs.  Cells have odd lengths (a short last CRC window); p + 1 erasures must be refused.
"""
import itertools

import numpy as np
import pytest

import oracle
from synth import SEED, cells

torch = pytest.importorskip("torch")
from devcopy import to_dev, to_host  # noqa: E402
pytestmark = pytest.mark.gpu

from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

DEV = "cuda:0"


def _units(k, p, n, S, first):
    data = [cells(SEED, first + s * k, k, n) for s in range(S)]
    return np.stack([np.stack(d + oracle.rs_encode(k, p, d)) for d in data])  # [S][k+p][n]


def _sets(k, p):
    return [list(c) for ne in range(1, p + 1) for c in itertools.combinations(range(k + p), ne)]


@pytest.mark.parametrize("k,p", [(3, 2), (6, 3), (10, 4)])
def test_decode_every_recoverable_set(k, p):
    n, S = 3001, 2
    units = _units(k, p, n, S, 600000 + k)
    d_in = to_dev(units)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    sets = _sets(k, p)
    d_out = torch.empty((S, p, n), dtype=torch.uint8, device=DEV)
    for erased in sets:
        present = [u for u in range(k + p) if u not in erased]
        d_out.fill_(0xA5)
        dec.decode_batch(d_in, (k + p) * n, n, present, erased, d_out, p * n, n, S, n)
        got = to_host(d_out)
        for i, e in enumerate(erased):
            assert (got[:, i] == units[:, e]).all(), (k, p, erased, e)
    assert len(sets) == sum(len(list(itertools.combinations(range(k + p), ne))) for ne in range(1, p + 1))
    too_many = list(range(p + 1))
    with pytest.raises(Exception):
        dec.decode_batch(d_in, (k + p) * n, n, [u for u in range(k + p) if u not in too_many], too_many, d_out,
                         p * n, n, S, n)


@pytest.mark.parametrize("k,p,bpc", [(3, 2, 1024), (6, 3, 512)])
def test_reconstruct_every_recoverable_set_with_crcs(k, p, bpc):
    """Fused verify + decode + CRC for every erasure set: rebuilt units equal the originals, their window CRCs equal
    the oracle's, and no stored CRC of a read unit is reported."""
    n, S = 4 * bpc + 100, 2
    units = _units(k, p, n, S, 610000 + k)
    nwin = -(-n // bpc)
    stored = np.stack([np.stack([oracle.crc_windows(oracle.CRC32C, units[s, u], bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32)
    d_in = to_dev(units)
    d_exp = to_dev(stored.view(np.int32))
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    d_out = torch.empty((S, p, n), dtype=torch.uint8, device=DEV)
    mism = torch.empty(S, dtype=torch.int32, device=DEV)
    for erased in _sets(k, p):
        present = [u for u in range(k + p) if u not in erased]
        d_out.fill_(0xA5)
        d_crc = torch.empty((S, len(erased), nwin), dtype=torch.int32, device=DEV)  # [stripe][rebuilt unit][window]
        dec.reconstruct_crc_batch(d_in, (k + p) * n, n, present, erased, d_out, p * n, n, S, n,
                                  ck.ChecksumType.CRC32C, bpc, d_crc, d_expected=d_exp, d_mismatch=mism)
        got, crcs, m = to_host(d_out), to_host(d_crc).view(np.uint32), to_host(mism)
        assert (m == -1).all(), (k, p, erased, m)
        for i, e in enumerate(erased):
            assert (got[:, i] == units[:, e]).all(), (k, p, erased, e)
            assert (crcs[:, i] == stored[:, e]).all(), (k, p, erased, e)
