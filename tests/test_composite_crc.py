"""COMPOSITE_CRC (CrcUtil, CrcComposer, block checksum computers) and stripe checksums.

Pinning: CrcUtil.compose is the CRC concatenation operator, so composing window CRCs must give the CRC of the
concatenated bytes -- checked against zlib.crc32 (an implementation independent of the reference and of this
repo) for CRC32, and against the oracle's CrcIntTable restatement for CRC32C. The oracle's CrcComposer and block
computers (oracle/ozec_oracle.c, oracle/oracle.py) restate the reference line by line; libozec must agree."""
import hashlib
import zlib

import numpy as np
import pytest

import oracle
from synth import SEED, cells

from ozone_amd import composite as cc
from ozone_amd.checksum import ChecksumData, ChecksumType
from ozone_amd.rawcoder import IllegalArgumentException, IOException

OT = {ChecksumType.CRC32: oracle.CRC32, ChecksumType.CRC32C: oracle.CRC32C}
TYPES = [ChecksumType.CRC32, ChecksumType.CRC32C]


def _rng(i):
    return np.random.default_rng(1000 + i)


# ---------------------------------------------------------------- oracle pinning


def test_oracle_compose_is_crc_concatenation():
    r = _rng(0)
    for _ in range(300):
        a = r.integers(0, 256, r.integers(0, 700), dtype=np.uint8).tobytes()
        b = r.integers(0, 256, r.integers(0, 700), dtype=np.uint8).tobytes()
        assert oracle.crc_compose(oracle.CRC32, zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)
        assert oracle.crc_compose(oracle.CRC32C, oracle.crc(oracle.CRC32C, a), oracle.crc(oracle.CRC32C, b),
                                  len(b)) == oracle.crc(oracle.CRC32C, a + b)
    assert oracle.crc_monomial(oracle.CRC32, 0) == 0x80000000
    with pytest.raises(ValueError):
        oracle.crc_monomial(oracle.CRC32, -1)


def test_oracle_composer_windows_equal_whole_crc():
    data = cells(SEED, 77000, 1, 100_000)[0]
    for ct in (oracle.CRC32, oracle.CRC32C):
        c = oracle.Composer(ct, 4096)
        w = oracle.crc_windows(ct, data, 4096)
        for i, v in enumerate(w):
            c.update(int(v), min(4096, data.size - i * 4096))
        assert int.from_bytes(c.digest(), "big") == oracle.crc(ct, data)
    assert zlib.crc32(data.tobytes()) == oracle.crc(oracle.CRC32, data)


# ---------------------------------------------------------------- libozec vs oracle (host ABI)


@pytest.mark.parametrize("ctype", TYPES)
def test_crcutil_matches_oracle(ctype):
    r = _rng(1)
    for length in [0, 1, 3, 16, 4096, 16384, 1 << 20, 1524 * 1024, (1 << 40) + 12345, 2 ** 62]:
        assert cc.CrcUtil.get_monomial(length, ctype) == oracle.crc_monomial(OT[ctype], length)
    for _ in range(200):
        a, b = (int(x) for x in r.integers(0, 1 << 32, 2, dtype=np.uint64))
        n = int(r.integers(0, 1 << 34))
        assert cc.CrcUtil.compose(a, b, n, ctype) == oracle.crc_compose(OT[ctype], a, b, n)
    assert cc.CrcUtil.compose(-5, 7, 0, ctype) == oracle.crc_compose(OT[ctype], -5 & 0xFFFFFFFF, 7, 0)
    with pytest.raises(IllegalArgumentException):
        cc.CrcUtil.get_monomial(-1, ctype)
    with pytest.raises(IllegalArgumentException):
        cc.CrcUtil.compose(1, 2, -3, ctype)
    with pytest.raises(IOException):
        cc.CrcUtil.get_crc_polynomial_for_type(ChecksumType.SHA256)
    assert cc.CrcUtil.get_crc_polynomial_for_type(ctype) == (0xEDB88320 if ctype == ChecksumType.CRC32 else 0x82F63B78)


def test_crcutil_byte_helpers():
    assert cc.CrcUtil.int_to_bytes(-2) == b"\xff\xff\xff\xfe"
    assert cc.CrcUtil.read_int(b"\x00\x01\x02\x03\x04", 1) == 0x01020304
    assert cc.CrcUtil.to_single_crc_string(b"\xde\xad\xbe\xef") == "0xdeadbeef"
    assert cc.CrcUtil.to_multi_crc_string(b"\x00\x00\x00\x01\x00\x00\x00\x02") == "[0x00000001, 0x00000002]"
    with pytest.raises(IOException):
        cc.CrcUtil.read_int(b"\x00\x01", 0)
    with pytest.raises(IOException):
        cc.CrcUtil.to_multi_crc_string(b"\x00\x01\x02")


@pytest.mark.parametrize("ctype", TYPES)
@pytest.mark.parametrize("hint,stripe", [(4096, 0), (4096, 16384), (512, 1536), (1, 7)])
def test_composer_matches_oracle(ctype, hint, stripe):
    r = _rng(hint + stripe)
    mine = cc.CrcComposer(ctype, hint, stripe)
    ref = oracle.Composer(OT[ctype], hint, stripe if stripe > 0 else (1 << 63) - 1)
    for step in range(400):
        crc = int(r.integers(0, 1 << 32, dtype=np.uint64)) if step % 37 else 0  # cur == 0 shortcut too
        n = hint if r.random() < 0.8 else int(r.integers(0, hint + 1))
        if stripe:
            n = hint if hint <= stripe else stripe
        mine.update(crc, n)
        ref.update(crc, n)
        if step % 53 == 0:
            assert mine.digest() == ref.digest()
    assert mine.digest() == ref.digest()
    assert mine.digest() == b""


def test_composer_errors_and_bytes():
    c = cc.CrcComposer.new_striped_crc_composer(ChecksumType.CRC32C, 4, 10)
    c.update(5, 4)
    c.update(6, 4)
    with pytest.raises(IOException):
        c.update(7, 4)  # position 12 passes the 10-byte stripe without landing on it
    c2 = cc.CrcComposer.new_crc_composer(ChecksumType.CRC32C, 4)
    with pytest.raises(IOException):
        c2.update_bytes(b"\x00" * 6, 0, 6, 4)
    c2.update_bytes(b"\x00\x00\x00\x05\x00\x00\x00\x06", 0, 8, 4)
    ref = oracle.Composer(oracle.CRC32C, 4)
    ref.update(5, 4)
    ref.update(6, 4)
    assert c2.digest() == ref.digest()
    c3 = cc.CrcComposer.new_crc_composer(ChecksumType.CRC32, 4)
    c3.update(9, 4)
    with pytest.raises(IllegalArgumentException):
        c3.update(1, -4)  # CrcUtil.compose -> getMonomial(negative)


# ---------------------------------------------------------------- block checksum computers


def _chunk(ctype, data, bpc):
    w = oracle.crc_windows(OT[ctype], data, bpc)
    return cc.ChunkInfo(len(data), ChecksumData(ctype, bpc, [int(x).to_bytes(4, "big") for x in w]))


def test_replicated_block_computer_reference_cases():
    """TestReplicatedBlockChecksumComputer.java:38-73."""
    chk = _rng(3).integers(0, 256, 32, dtype=np.uint8).tobytes()
    ci = cc.ChunkInfo(32, ChecksumData(ChecksumType.CRC32, 4, [chk]))
    comp = cc.ReplicatedBlockChecksumComputer([ci])
    comp.compute(cc.ChecksumCombineMode.MD5MD5CRC)
    assert comp.get_out_bytes() == hashlib.md5(chk).digest()
    ci = cc.ChunkInfo(32, ChecksumData(ChecksumType.CRC32C, 4, [chk]))
    comp = cc.ReplicatedBlockChecksumComputer([ci])
    comp.compute(cc.ChecksumCombineMode.COMPOSITE_CRC)
    ref = cc.CrcComposer.new_crc_composer(ChecksumType.CRC32C, 4)
    ref.update(cc.CrcUtil.read_int(chk), 4)
    assert comp.get_out_bytes() == ref.digest()


@pytest.mark.parametrize("ctype", TYPES)
def test_replicated_block_composite_is_block_crc(ctype):
    data = cells(SEED, 78000, 1, 3 * 50000 + 1234)[0]
    chunks = [data[i:i + 50000] for i in range(0, data.size, 50000)]
    infos = [_chunk(ctype, c, 4096) for c in chunks]
    comp = cc.ReplicatedBlockChecksumComputer(infos)
    comp.compute(cc.ChecksumCombineMode.COMPOSITE_CRC)
    got = int.from_bytes(comp.get_out_bytes(), "big")
    assert got == oracle.crc(OT[ctype], data)
    if ctype == ChecksumType.CRC32:
        assert got == zlib.crc32(data.tobytes())
    ref = oracle.replicated_block_composite_crc(
        OT[ctype], [(ci.length, [cc.CrcUtil.read_int(b) for b in ci.checksum_data.get_checksums()]) for ci in infos],
        4096)
    assert comp.get_out_bytes() == ref


def _ec_stripes(ctype, key, k, p, chunk, bpc):
    """Stripe checksums as ECBlockOutputStreamEntry.calculateChecksum builds them: cell u of stripe s holds key
    bytes [(s*k+u)*chunk, +chunk); parity cells are as long as the stripe's first cell."""
    infos = []
    stripes = -(-key.size // (k * chunk))
    for s in range(stripes):
        cds = []
        first = None
        for u in range(k):
            cell = key[(s * k + u) * chunk:(s * k + u + 1) * chunk]
            if cell.size == 0:
                continue
            first = cell.size if first is None else first
            cds.append(_chunk(ctype, cell, bpc).checksum_data)
        d = [key[(s * k + u) * chunk:(s * k + u + 1) * chunk] for u in range(k)]
        d = [np.concatenate([x, np.zeros(first - x.size, np.uint8)]) for x in d]
        par = oracle.rs_encode(k, p, d)
        cds += [_chunk(ctype, x, bpc).checksum_data for x in par]
        infos.append(cc.ChunkInfo(chunk, cds[0], cc.stripe_checksum(cds)))
    return infos


@pytest.mark.parametrize("ctype", TYPES)
@pytest.mark.parametrize("chunk,bpc,key_size", [(8192, 4096, 3 * 8192 * 4),        # aligned, whole stripes
                                                (10000, 4096, 3 * 10000 * 2),      # bpc does not divide the chunk
                                                (8192, 4096, 3 * 8192 * 2 + 5000),  # partial last stripe
                                                (10000, 4096, 3 * 10000 + 12345)])
def test_ec_block_composite_crc(ctype, chunk, bpc, key_size):
    k, p = 3, 2
    key = cells(SEED, 79000, 1, key_size)[0]
    infos = _ec_stripes(ctype, key, k, p, chunk, bpc)
    comp = cc.ECBlockChecksumComputer(infos, key_size, p)
    comp.compute(cc.ChecksumCombineMode.COMPOSITE_CRC)
    ref = oracle.ec_block_composite_crc(OT[ctype], [ci.stripe_checksum for ci in infos], chunk, bpc, key_size, p)
    assert comp.get_out_bytes() == ref
    if key_size % (k * chunk) == 0:  # whole stripes: the composite is the CRC of the key
        assert int.from_bytes(comp.get_out_bytes(), "big") == oracle.crc(OT[ctype], key)
    comp.compute(cc.ChecksumCombineMode.MD5MD5CRC)
    assert comp.get_out_bytes() == hashlib.md5(b"").digest()  # the reference's double digest()
