"""The CPU oracle (oracle/) pinned against the reference: literal-table hashes, Appendix B constants,
standard CRC check values, zlib, and the independent pyref restatement's golden vectors."""
import hashlib
import zlib

import numpy as np
import pytest

import oracle
import pyref
from golden_io import case_id, case_inputs, ec_cases, load, matches
from synth import SEED, cells


def test_gf_tables_match_reference_literals():
    pins = load("ref_pins.json")
    base, logb = oracle.gf_tables()
    assert hashlib.sha256(base.tobytes()).hexdigest() == pins["gf_base"]["sha256"]
    assert hashlib.sha256(logb.tobytes()).hexdigest() == pins["gf_log_base"]["sha256"]
    assert pins["gf_base"]["oracle_match"] and pins["gf_log_base"]["oracle_match"]
    assert pins["gf_mul_table_matches_bitwise"]


@pytest.mark.parametrize("ctype,key", [(oracle.CRC32, "crc32_table"), (oracle.CRC32C, "crc32c_table")])
def test_crc_tables_match_reference_literals(ctype, key):
    pins = load("ref_pins.json")
    t = oracle.crc_table(ctype)
    assert hashlib.sha256(t.astype("<u4").tobytes()).hexdigest() == pins[key]["sha256"]


def test_gf_mul_all_pairs_vs_bitwise():
    for a in range(256):
        row = [oracle.gf_mul(a, b) for b in range(0, 256, 7)]
        assert row == [pyref.gf_mul(a, b) for b in range(0, 256, 7)]
    assert all(oracle.gf_mul(a, oracle.gf_inv(a)) == 1 for a in range(1, 256))
    assert oracle.gf_inv(0) == 0


# SURVEY.md Appendix B (derived from the reference's GF tables)
APPENDIX_B = {
    (3, 2): ["f48e01", "47a77a"],
    (6, 3): ["7aba47a78ef4", "ba7aa747f48e", "ad9ddd983daa"],
    (10, 4): ["dd98ad9d5d963daa8ef4", "98dd9dad965daa3df48e", "3daa5d96ad9ddd9847a7", "aa3d965d9dad98dda747"],
}


@pytest.mark.parametrize("kp", list(APPENDIX_B))
def test_cauchy_parity_rows_appendix_b(kp):
    k, p = kp
    m = oracle.cauchy_matrix(k, p)
    assert (m[:k] == np.eye(k, dtype=np.uint8)).all()
    assert [bytes(r).hex() for r in m[k:]] == APPENDIX_B[kp]
    assert [bytes(r).hex() for r in pyref.cauchy(k, p)[k:]] == APPENDIX_B[kp]


def test_crc_check_values_and_zlib():
    assert oracle.crc(oracle.CRC32, b"123456789") == 0xCBF43926
    assert oracle.crc(oracle.CRC32C, b"123456789") == 0xE3069283
    for n in (0, 1, 7, 8, 9, 1000, 65537):
        d = cells(SEED, 777, 1, n)[0]
        assert oracle.crc(oracle.CRC32, d) == zlib.crc32(d.tobytes())
        assert oracle.crc(oracle.CRC32C, d) == pyref.crc(1, d.tobytes())
    assert oracle.crc(oracle.CRC32C, b"\x01" * 33) == pyref.crc_bitwise(1, b"\x01" * 33)


@pytest.mark.parametrize("case", ec_cases("encode"), ids=case_id)
def test_oracle_encode_golden(case):
    data = case_inputs(case)
    par = oracle.rs_encode(case["k"], case["p"], data) if case["codec"] == "rs" else [oracle.xor_encode(data)]
    assert all(matches(b, x) for b, x in zip(case["parity"], par))


@pytest.mark.parametrize("case", ec_cases("decode"), ids=case_id)
def test_oracle_decode_golden(case):
    k, p = case["k"], case["p"]
    data = case_inputs(case)
    if case["codec"] == "rs":
        units = data + oracle.rs_encode(k, p, data)
        inputs = [units[u] if u in case["present"] else None for u in range(k + p)]
        out = oracle.rs_decode(k, p, inputs, case["erased"])
        dm = oracle.rs_decode_matrix(k, p, case["present"], case["erased"])
        assert [bytes(r).hex() for r in dm] == case["decode_matrix"]
    else:
        units = data + [oracle.xor_encode(data)]
        inputs = [units[u] if u in case["present"] else None for u in range(k + 1)]
        out = [oracle.xor_decode(inputs, case["erased"][0])]
    assert all(matches(b, x) for b, x in zip(case["outputs"], out))


def test_oracle_decode_not_invertible_and_too_few():
    with pytest.raises(ValueError):
        oracle.rs_decode(6, 3, [None] * 4 + [np.zeros(4, np.uint8)] * 5, [0, 1, 2, 3])
    m = np.array([[1, 2], [2, 4]], np.uint8)  # 2*row0 == row1 in GF(2^8)
    with pytest.raises(RuntimeError):
        oracle.invert_matrix(m)


def test_oracle_crc_golden():
    g = load("crc_vectors.json")
    assert g["check_123456789"] == {"crc32": 0xCBF43926, "crc32c": 0xE3069283}
    for c in g["cases"]:
        data = cells(c["seed"], c["stream"], 1, c["len"])[0]
        ctype = oracle.CRC32 if c["type"] == "crc32" else oracle.CRC32C
        assert [int(x) for x in oracle.crc_windows(ctype, data, c["bpc"])] == c["crcs"]


def test_window_count_reference_case():
    # TestChecksum.java:48-60: 55 bytes at bpc 10 -> ceil(55/10) = 6 checksums
    assert len(oracle.crc_windows(oracle.CRC32, np.arange(55, dtype=np.uint8), 10)) == 6


def test_golden_generator_is_reproducible():
    import make_golden
    assert make_golden.crc_vectors() == load("crc_vectors.json")
