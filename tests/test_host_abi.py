"""libozec.so on the CPU: it loads, exports every symbol include/ozec.h declares, and its host-side coding
math (matrices, inversion, config parsing, CRC combine) equals the oracle.  No compute call needs a GPU here."""
import ctypes
import subprocess

import numpy as np
import pytest

import oracle
from golden_io import ec_cases
from ozone_amd import _lib as L
from ozone_amd import rawcoder as rc
from synth import SEED, cells


def test_library_loads_and_exports_header_symbols():
    lib = L.lib()
    syms = L.header_symbols()
    assert len(syms) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:
        assert hasattr(lib, s)
    assert lib.ozec_version() >= 1


def test_library_is_gfx950_code_object():
    data = open(L.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle id of the embedded code object


@pytest.mark.parametrize("k,p", [(3, 2), (6, 3), (10, 4), (1, 1), (12, 4), (200, 55)])
def test_encode_matrix_vs_oracle(k, p):
    assert (rc.rs_encode_matrix(k, p) == oracle.cauchy_matrix(k, p)).all()


def test_encode_matrix_rejects_256_units():
    with pytest.raises(rc.HadoopIllegalArgumentException):
        rc.rs_encode_matrix(200, 56)


@pytest.mark.parametrize("case", [c for c in ec_cases("decode") if c["codec"] == "rs" and c["len"] == 1007],
                         ids=lambda c: f"rs{c['k']}-{c['p']}-e{'_'.join(map(str, c['erased']))}")
def test_decode_matrix_vs_golden(case):
    dm = rc.rs_decode_matrix(case["k"], case["p"], case["present"], case["erased"])
    assert [bytes(r).hex() for r in dm] == case["decode_matrix"]


def test_decode_matrix_random_patterns_vs_oracle():
    rng = np.random.default_rng(5)
    for _ in range(200):
        k = int(rng.integers(1, 14))
        p = int(rng.integers(1, 6))
        n_er = int(rng.integers(0, p + 1))
        erased = [int(x) for x in rng.choice(k + p, n_er, replace=False)]  # any order, incl. the quirk
        alive = sorted(set(range(k + p)) - set(erased))
        valid = alive[:k]
        assert (rc.rs_decode_matrix(k, p, valid, erased) == oracle.rs_decode_matrix(k, p, valid, erased)).all()


def test_gf_invert_matrix_vs_oracle_and_singular():
    rng = np.random.default_rng(9)
    for n in (1, 2, 3, 6, 10):
        m = oracle.cauchy_matrix(n, n)[n:]  # Cauchy blocks are invertible
        assert (rc.gf_invert_matrix(m) == oracle.invert_matrix(m)).all()
    m = rng.integers(0, 256, (5, 5), dtype=np.uint8)
    m[:, 0] = 0
    with pytest.raises(rc.NotInvertibleException):
        rc.gf_invert_matrix(m)


def test_gf_mul_all_pairs():
    for a in range(256):
        for b in range(0, 256, 3):
            assert rc.gf_mul(a, b) == oracle.gf_mul(a, b)


@pytest.mark.parametrize("s,expect", [
    ("rs-3-2-1024k", ("rs", 3, 2, 1 << 20)), ("RS-6-3-2048", ("rs", 6, 3, 2048)),
    ("XOR-10-4-4096K", ("xor", 10, 4, 4 << 20)), ("rs-10-4-1024k", ("rs", 10, 4, 1 << 20))])
def test_parse_replication(s, expect):
    c = rc.ECReplicationConfig(s)
    assert (c.get_codec(), c.get_data(), c.get_parity(), c.get_ec_chunk_size()) == expect


@pytest.mark.parametrize("s", ["rs-3-2", "foo-3-2-1024k", "rs-0-2-1024k", "rs-3-0-1024k", "rs-3-2-0k", "rs-3-2-1024m"])
def test_parse_replication_rejects(s):
    with pytest.raises(rc.IllegalArgumentException):
        rc.ECReplicationConfig(s)


@pytest.mark.parametrize("ctype,otype", [(L.OZEC_CHECKSUM_CRC32, oracle.CRC32), (L.OZEC_CHECKSUM_CRC32C, oracle.CRC32C)])
def test_crc_combine_vs_oracle(ctype, otype):
    d = cells(SEED, 4242, 1, 70000)[0]
    for cut in (0, 1, 17, 4096, 69999, 70000):
        a, b = d[:cut], d[cut:]
        got = L.lib().ozec_crc_combine(ctype, oracle.crc(otype, a), oracle.crc(otype, b), b.size)
        assert got == oracle.crc(otype, d)


def test_coder_construction_without_gpu_fails_loudly():
    """No CPU fallback: with no device the factory throws, so CodecUtil falls through (CodecUtil.java:62-78)."""
    if L.lib().ozec_device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        rc.RawErasureEncoder(rc.ECReplicationConfig(6, 3))
    with pytest.raises(rc.IllegalArgumentException, match="Fail to create raw erasure encoder"):
        rc.CodecUtil.create_raw_encoder_with_fallback(rc.ECReplicationConfig(6, 3))


def test_registry_names():
    reg = rc.CodecRegistry.get_instance()
    assert reg.get_codec_names() == ["rs", "xor"]
    assert reg.get_coder_names("rs") == ["rs_hip"]
    assert reg.get_coder_names("xor") == ["xor_hip"]
    assert reg.get_coder_by_name("rs", "rs_hip").get_codec_name() == "rs"
    reg.update_coders([rc.HipRSRawErasureCoderFactory()])  # duplicate names are ignored
    assert reg.get_coder_names("rs") == ["rs_hip"]


def test_last_error_is_thread_local_message():
    out = ctypes.c_void_p()
    assert L.lib().ozec_encoder_create(7, 3, 2, ctypes.byref(out)) == L.OZEC_EINVAL
    assert "codec" in L.last_error()


def test_per_call_counters_record_calls_bytes_and_failures():
    """ozec_stats (SURVEY §5 metrics): every entry-point family counts calls, data bytes of successful calls,
    failures and host time; nested calls count once (the outermost)."""
    import ctypes
    from ozone_amd import _lib
    L = _lib.lib()
    _lib.stats_reset()
    assert all(v == {"calls": 0, "bytes": 0, "errors": 0, "host_ns": 0} for v in _lib.stats().values())
    out = (ctypes.c_uint32 * 4)()
    data = (ctypes.c_uint8 * 64)()
    assert L.ozec_checksum_windows(3, data, 64, 0, out, 0) == _lib.OZEC_EINVAL  # bpc 0: fails before the device
    st = ctypes.c_uint32(0xFFFFFFFF)
    assert L.ozec_crc_update(3, ctypes.byref(st), data, 0) == 0                # empty update: succeeds
    s = _lib.stats()["checksum"]
    assert s["calls"] == 2 and s["errors"] == 1 and s["bytes"] == 0 and s["host_ns"] > 0
    assert L.ozec_encode(None, None, None, 4096) == _lib.OZEC_EINVAL
    assert _lib.stats()["encode"]["errors"] == 1
    with pytest.raises(Exception):
        _lib.check(L.ozec_stats(99, None))
    _lib.stats_reset()
