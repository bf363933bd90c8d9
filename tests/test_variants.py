"""The kernel alternates the shipped libozec.so lets a caller select (ozec_set_tuning "gf_variant" / "crc_variant") are
exactly the ones the GPU parity tests sweep (tests/variants.py), probe ids of earlier rounds are rejected, and the
other tuning knobs reject out-of-range values.  CPU only: setting a knob touches no GPU."""
import ctypes
import re
from pathlib import Path

import pytest

import variants
from ozone_amd import _lib as L

ROOT = Path(__file__).resolve().parent.parent


def _listed(key):
    lib = L.lib()
    n = lib.ozec_tuning_variants(key, None, 0)
    assert n > 0
    buf = (ctypes.c_int * n)()
    assert lib.ozec_tuning_variants(key, buf, n) == n
    return sorted(buf)


def test_library_variants_are_the_parity_tested_ones():
    assert _listed(b"gf_variant") == sorted(variants.GF)
    assert _listed(b"crc_variant") == variants.CRC


def test_every_variant_family_is_swept_by_a_gpu_test():
    """Each family list of tests/variants.py parametrizes at least one GPU parity test."""
    src = "".join(p.read_text() for p in (ROOT / "tests").glob("test_gpu_*.py"))
    for fam in ("GF", "CRC_STREAM", "XOR_FUSED", "RS_FUSED", "NB_PERSISTENT"):
        assert re.search(r"parametrize\(\"variant\",[^)]*variants\." + fam + r"\b", src), fam


@pytest.mark.parametrize("v", list(range(140, 150)) + [1, 11, 12, 13, 17, 23, 51, 61, 100, 151, 175, 178, 185, 186, 188, 195, 197, 199, 200, 202, 203, 210, 211, 212, 213, 230, 232, 233, 999, -1])
def test_removed_and_unknown_crc_variants_rejected(v):
    lib = L.lib()
    assert lib.ozec_set_tuning(b"crc_variant", v) == L.OZEC_EINVAL
    assert b"crc_variant" in lib.ozec_last_error()


@pytest.mark.parametrize("v", [2, 3, 4, 6, 7, 12, 13, 99])
def test_removed_gf_variants_rejected(v):
    assert L.lib().ozec_set_tuning(b"gf_variant", v) == L.OZEC_EINVAL


def test_listed_variants_accepted_and_reset():
    lib = L.lib()
    try:
        for v in variants.CRC:
            assert lib.ozec_set_tuning(b"crc_variant", v) == 0
        for v in variants.GF:
            assert lib.ozec_set_tuning(b"gf_variant", v) == 0
    finally:
        assert lib.ozec_set_tuning(b"crc_variant", 0) == 0
        assert lib.ozec_set_tuning(b"gf_variant", 0) == 0


@pytest.mark.parametrize("key,bad,good", [(b"copy_stream", 4, 2), (b"copy_stream", -2, 3), (b"unit_map", 2, 1),
                                          (b"e2e_rect", 5, 1), (b"host_chunk", 0, 4 << 20), (b"host_slots", 0, 8),
                                          (b"queue_batches", 65, 0), (b"crc_grid", -1, 0), (b"host_graph", -1, 256 << 10),
                                          (b"host_duplex", -1, 0), (b"fused_min_units", -1, 1024),
                                          (b"rec_min_units", -1, 0), (b"nb_small_units", -1, 16384),
                                          (b"host_pitch16", 2, 0)])
def test_knob_ranges(key, bad, good):
    lib = L.lib()
    assert lib.ozec_set_tuning(key, bad) == L.OZEC_EINVAL
    assert lib.ozec_set_tuning(key, good) == 0


def test_copy_stream_modes_reach_the_pool():
    """copy_stream 2 and 3 are stored as given (they used to be clamped to 1); -1 restores the automatic choice."""
    lib = L.lib()
    try:
        for m in (0, 1, 2, 3):
            assert lib.ozec_set_tuning(b"copy_stream", m) == 0
    finally:
        assert lib.ozec_set_tuning(b"copy_stream", -1) == 0
