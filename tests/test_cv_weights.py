"""The weights of the combined input verification (fused_nb.hpp CV variants, kernels.hpp kCv*) separate every pair
of inputs (CPU test).

The CV kernel checks XOR_j x^(8 w_j) raw_j against the same combination of the stored CRCs, w_j = j * kCvStride
bytes (mod P, the CRC polynomial).  An error pattern in unit j changes raw_j by its CRC delta D_j (nonzero for every
error the per-unit check would catch), so the combined check misses a corruption only if XOR_j x^(8 w_j) D_j = 0:
  * one unit: x is a unit mod P (P(0) = 1), so x^(8 w_j) D_j != 0 -- always caught;
  * two units with the SAME error pattern (D_a = D_b = D, e.g. the same bytes flipped at the same offsets):
    (x^(8 w_a) + x^(8 w_b)) D = x^(8 w_a) (1 + x^(8 (w_b - w_a))) D, zero only if 1 + x^(8 (w_b - w_a)) shares a
    factor with P.  CRC-32: gcd(1 + x^(8 kCvStride d), P) = 1 for every d = 1..15 (this test), so such a pair is
    always caught.  CRC-32C: its polynomial is (x + 1) Q with Q of degree 31 (even number of terms), and x + 1
    divides every 1 + x^m; the test shows the gcd is exactly x + 1, so the pair cancels only for the one nonzero
    delta D = Q -- an odd-weight error pattern that is a multiple of Q, the same kind of pattern (a multiple of a
    degree-31/32 polynomial) that the per-unit CRC itself misses, and as rare.
Anything else needs D's that cancel under the weights, as likely as a collision of the CRC itself (2^-32).  A stripe
whose combination fails is re-checked unit by unit on the GPU (nb_reverify), so the reported first failure is the
reference's (ChecksumData.java:118-150).
"""
import re
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# CRC-32 (IEEE, ChecksumByteBuffer CRC32) and CRC-32C (Castagnoli) in normal (non-reflected) form, x^32 included
POLYS = {"CRC32": 0x104C11DB7, "CRC32C": 0x11EDC6F41}


def _hdr_int(name):
    text = open(os.path.join(ROOT, "ozone_amd", "csrc", "kernels.hpp")).read()
    return int(re.search(rf"constexpr int {name} = (\d+);", text).group(1))


def _mod(a, p):
    dp = p.bit_length() - 1
    while a and a.bit_length() - 1 >= dp:
        a ^= p << (a.bit_length() - 1 - dp)
    return a


def _mulmod(a, b, p):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a = _mod(a << 1, p)
    return _mod(r, p)


def _xpow(m, p):
    r, base = 1, 2
    while m:
        if m & 1:
            r = _mulmod(r, base, p)
        base = _mulmod(base, base, p)
        m >>= 1
    return r


def _gcd(a, b):
    while b:
        a, b = b, _mod(a, b)
    return a


@pytest.mark.parametrize("crc", sorted(POLYS))
def test_weight_differences_are_units_mod_p(crc):
    p = POLYS[crc]
    stride, kmax = _hdr_int("kCvStride"), _hdr_int("kCvMaxK")
    x_plus_1_divides_p = bin(p).count("1") % 2 == 0
    assert x_plus_1_divides_p == (crc == "CRC32C")
    for d in range(1, kmax):
        f = _xpow(8 * stride * d, p) ^ 1  # 1 + x^(8 stride d), reduced mod P
        assert f != 0 and _gcd(p, f) == (0b11 if x_plus_1_divides_p else 1), (crc, d)


def test_gf2_helpers():
    p = POLYS["CRC32"]
    assert _xpow(32, p) == p ^ (1 << 32)          # x^32 = P - x^32
    assert _gcd(p, 1) == 1 and _gcd(0b110, 0b11) == 0b11  # x^2 + x = x (x + 1)


@pytest.mark.parametrize("crc", sorted(POLYS))
def test_run_check_window_distances(crc):
    """The streaming verify kernel's run check (kernels.hip crc_windows_g26s VR) weights window w of a run by
    x^(8 bpc (m - 1 - w)); two windows k apart with the same error pattern cancel only if 1 + x^(8 bpc k) shares a
    factor with P: none for CRC-32, only x + 1 for CRC-32C (then only the one delta D = P / (x + 1)), for every bpc the
    check runs with (4 KiB << i, i < kBshiftN) and runs of up to 256 windows."""
    p = POLYS[crc]
    want = 0b11 if crc == "CRC32C" else 1
    for i in range(_hdr_int("kBshiftN")):
        bpc = 4096 << i
        for k in range(1, 256):
            f = _xpow(8 * bpc * k, p) ^ 1
            assert f != 0 and _gcd(p, f) == want, (crc, bpc, k)
