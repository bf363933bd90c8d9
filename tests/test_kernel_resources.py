"""The default kernels of the shipped libozec.so use no scratch memory and spill no VGPRs (CPU test: reads the gfx950
code objects' metadata notes, scripts/kernel_resources.py).  Alternates may spill; the defaults the launchers pick
(fused.hip launch_encode_crc_lv, kernels.hip gf_code_vec launch) must not, and must fit the CU's 160 KiB of LDS."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "ozone_amd", "lib", "libozec.so")
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _i(v):
    return f"Li{v}E"


def _b(v):
    return f"Lb{int(v)}E"


def _nb(K, R, D, NB, WPB, DYN, H, tail, cv=False, wide=False):
    """Mangled template-argument list of encode_crc_nb<K, R, D, NB, WPB, 4, 2, true, DYN, XO, EM, H, TAIL, CV, WIDE>
    (XO, EM on), closed, so that it names exactly one instantiation."""
    return "encode_crc_nbI" + "".join([_i(K), _i(R), _i(D), _i(NB), _i(WPB), _i(4), _i(2), _b(1), _i(DYN), _b(1),
                                       _b(1), _i(H), _b(tail), _b(cv), _b(wide)]) + "EEvN"


def _defaults():
    """fused.hip: rs-10-x 177 (queue) / 173, rs-6-x 171 / 174, rs-3-x 172 / 174 (fused_nb.hpp launch_nb_kr), x = 1-4;
    their byte-tail instantiations; 231 for verifying reconstructions."""
    out = []
    for t in (False, True):  # 16-B cells, and the byte-tail (TAIL) instantiation of the same variant
        out += [_nb(10, R, 2, 5, 16, 1, 5, t) for R in (1, 2, 3, 4)]     # 177
        out += [_nb(10, R, 1, 5, 8, 0, 10, t) for R in (1, 2, 3, 4)]    # 173
        out += [_nb(6, R, 2, 3, 16, 1, 6, t) for R in (1, 2, 3)]   # 171
        out += [_nb(6, R, 2, 2, 12, 0, 6, t) for R in (1, 2, 3)]   # 174 (kD2 = 2 for K = 6)
        out += [_nb(3, R, 2, 2, 16, 1, 3, t) for R in (1, 2)] + [_nb(3, R, 2, 2, 12, 0, 3, t) for R in (1, 2)]
    # 231: the combined-verify reconstruction default for rs-10-x and rs-6-x
    out += [_nb(10, R, 1, 5, 16, 1, 10, False, True) for R in (1, 2, 3, 4)]
    out += [_nb(6, R, 1, 3, 16, 1, 6, False, True) for R in (1, 2, 3)]
    # round 6: units 2 GiB or more apart (WIDE, one descriptor per unit), 16-B cells and byte tails
    for t in (False, True):
        out += [_nb(10, R, 1, 5, 8, 0, 10, t, False, True) for R in (1, 2, 3, 4)]
        out += [_nb(6, R, 1, 3, 8, 0, 6, t, False, True) for R in (1, 2, 3)]
        out += [_nb(3, R, 1, 3, 8, 0, 3, t, False, True) for R in (1, 2)]
    return out


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(SO):
        pytest.skip("libozec.so not built")
    import kernel_resources
    return kernel_resources.kernels(SO)


@pytest.mark.parametrize("pat", _defaults())
def test_fused_defaults_no_scratch(kernels, pat):
    found = [k for k in kernels if pat in k["name"]]
    assert found, f"default kernel {pat} not in libozec.so"
    for k in found:
        assert k.get("private_segment_fixed_size") == 0, k
        assert k.get("vgpr_spill_count") == 0, k
        assert k.get("group_segment_fixed_size", 0) <= 160 * 1024, k


@pytest.mark.parametrize("K,R", [(6, 3), (3, 2), (10, 4), (6, 2), (10, 1), (10, 3)])
def test_coding_kernel_defaults_no_scratch(kernels, K, R):
    """gf_code_vec<K, R, K * R <= 18, 1, 2, 2, 0>: the coding kernel of C1-C3 (one vector per thread; coefficient
    tables in SGPRs up to 18 coefficients, kernels.hip launch_krv)."""
    pat = "gf_code_vecI" + "".join([_i(K), _i(R), _b(K * R <= 18), _i(1), _i(2), _i(2), _i(0), _b(0)]) + "EEvN"
    found = [k for k in kernels if pat in k["name"]]
    assert found, pat
    for k in found:
        assert k.get("private_segment_fixed_size") == 0 and k.get("vgpr_spill_count") == 0, k


@pytest.mark.parametrize("K,R", [(3, 1), (3, 2), (6, 1), (6, 2), (6, 3), (10, 1)])
def test_wide_coding_kernels_no_scratch(kernels, K, R):
    """gf_code_vec<K, R, false, 1, 2, 2, 0, WIDE>: one descriptor per unit for units 2 GiB or more apart, instantiated
    up to 18 coefficients (kernels.hip kWideMaxKR; rs-10-2..4 spilled in that form and are not instantiated)."""
    pat = "gf_code_vecI" + "".join([_i(K), _i(R), _b(0), _i(1), _i(2), _i(2), _i(0), _b(1)]) + "EEvN"
    found = [k for k in kernels if pat in k["name"]]
    assert found, pat
    for k in found:
        assert k.get("private_segment_fixed_size") == 0 and k.get("vgpr_spill_count") == 0, k
    assert not [k for k in kernels if "gf_code_vecI" + _i(10) + _i(4) in k["name"] and k["name"].endswith(
        _b(1) + "EEvNS_8CodeArgsENS0_7TabArgsIXmlT_T0_EEE")], "rs-10-4 WIDE instantiated"
