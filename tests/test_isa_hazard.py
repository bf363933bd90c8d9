"""CPU test: the shipped gfx950 code object has no wide VMEM store whose data VGPRs a VALU op rewrites within 2
wait states (the store-data hazard of DESIGN §2.3a).  The scanner itself is checked on a positive and a negative
control compiled from tests/native/store_hazard.hip."""
import os
import subprocess
import tempfile

import pytest

import isa_scan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ozone_amd", "lib", "libozec.so")


def test_scanner_flags_the_pattern_and_accepts_the_hold():
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "k.co")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only",
                        "--no-gpu-bundle-output", "-c", "-o", co, os.path.join(ROOT, "tests", "native", "store_hazard.hip")],
                       check=True, capture_output=True, timeout=300)
        bad = isa_scan.scan(isa_scan.disassemble_code_object(co))
    funcs = {b[0] for b in bad}
    assert any("store_then_rewrite" in f for f in funcs), bad
    assert not any("store_hold_rewrite" in f for f in funcs), bad


@pytest.mark.skipif(not os.path.exists(LIB), reason="libozec.so not built")
def test_shipped_kernels_have_no_store_data_hazard():
    text = isa_scan.disassemble_shared_object(LIB)
    assert text.count("store_dwordx4") > 100  # the scan saw the kernels
    bad = isa_scan.scan(text)
    assert not bad, "\n".join(f"{f}: {s}  ->  {w} after {ws} wait states" for f, s, w, ws in bad)
