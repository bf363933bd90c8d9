"""The WorkQueue counter-slot pool of the persistent fused kernels (ozone_amd/csrc/work_slots.cpp; ADVICE r3: slots
must not be keyed by stream handle) on the CPU, against a fake HIP runtime whose events complete on demand
(tests/native/work_slots.cpp): no slot is leased twice while its last kernel (or its zeroing) may still run."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary():
    d = tempfile.mkdtemp(prefix="ozec_work_slots_")
    exe = os.path.join(d, "work_slots")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Werror", "-fsanitize=thread",
                        "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", ROOT,
                        os.path.join(ROOT, "tests", "native", "work_slots.cpp"),
                        os.path.join(ROOT, "ozone_amd", "csrc", "work_slots.cpp"), "-o", exe, "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail(r.stderr[-3000:])
    return exe


def test_work_slot_pool(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "work slots OK" in r.stdout
