"""libozec's pinned blocks (ozone_amd/csrc/numa.cpp pinned_alloc / pinned_free) on the CPU, against a fake HIP runtime
that counts registrations (tests/native/pinned_cache.cpp), under TSan: a freed block is unregistered and its pages
returned at once, its address range is retired (PROT_NONE, never reused for a later block, bounded); a refused
unregistration leaves the block untouched and is counted; foreign / double frees are refused; concurrent cycles never
share a block.  Why: DESIGN.md §4, "GPU faults"."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary():
    d = tempfile.mkdtemp(prefix="ozec_pinned_cache_")
    exe = os.path.join(d, "pinned_cache")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Werror", "-fsanitize=thread",
                        "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", ROOT,
                        os.path.join(ROOT, "tests", "native", "pinned_cache.cpp"),
                        os.path.join(ROOT, "ozone_amd", "csrc", "numa.cpp"), "-o", exe, "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail(r.stderr[-3000:])
    return exe


def test_pinned_block_cache(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "pinned blocks OK" in r.stdout
