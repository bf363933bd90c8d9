"""The C ABI's host code (capi.cpp, stripe_queue.cpp, the staging copy pool, GF and CRC setup) under AddressSanitizer
and UBSan: `make asan-host` instruments the host translation units of libozec (the kernel objects of the regular
build are linked unchanged), and the CPU tests that drive the C ABI through ctypes -- argument validation, decode
matrices, CRC combine / composer, the JNI marshaling core and glue, the stripe-queue argument checks -- run against
it with the ASan runtime preloaded.  It caught a memcpy from an empty vector (null source) in
ozec_rs_decode_matrix with zero erasures.  CPU only; the GPU paths are checked bit-exactly on the GPU."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNTIME = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

pytestmark = pytest.mark.skipif(
    not RUNTIME or not os.path.exists(os.path.join(ROOT, "build", "obj", "kernels.o")),
    reason="needs the ROCm clang ASan runtime and a regular build (build/obj/kernels.o)")


def test_c_abi_host_tests_under_asan(tmp_path):
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "ozone_amd", "csrc"), "asan-host", "ARCH=gfx950"],
                   check=True, capture_output=True)
    log = str(tmp_path / "asan")
    r = subprocess.run([os.path.join(ROOT, "scripts", "asan_host_tests.sh")], capture_output=True, text=True,
                       timeout=900, env=dict(os.environ, ASAN_LOG=log))
    reports = "".join(open(f).read() for f in glob.glob(log + "*"))
    assert r.returncode == 0 and not reports, (r.stdout[-3000:] + r.stderr[-2000:] + reports[-6000:])
    assert " passed" in r.stdout
