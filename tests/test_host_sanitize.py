"""libozec's host code under the sanitizers (race detection / sanitizers): the GF(2^8) setup
(gf256.cpp), the CRC table / shift / combine math (crc_host.cpp) and the parallel staging copy (copy_pool.cpp),
built with g++ -fsanitize=address,undefined and -fsanitize=thread around tests/native/host_sanitize.cpp, which
checks them against the C oracle (every erasure pattern of rs-3-2 / rs-6-3 / rs-10-4 and wider schemas, in both
caller orders).  CPU only: the kernels are checked bit-exactly on the GPU instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ozone_amd", "csrc")
ROCM = "/opt/rocm"

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir(os.path.join(ROCM, "include", "hip")),
                                reason="needs g++ and the HIP headers")


def _build(tmp_path, name, sanitize):
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"]
    if sanitize != "thread":
        flags.append("-fno-sanitize-recover=all")
    obj = tmp_path / f"oracle_{name}.o"
    subprocess.run(["gcc", *flags, "-std=gnu11", "-c", os.path.join(ROOT, "oracle", "ozec_oracle.c"), "-o", str(obj)],
                   check=True)
    exe = tmp_path / name
    subprocess.run(["g++", *flags, "-std=c++17", f"-I{SRC}", f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__",
                    os.path.join(ROOT, "tests", "native", "host_sanitize.cpp"),
                    *(os.path.join(SRC, f) for f in ("gf256.cpp", "crc_host.cpp", "copy_pool.cpp", "numa.cpp")),
                    str(obj), "-o", str(exe), f"-L{ROCM}/lib", "-lamdhip64", "-lpthread", f"-Wl,-rpath,{ROCM}/lib"],
                   check=True)
    return exe


def _run(exe, mode, env_key, env_val):
    env = dict(os.environ, **{env_key: env_val})
    r = subprocess.run([str(exe), mode], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "ok" in r.stdout, r.stdout
    return r.stdout


def test_host_math_and_copy_under_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "hs_asan", "address,undefined")
    out = _run(exe, "math", "ASAN_OPTIONS", "detect_leaks=1:halt_on_error=1")
    assert "decode patterns" in out
    _run(exe, "copy", "ASAN_OPTIONS", "detect_leaks=1:halt_on_error=1")


def test_copy_pool_under_tsan(tmp_path):
    exe = _build(tmp_path, "hs_tsan", "thread")
    _run(exe, "copy", "TSAN_OPTIONS", "halt_on_error=1")
