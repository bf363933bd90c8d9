"""G26 CRC tables and bit-group map, checked on the CPU (no GPU): tests/native/g26_emulate.cpp runs the device
algorithm of kernels.hip crc_windows_g26 / g26_block on the host, on the table blobs libozec uploads, and compares
every window with the byte-wise CRC32 / CRC32C register (the CrcIntTable arithmetic, CM/ChecksumByteBuffer.java)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ozone_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_g26_host_emulation(tmp_path):
    exe = tmp_path / "g26_emulate"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", CSRC, "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                           "-o", str(exe), os.path.join(ROOT, "tests", "native", "g26_emulate.cpp"),
                           os.path.join(CSRC, "crc_host.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bit-exact" in out.stdout and "XO:" in out.stdout and "G5 re-check:" in out.stdout
