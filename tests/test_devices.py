"""The device list and device policies of one drop-in process (ozone_amd/csrc/devices.cpp) on the
CPU: devices.cpp compiled against a fake HIP runtime of four devices on two NUMA nodes (tests/native/
devices_policy.cpp) -- default list, OZEC_DEVICES, duplicates, bad ordinals, round robin, NUMA-first, "current",
per-thread devices re-picked after a list change, DeviceScope restoring the caller's device."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary():
    d = tempfile.mkdtemp(prefix="ozec_devices_")
    exe = os.path.join(d, "devices_policy")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-I", ROOT, os.path.join(ROOT, "tests", "native", "devices_policy.cpp"),
                        os.path.join(ROOT, "ozone_amd", "csrc", "devices.cpp"), "-o", exe, "-lpthread"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail(r.stderr[-2000:])
    return exe


@pytest.mark.parametrize("env", [None, "3,x,1,9"])
def test_device_policies(binary, env):
    e = dict(os.environ)
    e.pop("OZEC_DEVICES", None)
    e.pop("OZEC_DEVICE_POLICY", None)
    if env:
        e["OZEC_DEVICES"] = env
    r = subprocess.run([binary], capture_output=True, text=True, timeout=60, env=e)
    assert r.returncode == 0, r.stderr
    assert "devices policy OK" in r.stdout


@pytest.mark.parametrize("S,chunk,ndev", [(8192, 32, 8), (8192, 32, 1), (8192, 32, 3), (100, 32, 8), (31, 32, 4),
                                          (4097, 32, 8), (8192, 0, 5), (257, 16, 7)])
def test_host_batch_partition_matches_the_bench_ranks(binary, S, chunk, ndev):
    """bench.py's in-process C5 leg registers rank r's range = shard.stripe_range(S, r, N) and
    relies on libozec splitting the same batch over N devices into exactly those ranges (devices.cpp split_parts /
    part_range, used by capi.cpp host_batch_split); fewer parts when the batch has fewer whole chunks than devices."""
    from ozone_amd.shard import stripe_range
    r = subprocess.run([binary, "parts", str(S), str(chunk), str(ndev)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    got = [tuple(map(int, line.split())) for line in r.stdout.splitlines()]
    parts = max(1, min(ndev, S // max(1, chunk)))
    assert got == [stripe_range(S, i, parts) for i in range(parts)]
    assert got[0][0] == 0 and got[-1][1] == S
