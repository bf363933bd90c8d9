import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: large-size property tests")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _fused_kernels_in_gpu_tests(request):
    """GPU tests run the fused kernels at every batch size: libozec's default sends batches of 16-B cells below
    fused_min_units (stripe x window units) to the unfused kernels, which would take the small parity batches away
    from the fused kernels and variants they are written for.  tests/test_gpu_bytes.py covers both routes.
    OZEC_TEST_PRODUCTION_ROUTING=1 keeps libozec's own routing instead (a whole-suite run of the production defaults)."""
    if request.node.get_closest_marker("gpu") is None or os.environ.get("OZEC_TEST_PRODUCTION_ROUTING") == "1":
        yield
        return
    from ozone_amd import _lib as L
    lib = L.lib()
    import ctypes
    prev = ctypes.c_int64(0)
    assert lib.ozec_get_tuning(b"fused_min_units", ctypes.byref(prev)) == 0
    assert lib.ozec_set_tuning(b"fused_min_units", 0) == 0
    try:
        yield
    finally:
        lib.ozec_set_tuning(b"fused_min_units", prev.value)


@pytest.fixture(autouse=True)
def _device_fault_check(request):
    """A GPU memory fault is reported asynchronously (the runtime learns of it from an interrupt after the faulting
    work has completed) and then fails whatever HIP call comes next, often in a later test.  Every GPU test ends with a
    device-wide synchronise after a short grace period, so a fault is charged to the test whose work raised it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import time
    import torch
    if not torch.cuda.is_initialized():
        return
    torch.cuda.synchronize()
    time.sleep(0.002)
    torch.cuda.synchronize()
