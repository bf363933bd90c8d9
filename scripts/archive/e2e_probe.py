"""C5 pipeline probe: H2D rate from differently allocated host memory, and ozec_encode_crc_host_batch throughput
for each allocation and chunk size (one GPU)."""
import ctypes
import json
import mmap
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402
from ozone_amd.stripe_queue import host_alloc, host_register, host_unregister  # noqa: E402

MIB = 1 << 20
S = int(os.environ.get("S", "1024"))
k, p, n = 6, 3, MIB
sb = 9 * n
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)


def h2d_rate(addr, nbytes, reps=3):
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    src = torch.from_numpy(np.frombuffer((ctypes.c_uint8 * nbytes).from_address(addr), np.uint8))
    d.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        d.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return reps * nbytes / (time.perf_counter() - t0) / 1e9


def run_e2e(addr, crc_addr, chunk, reps=2):
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    f = lambda: e.encode_crc_host_batch(addr, sb, n, addr + k * n, sb, n, S, n, ck.ChecksumType.CRC32C, 16384,
                                        crc_addr, False, chunk)
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return reps * S * k * n / (time.perf_counter() - t0) / 1e9


res = {}
crc_bytes = S * 9 * 64 * 4
# 1) torch pinned (hipHostMalloc)
t = torch.empty(S * sb, dtype=torch.uint8).pin_memory()
tc = torch.empty(crc_bytes, dtype=torch.uint8).pin_memory()
res["hipHostMalloc_h2d"] = h2d_rate(t.data_ptr(), 64 * 6 * MIB)
for c in (8, 16, 32, 64):
    res[f"hipHostMalloc_e2e_c{c}"] = run_e2e(t.data_ptr(), tc.data_ptr(), c)
del t, tc
# 2) ozec_host_alloc (mmap + THP + mbind + hipHostRegister)
a = host_alloc(S * sb)
ac = host_alloc(crc_bytes)
res["ozec_host_alloc_h2d"] = h2d_rate(a.array.ctypes.data, 64 * 6 * MIB)
for c in (16, 64):
    res[f"ozec_host_alloc_e2e_c{c}"] = run_e2e(a.array.ctypes.data, ac.array.ctypes.data, c)
a.free()
ac.free()
# 3) shared /dev/shm mapping registered (bench.py's C5 batch)
path = f"/dev/shm/ozec_probe_{os.getpid()}"
fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)
os.ftruncate(fd, S * sb + crc_bytes)
mm = mmap.mmap(fd, S * sb + crc_bytes, mmap.MAP_SHARED)
os.close(fd)
os.unlink(path)
anchor = ctypes.c_char.from_buffer(mm)
base = ctypes.addressof(anchor)
t0 = time.perf_counter()
host_register(base, S * sb + crc_bytes, 0)
res["shm_register_s"] = time.perf_counter() - t0
res["shm_h2d"] = h2d_rate(base, 64 * 6 * MIB)
for c in (16, 64):
    res[f"shm_e2e_c{c}"] = run_e2e(base, base + S * sb, c)
host_unregister(base)
# 4) shm with MADV_HUGEPAGE before the touch
path = f"/dev/shm/ozec_probe2_{os.getpid()}"
fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)
os.ftruncate(fd, S * sb + crc_bytes)
mm2 = mmap.mmap(fd, S * sb + crc_bytes, mmap.MAP_SHARED)
os.close(fd)
os.unlink(path)
anchor2 = ctypes.c_char.from_buffer(mm2)
base2 = ctypes.addressof(anchor2)
try:
    mm2.madvise(mmap.MADV_HUGEPAGE)
    res["shm_thp_madvise"] = True
except (AttributeError, OSError) as ex:
    res["shm_thp_madvise"] = repr(ex)
t0 = time.perf_counter()
host_register(base2, S * sb + crc_bytes, 0)
res["shm_thp_register_s"] = time.perf_counter() - t0
res["shm_thp_h2d"] = h2d_rate(base2, 64 * 6 * MIB)
res["shm_thp_e2e_c16"] = run_e2e(base2, base2 + S * sb, 16)
host_unregister(base2)
try:
    res["thp_shmem_enabled"] = open("/sys/kernel/mm/transparent_hugepage/shmem_enabled").read().strip()
    res["thp_enabled"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
except OSError:
    pass
print(json.dumps({k_: (round(v, 2) if isinstance(v, float) else v) for k_, v in res.items()}))
