"""C5 probe 2: shm batch of S stripes registered, e2e throughput per chunk size, with and without binding the
process to the GPU's NUMA node, and the time of each of several consecutive steps."""
import ctypes, json, mmap, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402
from ozone_amd.stripe_queue import host_register, host_unregister, device_numa_node  # noqa: E402

MIB = 1 << 20
S = int(os.environ.get("S", "8192"))
k, p, n = 6, 3, MIB
sb = 9 * n
torch.cuda.set_device(0)
res = {"S": S, "node": device_numa_node(0)}
if os.environ.get("BIND") == "1":
    cpus = set()
    for part in open(f"/sys/devices/system/node/node{res['node']}/cpulist").read().strip().split(","):
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    os.sched_setaffinity(0, cpus & os.sched_getaffinity(0))
    res["bound"] = True
crc_bytes = S * 9 * 64 * 4
path = f"/dev/shm/ozec_probe_{os.getpid()}"
fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)
os.ftruncate(fd, S * sb + crc_bytes)
mm = mmap.mmap(fd, S * sb + crc_bytes, mmap.MAP_SHARED)
os.close(fd)
os.unlink(path)
anchor = ctypes.c_char.from_buffer(mm)
base = ctypes.addressof(anchor)
t0 = time.perf_counter()
host_register(base, S * sb + crc_bytes, int(os.environ.get("REGDEV", "0")))
res["register_s"] = round(time.perf_counter() - t0, 2)
e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
from ozone_amd import _lib  # noqa: E402
res["rect"] = int(os.environ.get("RECT", "0"))
assert _lib.lib().ozec_set_tuning(b"e2e_rect", res["rect"]) == 0
for c in [int(x) for x in os.environ.get("CHUNKS", "16,64").split(",")]:
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        e.encode_crc_host_batch(base, sb, n, base + k * n, sb, n, S, n, ck.ChecksumType.CRC32C, 16384, base + S * sb,
                                False, c)
        ts.append(round(S * k * n / (time.perf_counter() - t0) / 1e9, 2))
    res[f"e2e_c{c}_GBps"] = ts
host_unregister(base)
print(json.dumps(res))
