"""Interleaved A/B of the CRC / fused encode+CRC kernel variants and grids in one process."""
import itertools, json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ozone_amd import _lib as L
from ozone_amd import checksum as ck
from ozone_amd import rawcoder as rc
torch.cuda.set_device(0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n, bpc = 1 << 20, 16384
lib = L.lib()
steps = {}
# fused rs-6-3 + CRC32C, 4096 stripes
k, p, S = 6, 3, 4096
U = torch.empty((S, k + p, n), dtype=torch.uint8, device="cuda")
for u in range(k):
    rc.fill_splitmix64_cells(U[:, u], (k + p) * n, S, n, 1, u * S)
crcs = torch.empty((S, k + p, n // bpc), dtype=torch.int32, device="cuda")
e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
st = (k + p) * n
steps["c5"] = (lambda: e.encode_crc_batch(U, st, n, U[:, k:], st, n, S, n, ck.ChecksumType.CRC32C, bpc, crcs), S * 9 * n)
# crc only over the 4096 x 6 data cells (as one 24 GiB batch of cells)
crc2 = torch.empty((S * k, n // bpc), dtype=torch.int32, device="cuda")
D = U[:, :k]
steps["crc"] = (lambda: [ck.checksum_windows_batch(ck.ChecksumType.CRC32C, U[:, j], st, S, n, bpc, crc2[j * S:]) for j in range(k)], S * k * n)
variants = [int(v) for v in os.environ.get("VARIANTS", "0,3,4").split(",")]
grids = [int(g) for g in os.environ.get("GRIDS", "0,4096,8192,16384,1000000").split(",")]
configs = list(itertools.product(steps, variants, grids))
times = {c: [] for c in configs}
for r in range(rounds):
    for c in configs:
        lib.ozec_set_tuning(b"crc_variant", c[1]); lib.ozec_set_tuning(b"crc_grid", c[2])
        fn, alg = steps[c[0]]
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); fn(); b.record(); torch.cuda.synchronize()
        times[c].append(a.elapsed_time(b) / 2)
for c in sorted(configs, key=lambda c: (c[0], np.median(times[c]))):
    med = float(np.median(times[c]))
    print(json.dumps({"wl": c[0], "variant": c[1], "grid": c[2], "median_ms": round(med, 3),
                      "frac": round(steps[c[0]][1] / (med * 1e-3) / 8e12, 4)}))
