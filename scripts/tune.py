"""Interleaved A/B of coding-kernel variants and grid sizes in ONE process (guide §5.4 rule 24).

  python scripts/tune.py [c2|c3] [rounds]
Prints one line per (variant, grid) with median/min kernel ms and the HBM fraction.
"""
import itertools
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from ozone_amd import _lib as L
from ozone_amd import rawcoder as rc

torch.cuda.set_device(0)
wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = 1 << 20
if wl == "c2":
    k, p, S = 6, 3, 4096
else:
    k, p, S = 10, 4, 2048
units = torch.empty((S, k + p, n), dtype=torch.uint8, device="cuda")
for u in range(k):
    rc.fill_splitmix64_cells(units[:, u], (k + p) * n, S, n, 1, u * S)
stride = (k + p) * n
if wl == "c2":
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    step = lambda: e.encode_batch(units, stride, n, units[:, k:], stride, n, S, n)
    alg = S * (k + p) * n
else:
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    e.encode_batch(units, stride, n, units[:, k:], stride, n, S, n)
    d = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    out = torch.empty((S, 4, n), dtype=torch.uint8, device="cuda")
    present = list(range(4, 14))
    step = lambda: d.decode_batch(units, stride, n, present, [0, 1, 2, 3], out, 4 * n, n, S, n)
    alg = S * 14 * n
variants = [int(v) for v in os.environ.get("VARIANTS", "1,2,3,4,5,6").split(",")]
grids = [int(g) for g in os.environ.get("GRIDS", "0,1024,1280,1536,2560,4096,8192,1000000").split(",")]
configs = list(itertools.product(variants, grids))
times = {c: [] for c in configs}
lib = L.lib()
for r in range(rounds):
    for c in configs:
        lib.ozec_set_tuning(b"gf_variant", c[0])
        lib.ozec_set_tuning(b"grid", c[1])
        step()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            step()
        b.record()
        torch.cuda.synchronize()
        times[c].append(a.elapsed_time(b) / 3)
res = []
for c in configs:
    med = float(np.median(times[c]))
    res.append({"variant": c[0], "grid": c[1], "median_ms": round(med, 4), "min_ms": round(min(times[c]), 4),
                "frac": round(alg / (med * 1e-3) / 8e12, 4)})
res.sort(key=lambda x: x["median_ms"])
for x in res:
    print(json.dumps(x))
