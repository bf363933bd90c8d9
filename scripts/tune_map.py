"""Interleaved A/B of block->unit mappings x unit-stride pads for rs-6-3 encode (c2)."""
import itertools, json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ozone_amd import _lib as L
from ozone_amd import rawcoder as rc
torch.cuda.set_device(0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n, k, p, S = 1 << 20, 6, 3, 4096
lib = L.lib()
pads = [int(x) for x in os.environ.get("PADS", "0,65536").split(",")]
maps = [int(x) for x in os.environ.get("MAPS", "0,1,2").split(",")]
bufs = {}
for pad in pads:
    us = n + pad
    U = torch.empty((S, (k + p) * us), dtype=torch.uint8, device="cuda")
    for u in range(k):
        rc.fill_splitmix64_cells(U[:, u * us:], (k + p) * us, S, n, 1, u * S)
    bufs[pad] = U
e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
cfgs = list(itertools.product(pads, maps))
times = {c: [] for c in cfgs}
for r in range(rounds):
    for pad, m in cfgs:
        lib.ozec_set_tuning(b"unit_map", m)
        us = n + pad; st = (k + p) * us; U = bufs[pad]
        f = lambda: e.encode_batch(U, st, us, U[:, k * us:], st, us, S, n)
        f()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); f(); f(); b.record(); torch.cuda.synchronize()
        times[(pad, m)].append(a.elapsed_time(b) / 2)
for c in sorted(cfgs, key=lambda c: np.median(times[c])):
    med = float(np.median(times[c]))
    print(json.dumps({"pad": c[0], "map": c[1], "median_ms": round(med, 3), "frac": round(S * 9 * n / (med * 1e-3) / 8e12, 4)}))
