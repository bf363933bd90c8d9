"""Interleaved A/B of the CRC / fused encode+CRC kernel variants and grids in one process.
Every variant's outputs are compared bit-for-bit with the default variant's before timing."""
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
k, p, S = 6, 3, 4096
U = torch.empty((S, k + p, n), dtype=torch.uint8, device="cuda")
for u in range(k):
    rc.fill_splitmix64_cells(U[:, u], (k + p) * n, S, n, 1, u * S)
crcs = torch.empty((S, k + p, n // bpc), dtype=torch.int32, device="cuda")
crc2 = torch.empty((S * k, n // bpc), dtype=torch.int32, device="cuda")
e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
st = (k + p) * n
X = torch.empty((S, 3, n), dtype=torch.uint8, device="cuda")
for u in range(2):
    rc.fill_splitmix64_cells(X[:, u], 3 * n, S, n, 2, u * S)
xcrcs = torch.empty((S, 3, n // bpc), dtype=torch.int32, device="cuda")
ex = rc.RawErasureEncoder(rc.ECReplicationConfig(2, 1, "xor"))
steps = {
    "c5": (lambda: e.encode_crc_batch(U, st, n, U[:, k:], st, n, S, n, ck.ChecksumType.CRC32C, bpc, crcs),
           S * 9 * n, lambda: (crcs.clone(), U[:, k:].clone())),
    "c4": (lambda: ex.encode_crc_batch(X, 3 * n, n, X[:, 2:], 3 * n, n, S, n, ck.ChecksumType.CRC32C, bpc, xcrcs),
           S * 3 * n, lambda: (xcrcs.clone(), X[:, 2].clone())),
    "crc": (lambda: [ck.checksum_windows_batch(ck.ChecksumType.CRC32C, U[:, j], st, S, n, bpc, crc2[j * S:])
                     for j in range(k)], S * k * n, lambda: (crc2.clone(),)),
}
VAR = {"c5": [int(v) for v in os.environ.get("C5VARIANTS", "0,3,5,6,7").split(",")],
       "c4": [int(v) for v in os.environ.get("C4VARIANTS", "0,13").split(",")],
       "crc": [int(v) for v in os.environ.get("CRCVARIANTS", "0,2,4").split(",")]}
grids = [int(g) for g in os.environ.get("GRIDS", "0,16384").split(",")]
GRID_KEY = os.environ.get("GRID_KEY", "crc_grid").encode()  # the knob GRIDS sweeps (crc_grid or crc_run)
configs = [(w, v, g) for w in steps for v in VAR[w] if v >= 0 for g in grids]
# correctness: every variant equals variant 0 bit for bit
for w in steps:
    if not any(v >= 0 for v in VAR[w]):
        continue
    lib.ozec_set_tuning(b"crc_variant", 0); lib.ozec_set_tuning(b"crc_grid", 0)
    steps[w][0](); torch.cuda.synchronize(); ref = steps[w][2]()
    for v in VAR[w]:
        lib.ozec_set_tuning(b"crc_variant", v)
        for t in ref: pass
        if w == "c5": crcs.zero_(); U[:, k:].zero_()
        elif w == "c4": xcrcs.zero_(); X[:, 2].zero_()
        else: crc2.zero_()
        steps[w][0](); torch.cuda.synchronize(); got = steps[w][2]()
        ok = all(torch.equal(a, b) for a, b in zip(ref, got))
        print(json.dumps({"check": w, "variant": v, "bit_exact_vs_default": ok}), flush=True)
        if not ok:
            sys.exit(2)
times = {c: [] for c in configs}
for r in range(rounds):
    for c in configs:
        lib.ozec_set_tuning(b"crc_variant", c[1]); lib.ozec_set_tuning(GRID_KEY, c[2])
        fn = steps[c[0]][0]
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); fn(); b.record(); torch.cuda.synchronize()
        times[c].append(a.elapsed_time(b) / 2)
for c in sorted(configs, key=lambda c: (c[0], np.median(times[c]))):
    med = float(np.median(times[c]))
    print(json.dumps({"wl": c[0], "variant": c[1], GRID_KEY.decode(): c[2], "median_ms": round(med, 3),
                      "frac": round(steps[c[0]][1] / (med * 1e-3) / 8e12, 4)}))
