"""Same-process A/B of the fused encode + CRC32C on cells that end in a short window: rs-3-2-1524k (1524 KiB cells,
16 KiB windows, a 4 KiB last window; ECBlockChecksumComputer.java:160-166) and rs-6-3-1524k, device-resident.
Variant 0 (the nibble kernel, which takes short last windows since round 4) against 49 (the per-window kernel that
took them before), interleaved rounds, HIP events on the launch stream; prints one JSON line per (shape, variant).
CELL (bytes, a multiple of 16) replaces 1524 KiB, e.g. 700000: 42 windows and an 11,872-B last window (a cell of the
last, partial stripe of a block group; cells that are not whole 2 KiB groups take the nibble kernel since round 4).
usage: python scripts/ab_short_window.py [ROUNDS [CELL]]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N, BPC = (int(sys.argv[2]) if len(sys.argv) > 2 else 1524 * 1024), 16384
lib = L.lib()
for k, p, S in ((3, 2, 4096), (6, 3, 2048)):
    nwin = -(-N // BPC)
    units = torch.empty((S, k + p, N), dtype=torch.uint8, device="cuda")
    for u in range(k):
        rc.fill_splitmix64_cells(units[:, u], (k + p) * N, S, N, 0x00EC5EED, 900000 + u * S)
    crcs = torch.empty((S, k + p, nwin), dtype=torch.int32, device="cuda")
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    alg = S * (k + p) * N + S * (k + p) * nwin * 4
    times = {0: [], 49: []}

    def run(v, steps=10):
        assert lib.ozec_set_tuning(b"crc_variant", v) == 0
        enc.encode_crc_batch(units, (k + p) * N, N, units[:, k:], (k + p) * N, N, S, N, ck.ChecksumType.CRC32C, BPC,
                             crcs)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(steps):
            enc.encode_crc_batch(units, (k + p) * N, N, units[:, k:], (k + p) * N, N, S, N, ck.ChecksumType.CRC32C,
                                 BPC, crcs)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / steps

    try:
        for _ in range(ROUNDS):
            for v in (0, 49):
                times[v].append(run(v))
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    for v, ts in times.items():
        med = sorted(ts)[len(ts) // 2]
        print(json.dumps({"shape": f"rs-{k}-{p} cells of {N} B", "stripes": S, "crc_variant": v, "median_ms": round(med, 3),
                          "frac": round(alg / (med * 1e-3) / 8e12, 4)}), flush=True)
    del units, crcs
    torch.cuda.empty_cache()
