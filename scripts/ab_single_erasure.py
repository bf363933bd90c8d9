"""Same-process A/B of the fused reconstruction (verify the CRCs of the k units read + decode + CRC of the rebuilt unit)
for a single lost unit of rs-6-3 and rs-3-2 -- the commonest datanode recovery (ECReconstructionCoordinator.java:240-352)
-- device-resident, 1 MiB cells, CRC32C per 16 KiB.  Variant 0 (the nibble kernel, which takes one-output shapes since
round 4) against 49 (the per-window kernel that took them before); interleaved rounds, HIP events.  VARIANTS (env,
default 0,49) picks the crc_variant ids compared; SHAPES=all adds rs-6-3 with three units lost (round 5, CV).
usage: [VARIANTS=0,231] [SHAPES=all] python scripts/ab_single_erasure.py [ROUNDS]"""
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
N, BPC = 1 << 20, 16384
lib = L.lib()
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,49").split(",")]
SHAPES = [(6, 3, [2], 3072), (3, 2, [1], 4096)]
if os.environ.get("SHAPES") == "all":
    SHAPES.append((6, 3, [0, 4, 7], 3072))
for k, p, erased, S in SHAPES:
    nwin = N // BPC
    units = torch.empty((S, k + p, N), dtype=torch.uint8, device="cuda")
    for u in range(k):
        rc.fill_splitmix64_cells(units[:, u], (k + p) * N, S, N, 0x00EC5EED, 910000 + u * S)
    rc.RawErasureEncoder(rc.ECReplicationConfig(k, p)).encode_batch(units, (k + p) * N, N, units[:, k:], (k + p) * N,
                                                                     N, S, N)
    stored = torch.empty((S, k + p, nwin), dtype=torch.int32, device="cuda")
    ck.checksum_windows_batch(ck.ChecksumType.CRC32C, units, N, S * (k + p), N, BPC, stored)
    present = [u for u in range(k + p) if u not in erased]
    out = torch.empty((S, len(erased), N), dtype=torch.uint8, device="cuda")
    ocrc = torch.empty((S, len(erased), nwin), dtype=torch.int32, device="cuda")
    mism = torch.empty(S, dtype=torch.int32, device="cuda")
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    e = len(erased)
    alg = S * (k + e) * N + S * (k + e) * nwin * 4 + S * 4  # k units + their stored CRCs read, e units + CRCs written
    times = {v: [] for v in VARIANTS}

    def launch():
        dec.reconstruct_crc_batch(units, (k + p) * N, N, present, erased, out, e * N, N, S, N, ck.ChecksumType.CRC32C,
                                  BPC, ocrc, d_expected=stored, d_mismatch=mism)

    def run(v, steps=10):
        assert lib.ozec_set_tuning(b"crc_variant", v) == 0
        launch()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(steps):
            launch()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) / steps

    try:
        for _ in range(ROUNDS):
            for v in VARIANTS:
                times[v].append(run(v))
        ok = bool((mism == -1).all().item()) and all(bool((out[:, i] == units[:, u]).all().item())
                                                     for i, u in enumerate(erased))
    finally:
        lib.ozec_set_tuning(b"crc_variant", 0)
    for v, ts in times.items():
        med = sorted(ts)[len(ts) // 2]
        print(json.dumps({"shape": f"rs-{k}-{p}-1024k reconstruct {erased}", "stripes": S, "crc_variant": v,
                          "median_ms": round(med, 3), "frac": round(alg / (med * 1e-3) / 8e12, 4), "verified": ok}),
              flush=True)
    del units, stored, out, ocrc
    torch.cuda.empty_cache()
