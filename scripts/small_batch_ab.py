"""Per-call time of small fused encode + CRC32C batches of 16-B cells, fused kernel vs unfused kernels (TuneKnobs
fused_min_units), device-resident and from pinned host memory, interleaved in one process: where the
fused_min_units default comes from.  (Byte-granular cells always run fused: their unfused kernels take byte paths,
7-8x slower in the first run of this script, profiles/r05/small/.)
usage: python scripts/small_batch_ab.py [ROUNDS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402
from ozone_amd.stripe_queue import host_alloc  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
lib = L.lib()
torch.cuda.set_device(0)
k, p, bpc = 6, 3, 16384
enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
MODES = {"fused": 0, "unfused": 1 << 40}


def dev_case(S, n):
    nwin = -(-n // bpc)
    units = torch.randint(0, 256, (S, k + p, n), dtype=torch.uint8, device="cuda")
    crcs = torch.empty((S, k + p, nwin), dtype=torch.int32, device="cuda")

    def call():
        enc.encode_crc_batch(units, (k + p) * n, n, units[:, k:], (k + p) * n, n, S, n, ck.ChecksumType.CRC32C, bpc,
                             crcs)
    return call, lambda: (units[:, k:].clone(), crcs.clone())


def host_case(S, n):
    nwin = -(-n // bpc)
    pb = host_alloc(S * (k + p) * n + S * (k + p) * nwin * 4)
    a = pb.array
    a[:] = np.random.default_rng(n).integers(0, 256, a.size, dtype=np.uint8)
    crc = a.ctypes.data + S * (k + p) * n

    def call():
        enc.encode_crc_host_batch(a.ctypes.data, (k + p) * n, n, a.ctypes.data + k * n, (k + p) * n, n, S, n,
                                  ck.ChecksumType.CRC32C, bpc, crc)
    call.keep = pb  # the pinned buffer lives as long as the call that uses it
    return call, None


def timed(call, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


for where, make in (("device", dev_case), ("host_pinned", host_case)):
    for n in (1 << 20, 700_000, 65536):
        for S in (1, 2, 4, 8, 16, 32, 64, 128):
            if where == "host_pinned" and S > 32:
                continue
            call, snap = make(S, n)
            ref = None
            for m, v in MODES.items():  # bit-exact across the two routes before timing
                lib.ozec_set_tuning(b"fused_min_units", v)
                call()
                torch.cuda.synchronize()
                if snap:
                    got = snap()
                    ref = ref or got
                    assert all(torch.equal(x, y) for x, y in zip(ref, got)), (where, n, S, m)
            reps = max(5, min(200, int(2e5 / (S * n / 1e3 + 50))))
            res = {m: [] for m in MODES}
            for _ in range(rounds):
                for m, v in MODES.items():
                    lib.ozec_set_tuning(b"fused_min_units", v)
                    call()
                    res[m].append(timed(call, reps))
            row = {"where": where, "cell_bytes": n, "stripes": S, "units": S * -(-n // bpc)}
            for m in MODES:
                row[f"{m}_us"] = round(float(np.median(res[m])), 1)
            row["unfused_over_fused"] = round(row["unfused_us"] / row["fused_us"], 3)
            print(json.dumps(row), flush=True)
lib.ozec_set_tuning(b"fused_min_units", 5120)
