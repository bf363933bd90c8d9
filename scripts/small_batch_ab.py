"""Per-call time of small fused batches: the fused nibble kernel's default geometry, its small-batch geometries
(variants 220-222: workgroups of 1 / 2 / 4 waves) and the unfused kernels (TuneKnobs fused_min_units /
rec_min_units), interleaved in one process with outputs checked bit-exact across the routes first.  Encode + CRC32C
of rs-6-3 stripes (device-resident and from pinned host memory) and verify + decode + CRC of rs-10-4 / rs-6-3
reconstructions (device-resident): where the fused_min_units / rec_min_units / nb_small_units defaults come from.
(Units at unaligned offsets always run fused: their unfused kernels take byte paths, 7-8x slower in the first run of
this script, profiles/r05/small/small_batch_ab_first.json.)
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
bpc = 16384
BIG = 1 << 40
DEFAULTS = {b"crc_variant": 0, b"fused_min_units": 1024, b"rec_min_units": 0, b"nb_small_units": 16384}
MODES = [("fused", {b"fused_min_units": 0, b"rec_min_units": 0, b"nb_small_units": 0}),
         ("nb220", {b"crc_variant": 220, b"fused_min_units": 0, b"rec_min_units": 0}),
         ("nb221", {b"crc_variant": 221, b"fused_min_units": 0, b"rec_min_units": 0}),
         ("nb222", {b"crc_variant": 222, b"fused_min_units": 0, b"rec_min_units": 0}),
         ("unfused", {b"fused_min_units": BIG, b"rec_min_units": BIG})]


def apply(settings):
    for key, v in {**DEFAULTS, **settings}.items():
        assert lib.ozec_set_tuning(key, v) == 0, key


def enc_dev(S, n, k=6, p=3):
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    nwin = -(-n // bpc)
    units = torch.randint(0, 256, (S, k + p, n), dtype=torch.uint8, device="cuda")
    crcs = torch.empty((S, k + p, nwin), dtype=torch.int32, device="cuda")

    def call():
        enc.encode_crc_batch(units, (k + p) * n, n, units[:, k:], (k + p) * n, n, S, n, ck.ChecksumType.CRC32C, bpc,
                             crcs)
    return call, lambda: (units[:, k:].clone(), crcs.clone())


def rec_dev(S, n, k, p, erased):
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    nwin = -(-n // bpc)
    units = torch.randint(0, 256, (S, k + p, n), dtype=torch.uint8, device="cuda")
    stored = torch.empty((S, k + p, nwin), dtype=torch.int32, device="cuda")
    enc.encode_crc_batch(units, (k + p) * n, n, units[:, k:], (k + p) * n, n, S, n, ck.ChecksumType.CRC32C, bpc, stored)
    present = [u for u in range(k + p) if u not in erased]
    out = torch.empty((S, len(erased), n), dtype=torch.uint8, device="cuda")
    ocrc = torch.empty((S, len(erased), nwin), dtype=torch.int32, device="cuda")
    mism = torch.empty(S, dtype=torch.int32, device="cuda")

    def call():
        dec.reconstruct_crc_batch(units, (k + p) * n, n, present, erased, out, len(erased) * n, n, S, n,
                                  ck.ChecksumType.CRC32C, bpc, ocrc, d_expected=stored, d_mismatch=mism)
    return call, lambda: (out.clone(), ocrc.clone(), mism.clone())


def enc_host(S, n, k=6, p=3):
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    nwin = -(-n // bpc)
    pb = host_alloc(S * (k + p) * n + S * (k + p) * nwin * 4)
    a = pb.array
    a[:] = np.random.default_rng(n).integers(0, 256, a.size, dtype=np.uint8)
    crc = a.ctypes.data + S * (k + p) * n

    def call():
        enc.encode_crc_host_batch(a.ctypes.data, (k + p) * n, n, a.ctypes.data + k * n, (k + p) * n, n, S, n,
                                  ck.ChecksumType.CRC32C, bpc, crc)
    call.keep = pb  # the pinned buffer lives as long as the call that uses it
    return call, lambda: (torch.from_numpy(a.copy()),)


def timed(call, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


CASES = [("encode rs-6-3 device", n, S, lambda S, n: enc_dev(S, n)) for n in (1 << 20, 65536)
         for S in (1, 2, 4, 8, 16, 32, 64, 128, 256)]
CASES += [("encode rs-6-3 device packed", 700_001, S, lambda S, n: enc_dev(S, n)) for S in (1, 8, 64)]
CASES += [(f"reconstruct rs-10-4 {{0,1,2,3}} device", 1 << 20, S, lambda S, n: rec_dev(S, n, 10, 4, [0, 1, 2, 3]))
          for S in (1, 2, 4, 8, 16, 32, 64, 128)]
CASES += [(f"reconstruct rs-6-3 {{1}} device", 1 << 20, S, lambda S, n: rec_dev(S, n, 6, 3, [1]))
          for S in (1, 4, 16, 64, 128)]
CASES += [("encode rs-6-3 host pinned", 1 << 20, S, lambda S, n: enc_host(S, n)) for S in (1, 4, 16)]

for what, n, S, make in CASES:
    call, snap = make(S, n)
    ref = None
    for name, st in MODES:  # bit-exact across the routes before timing
        apply(st)
        call()
        torch.cuda.synchronize()
        got = snap()
        ref = ref or got
        assert all(torch.equal(x, y) for x, y in zip(ref, got)), (what, n, S, name)
    reps = max(5, min(200, int(2e5 / (S * n / 1e3 + 50))))
    res = {name: [] for name, _ in MODES}
    for _ in range(rounds):
        for name, st in MODES:
            apply(st)
            call()
            res[name].append(timed(call, reps))
    row = {"case": what, "cell_bytes": n, "stripes": S, "units": S * -(-n // bpc)}
    for name, _ in MODES:
        row[f"{name}_us"] = round(float(np.median(res[name])), 1)
    row["best"] = min((row[f"{name}_us"], name) for name, _ in MODES)[1]
    print(json.dumps(row), flush=True)
    del call, snap
apply({})
