"""Coding throughput when a stripe's units lie 2 GiB or more apart (unit stride 768 MiB: cells spread over a large
HBM pool), for the library given by OZEC_LIB_OVERRIDE (or the in-tree one): rs-6-3 / rs-3-2 encode and rs-10-4
decode of 4 erased units, 64 stripes of 1 MiB cells, aligned and at an odd base, HIP-event timed, one JSON line per
case.  Run once per library (scripts/gpu_r5.sh step wide).
usage: python scripts/wide_ab.py [TAG]"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from ozone_amd import rawcoder as rc  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
torch.cuda.set_device(0)
US = 768 << 20
n, S = 1 << 20, 64
ss = n  # stripes side by side inside each unit slot
for mode, k, p in (("encode", 6, 3), ("encode", 3, 2), ("decode", 10, 4)):
    for shift in (0, 3):
        units = k + p
        buf = torch.empty(shift + (units - 1) * US + S * ss + 64, dtype=torch.uint8, device="cuda")
        base = buf[shift:]
        for u in range(units):
            base[u * US:u * US + S * ss].random_(0, 256)
        conf = rc.ECReplicationConfig(k, p)
        if mode == "encode":
            enc = rc.RawErasureEncoder(conf)

            def call():
                enc.encode_batch(base, ss, US, base[k * US:], ss, US, S, n)
            moved = (k + p) * n * S
        else:
            dec = rc.RawErasureDecoder(conf)
            erased = [0, 1, 2, 3]
            present = [u for u in range(units) if u not in erased][:k]
            out = torch.empty((S, len(erased), n), dtype=torch.uint8, device="cuda")

            def call():
                dec.decode_batch(base, ss, US, present, erased, out, len(erased) * n, n, S, n)
            moved = (k + len(erased)) * n * S
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        reps = 10
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            call()
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / reps
        print(json.dumps({"lib": tag, "op": f"{mode} rs-{k}-{p}", "offset": shift, "unit_stride": US, "ms": round(ms, 3),
                          "GB/s": round(moved / ms / 1e6, 1)}), flush=True)
        del buf
