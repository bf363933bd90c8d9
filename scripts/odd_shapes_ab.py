"""Coding throughput of the shapes without a gf_code_vec instantiation (XOR-k-1: xor_vec; RS outside 3/6/10 data
units: gf_code_vec_generic) on packed stripes at odd byte offsets, for the library given by OZEC_LIB_OVERRIDE (or
the in-tree one): ozec_encode_batch over S stripes, HIP-event timed, one JSON line per shape.  Run once per library
(scripts/gpu_r5.sh step oddshapes) to compare the round-5 BUF instantiations with the byte kernel they replace.
usage: python scripts/odd_shapes_ab.py [TAG]"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from ozone_amd import rawcoder as rc  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
torch.cuda.set_device(0)
SHAPES = [("xor", 2, 1), ("xor", 3, 1), ("rs", 4, 2), ("rs", 5, 6), ("rs", 6, 3)]
for codec, k, p in SHAPES:
    for n, S in ((1 << 20, 64), ((1 << 20) + 1, 64), (700_001, 64)):
        units = torch.randint(0, 256, (S * (k + p) * n + 16,), dtype=torch.uint8, device="cuda")
        base = units[3:]  # odd base: every unit at an odd offset
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec))

        def call():
            enc.encode_batch(base, (k + p) * n, n, base[k * n:], (k + p) * n, n, S, n)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        reps = 20
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            call()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1000 / reps
        gbs = S * (k + p) * n / us / 1e3
        print(json.dumps({"lib": tag, "shape": f"{codec}-{k}-{p}", "n": n, "stripes": S, "us": round(us, 1),
                          "GB/s": round(gbs, 1)}), flush=True)
        del units
