"""Interleaved A/B of HBM layouts: unit stride = 1 MiB + pad (channel/bank aliasing test) for encode (c2) and
decode (c3)."""
import json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from ozone_amd import rawcoder as rc
torch.cuda.set_device(0)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = 1 << 20
pads = [int(x) for x in os.environ.get("PADS", "0,256,1024,4096,12288,65536").split(",")]
res = []
for wl, (k, p, S) in (("c2", (6, 3, 4096)), ("c3", (10, 4, 2048))):
    cfgs = {}
    for pad in pads:
        us = n + pad
        U = torch.empty((S, (k + p) * us), dtype=torch.uint8, device="cuda")
        st = (k + p) * us
        for u in range(k):
            rc.fill_splitmix64_cells(U[:, u * us:], st, S, n, 1, u * S)
        e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
        if wl == "c2":
            f = (lambda U=U, e=e, st=st, us=us: e.encode_batch(U, st, us, U[:, k * us:], st, us, S, n))
            alg = S * (k + p) * n
        else:
            e.encode_batch(U, st, us, U[:, k * us:], st, us, S, n)
            d = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
            O = torch.empty((S, 4 * us), dtype=torch.uint8, device="cuda")
            f = (lambda U=U, d=d, st=st, us=us, O=O: d.decode_batch(U, st, us, list(range(4, 14)), [0, 1, 2, 3], O,
                                                                      4 * us, us, S, n))
            alg = S * 14 * n
        cfgs[pad] = (f, alg, U)
    times = {pd: [] for pd in cfgs}
    for r in range(rounds):
        for pd, (f, alg, _) in cfgs.items():
            f()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); f(); b.record(); torch.cuda.synchronize()
            times[pd].append(a.elapsed_time(b) / 2)
    for pd in cfgs:
        med = float(np.median(times[pd]))
        print(json.dumps({"wl": wl, "pad": pd, "median_ms": round(med, 3), "frac": round(cfgs[pd][1] / (med * 1e-3) / 8e12, 4)}), flush=True)
    del cfgs
    torch.cuda.empty_cache()
