"""Interleaved A/B of ozec_set_tuning variants on one bench.py workload, in one process.
usage: python scripts/ab.py WORKLOAD KEY V1,V2,... [ROUNDS]
Each variant's outputs are checked bit-for-bit against the first variant's before timing."""
import json, os, sys
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden"))
import numpy as np, torch
import bench
from ozone_amd import _lib as L

wl_name, key, vals = sys.argv[1], sys.argv[2].encode(), [int(v) for v in sys.argv[3].split(",")]
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
torch.cuda.set_device(0)
lib = L.lib()
for kv in filter(None, os.environ.get("FIX", "").split(",")):  # knobs held fixed for every variant (FIX=k=v,k=v)
    fk, fv = kv.split("=")
    assert lib.ozec_set_tuning(fk.encode(), int(fv)) == 0, kv
wl = bench.Workload(wl_name, 0, 1, int(os.environ["STRIPES"]) if os.environ.get("STRIPES") else None,
                   int(os.environ.get("THREADS", "1")))
if os.environ.get("ZERO"):  # all-zero data cells: separates data-dependent power/clock effects
    for name in ("units", "data", "blocks"):
        if hasattr(wl, name):
            getattr(wl, name).zero_()
    torch.cuda.synchronize()


def outputs():
    return [t.clone() for t in (getattr(wl, a, None) for a in ("crcs", "out", "out_crc", "mism")) if t is not None] + \
        ([wl.units[:, wl.k:].clone()] if hasattr(wl, "units") else [])


ref = None
for v in vals:
    lib.ozec_set_tuning(key, v)
    wl._step(); torch.cuda.synchronize()
    got = outputs()
    if ref is None:
        ref = got
    ok = all(torch.equal(a, b) for a, b in zip(ref, got))
    print(json.dumps({"variant": v, "bit_exact_vs_first": ok}), flush=True)
    if not ok and not os.environ.get("NOCHECK"):  # NOCHECK: timing probes that compute wrong results on purpose
        sys.exit(2)
times = {v: [] for v in vals}
for _ in range(rounds):
    for v in vals:
        lib.ozec_set_tuning(key, v)
        wl._step()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); wl._step(); wl._step(); wl._step(); b.record(); torch.cuda.synchronize()
        times[v].append(a.elapsed_time(b) / 3)
for v in sorted(vals, key=lambda v: np.median(times[v])):
    med = float(np.median(times[v]))
    print(json.dumps({"wl": wl_name, "fix": os.environ.get("FIX", ""), key.decode(): v, "median_ms": round(med, 3),
                      "frac": round(wl.alg_bytes / (med * 1e-3) / 8e12, 4)}), flush=True)
