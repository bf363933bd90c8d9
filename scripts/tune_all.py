"""Interleaved A/B over tuning knobs for every bench workload, in one process.

  KNOBS='unit_map=0,1;gf_variant=0,4' python scripts/tune_all.py c2,c3 3
Each configuration is a combination of the listed knob values; outputs are checked bit-exact vs the first."""
import itertools, json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import bench
from ozone_amd import _lib as L
torch.cuda.set_device(0)
wls = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2"]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
knobs = [kv.split("=") for kv in os.environ.get("KNOBS", "unit_map=0,1").split(";")]
names = [k for k, _ in knobs]
combos = list(itertools.product(*[[int(x) for x in v.split(",")] for _, v in knobs]))
lib = L.lib()

def setk(c):
    for n_, v in zip(names, c):
        lib.ozec_set_tuning(n_.encode(), v)

def outputs(w):
    outs = []
    for attr in ("units", "out", "crcs", "out_crc", "mism", "data"):
        t = getattr(w, attr, None)
        if t is not None and attr != "data" and attr != "units":
            outs.append(t.clone())
    if w.name in ("c2", "c4", "c5"):
        outs.append(w.units[:, w.k:].clone())
    return outs

for name in wls:
    w = bench.Workload(name, 0, 1, None)
    setk(combos[0]); w.step(); torch.cuda.synchronize(); ref = outputs(w)
    for c in combos[1:]:
        setk(c); w.step(); torch.cuda.synchronize()
        ok = all(torch.equal(a, b) for a, b in zip(ref, outputs(w)))
        if not ok:
            print(json.dumps({"wl": name, "config": dict(zip(names, c)), "bit_exact": False})); sys.exit(2)
    times = {c: [] for c in combos}
    for r in range(rounds):
        for c in combos:
            setk(c); w.step()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); w.step(); w.step(); b.record(); torch.cuda.synchronize()
            times[c].append(a.elapsed_time(b) / 2)
    for c in sorted(combos, key=lambda c: np.median(times[c])):
        med = float(np.median(times[c]))
        print(json.dumps({"wl": name, "config": dict(zip(names, c)), "median_ms": round(med, 3),
                          "frac": round(w.alg_bytes / (med * 1e-3) / 8e12, 4)}), flush=True)
    del w
    torch.cuda.empty_cache()
setk([0] * len(names))
