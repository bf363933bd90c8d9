"""How much of a per-launch HIP-event time is the launch boundary: time N back-to-back steps of a bench workload
between one event pair, for N = 1, 3, 10 (median over rounds).  usage: python scripts/event_bracket.py WORKLOAD"""
import json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import bench

wl = bench.Workload(sys.argv[1], 0, 1, None)
torch.cuda.set_device(0)
for _ in range(5):
    wl._step()
torch.cuda.synchronize()
st = torch.cuda.current_stream()
for n in (1, 3, 10, 1):
    ts = []
    for _ in range(15):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(n):
            wl._step()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / n)
    med = float(np.median(ts))
    print(json.dumps({"wl": sys.argv[1], "steps_per_event_pair": n, "ms_per_step": round(med, 4),
                      "frac": round(wl.alg_bytes / (med * 1e-3) / 8e12, 4)}), flush=True)
