"""Ranges of the default bench line's fields over several runs (README): headline, every leg's
data GB/s, roofline fraction, rocprof/event ratio and PMC traffic ratio, and the e2e legs.
usage: python scripts/line_ranges.py BENCH_JSON...  (files holding the bench.py line, or the driver's BENCH_rNN.json)"""
import json
import sys
from collections import defaultdict


def line(path):
    """the bench.py JSON line of a run's output file, or of a driver record (its "run" -> "stdout_tail")"""
    text = open(path).read()
    try:
        rec = json.loads(text)
        if "run" in rec:
            text = rec["run"]["stdout_tail"]
    except json.JSONDecodeError:
        pass
    return json.loads([x for x in text.splitlines() if x.startswith("{")][-1])


agg = defaultdict(lambda: defaultdict(list))
for p in sys.argv[1:]:
    d = line(p)
    r = d["roofline"]
    agg["c2"]["GBps"].append(d["value"])
    agg["c2"]["frac"].append(r["frac"])
    if r.get("rocprof_avg_over_events"):
        agg["c2"]["rocprof/events"].append(r["rocprof_avg_over_events"])
    legs = d.get("legs") or d.get("fused") or []
    for i, leg in enumerate(legs):
        name = leg.get("leg") or ("c5dev" if i == 0 else f"c3r#{i}")
        if "frac" not in leg:
            continue
        agg[name]["GBps"].append(leg["value"])
        agg[name]["frac"].append(leg["frac"])
        if leg.get("rocprof_avg_ms"):
            agg[name]["rocprof/events"].append(leg["rocprof_avg_ms"] / leg["kernel_ms"])
        if leg.get("traffic"):
            agg[name]["traffic/alg"].append(leg["traffic"] / leg["alg_bytes_per_launch"])
    for k in ("e2e", "e2e_in_process"):
        if d.get(k) and d[k].get("value"):
            agg[k]["GBps"].append(d[k]["value"])
for name, fields in agg.items():
    print(name, {f: (round(min(v), 4), round(max(v), 4), len(v)) for f, v in fields.items()})
