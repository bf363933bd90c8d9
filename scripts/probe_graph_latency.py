"""Probe: does a hipGraph cut the per-call latency of a one-stripe host encode?  One rs-6-3 stripe from pinned host
memory: H2D of the k cells, the coding kernel, D2H of the p parity cells, then a host wait -- issued as three stream
operations, or as one captured graph replayed (torch.cuda.graph drives hipStreamBeginCapture; libozec's coding
kernel is capture-safe).  Both are checked against each other and timed per call (median of ROUNDS x 200 calls).
usage: python scripts/probe_graph_latency.py [ROUNDS]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ozone_amd import rawcoder as rc  # noqa: E402

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 5
torch.cuda.set_device(0)
k, p = 6, 3
enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
for n in (64 << 10, 1 << 20):
    h_in = torch.randint(0, 256, (k, n), dtype=torch.uint8).pin_memory()
    h_out = torch.empty((p, n), dtype=torch.uint8).pin_memory()
    d_in = torch.empty((k, n), dtype=torch.uint8, device="cuda")
    d_out = torch.empty((p, n), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()

    def ops():
        d_in.copy_(h_in, non_blocking=True)
        enc.encode_batch(d_in, k * n, n, d_out, p * n, n, 1, n)
        h_out.copy_(d_out, non_blocking=True)

    with torch.cuda.stream(s):
        ops()
    s.synchronize()
    ref = h_out.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ops()
    h_out.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(ref, h_out))

    def time_calls(fn, calls=200):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
            torch.cuda.synchronize()  # device-wide: a replay runs on the current stream, not on s
        return (time.perf_counter() - t0) / calls * 1e6

    def plain():
        with torch.cuda.stream(s):
            ops()

    res = {"plain": [], "graph": []}
    for _ in range(ROUNDS):
        res["plain"].append(time_calls(plain))
        res["graph"].append(time_calls(g.replay))
    med = {kk: sorted(v)[len(v) // 2] for kk, v in res.items()}
    print(json.dumps({"cell_bytes": n, "stripe": f"rs-{k}-{p}", "plain_us": round(med["plain"], 1),
                      "graph_us": round(med["graph"], 1), "graph_output_equal": same}), flush=True)
    del g
