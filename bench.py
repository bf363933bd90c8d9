#!/usr/bin/env python3
"""Benchmark of the MI355X EC + checksum hot path (driver contract: one JSON line on rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c3r|c4|c5|crc|verify|e2e|host|queue]

Default workload = BASELINE.json configs[1]: rs-6-3-1024k encode of 4096 stripes, device-resident on one
MI355X.  A "step" is one ozec_encode_batch over the whole 4096-stripe batch (24 GiB of data cells read,
12 GiB of parity written).  For N > 1 (torchrun) every rank encodes its own 4096 stripes on its own GPU
(stripes are independent: no collective on the data path, "scaling": "weak"); RCCL is used only for the
start/stop barriers and the max-over-ranks reduction of the elapsed time.

value      = data bytes of all ranks / max-over-ranks wall time of the K timed steps (GB = 1e9 B)
roofline   = algorithmic bytes per launch (9 x 1 MiB per stripe x 4096) / mean kernel time measured with
             HIP events on the launch stream, against 8.0 TB/s; traffic = rocprofv3 PMC bytes per launch
             read from profiles/traffic_<workload>.json when it has been measured, else null
cpu_baseline (rank 0, N = 1): the oracle/ C restatement of the same work timed on this host's cores on a
             bounded sample (threads share one coder, as RawErasureCoderBenchmark.java:201-206 does)
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

MIB = 1 << 20
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED = 0x00EC5EED
METRIC = "EC encode GB/s (data bytes) rs-6-3-1024k @1/8 GPUs + % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c3r", "c4", "c5", "crc", "verify", "e2e", "host", "queue", "queue_pageable"])
    ap.add_argument("--stripes", type=int, default=0, help="override the stripe count (profiling only)")
    ap.add_argument("--erased", default="0,1,2,3",
                    help="c3/c3r: erased unit indexes of rs-10-4 (SURVEY 8(d): 0,1,2,3 all data; 1,4,10,13 mixed)")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--threads", type=int, default=1, help="host workload: caller threads sharing one coder")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="ozec_set_tuning knob (A/B and profiling runs only; defaults are the measured best)")
    return ap.parse_args()


# ------------------------------------------------------------------------------------------ workloads


class Workload:
    """Allocates device-resident inputs once; step() launches one batch on the current stream."""

    def __init__(self, name, rank, stripes_override, threads=1, erased=(0, 1, 2, 3)):
        from ozone_amd import checksum as ck
        from ozone_amd import rawcoder as rc
        self.name = name
        dev = torch.device("cuda", torch.cuda.current_device())
        n = MIB
        self.n = n
        if name == "host":
            k, p, S = 6, 3, stripes_override or 64
            T = max(1, threads)
            rng = np.random.default_rng(rank)
            self.hd = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for _ in range(T)]
            self.hp = [[np.empty(n, np.uint8) for _ in range(p)] for _ in range(T)]
            self.k, self.p, self.S = k, p, S
            enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + p) * n
            self.kernel = "gf_code_vec<6,3> (+pageable->pinned staging, H2D, D2H, per stripe)"
            self.config = {"workload": f"rs-6-3-1024k encode through the host-pointer ABI (ozec_encode: the JNI "
                                       f"drop-in path), {S} single-stripe calls from {T} threads sharing one coder",
                           "stripes": S, "threads": T}

            def run(t):
                for _ in range(t, S, T):
                    enc.encode(self.hd[t], self.hp[t])

            def step():
                if T == 1:
                    return run(0)
                ts = [threading.Thread(target=run, args=(t,)) for t in range(T)]
                for th in ts:
                    th.start()
                for th in ts:
                    th.join()
            self._step = step
            return
        if name in ("queue", "queue_pageable"):
            from ozone_amd.stripe_queue import StripeQueue, host_alloc
            k, p, S, pool = 6, 3, stripes_override or 1024, 64
            pinned = name == "queue"
            self.crc_type, self.bpc = ck.ChecksumType.CRC32C, 16384
            nwin = n // self.bpc
            self._pool = []

            def buf(nbytes, dtype=np.uint8):
                if not pinned:
                    return np.zeros(nbytes // np.dtype(dtype).itemsize, dtype)
                pb = host_alloc(nbytes)
                self._pool.append(pb)
                return pb.array.view(dtype)
            rng = np.random.default_rng(rank)
            # one buffer per stripe with its k data then p parity cells back to back (the layout a writer's
            # pinned cell pool would use); the queue then moves a stripe in one H2D and one D2H copy
            slabs = [buf((k + p) * n) for _ in range(pool)]
            self.qd = [[sl[j * n:(j + 1) * n] for j in range(k)] for sl in slabs]
            for st in self.qd:
                for a in st:
                    a[:] = rng.integers(0, 256, n, dtype=np.uint8)
            self.qp = [[sl[(k + r) * n:(k + r + 1) * n] for r in range(p)] for sl in slabs]
            self.qc = [buf((k + p) * nwin * 4, np.uint32) for _ in range(pool)]
            enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
            self.q = StripeQueue(enc, n, 64, self.crc_type, self.bpc)
            self.k, self.p, self.S = k, p, S
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + p) * n
            self.kernel = "encode_crc_g26<6,3> via ozec_stripe_queue (+H2D/D2H per cell)"
            self.config = {"workload": f"rs-6-3-1024k + CRC32C/16 KiB through the stripe queue (SURVEY 8(f) row 3) "
                                       f"from {'pinned' if pinned else 'pageable'} host cells, {S} stripes, "
                                       f"batches of 64", "stripes": S}

            def step():
                t = 0
                for i in range(S):
                    j = i % pool
                    t = self.q.submit(self.qd[j], self.qp[j], crcs=self.qc[j])
                self.q.wait(t)
            self._step = step
            return
        if name == "c1":
            k, p, S = 3, 2, stripes_override or 1024
        elif name in ("c2", "c5", "e2e"):
            k, p, S = 6, 3, stripes_override or (4096 if name != "e2e" else 1024)
        elif name in ("c3", "c3r"):
            k, p, S = 10, 4, stripes_override or 2048
        elif name == "c4":
            k, p, S = 2, 1, stripes_override or 16 * 256
        else:  # crc
            k, p, S = 1, 0, stripes_override or 8192
        self.k, self.p, self.S = k, p, S
        self.bpc = 16384
        self.nwin = n // self.bpc
        self.crc_type = ck.ChecksumType.CRC32C
        if name in ("crc", "verify"):
            self.data = torch.empty((S, n), dtype=torch.uint8, device=dev)
            rc.fill_splitmix64_cells(self.data, n, S, n, SEED, rank * 10_000_000)
            self.crcs = torch.empty((S, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * n
            if name == "crc":
                self.alg_bytes = S * n + S * self.nwin * 4
                self.kernel = "crc_windows_g26s<4,4>"
                self.config = {"workload": "CRC32C per 16 KiB window, device-resident", "cells": S, "cell_bytes": n,
                               "bytes_per_checksum": self.bpc}
                self._step = lambda: ck.checksum_windows_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs)
            else:
                ck.checksum_windows_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs)
                self.mism = torch.empty(S, dtype=torch.int32, device=dev)
                # every data byte and every stored CRC read, one first-failure index per cell written
                self.alg_bytes = S * n + S * self.nwin * 4 + S * 4
                self.kernel = "crc_windows_g26s<4,4> (verify mode)"
                self.config = {"workload": "CRC32C verify per 16 KiB window against stored CRCs (datanode scanner, "
                                           "SURVEY 8(f) row 2), device-resident", "cells": S, "cell_bytes": n,
                               "bytes_per_checksum": self.bpc}
                self._step = lambda: ck.checksum_verify_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs,
                                                              self.mism)
            torch.cuda.synchronize()
            return
        units = k + p
        if name == "e2e":
            self.host_in = torch.empty((S, k, n), dtype=torch.uint8).pin_memory()
            self.host_out = torch.empty((S, p, n), dtype=torch.uint8).pin_memory()
            self.host_crc = torch.empty((S, units, self.nwin), dtype=torch.int32).pin_memory()
            tmp = torch.empty((S, k, n), dtype=torch.uint8, device=dev)
            rc.fill_splitmix64_cells(tmp, n, S * k, n, SEED, rank * 10_000_000)
            self.host_in.copy_(tmp)
            del tmp
        # HBM layout: stripe-major, units contiguous: unit u of stripe s at s*(k+p)*n + u*n
        self.units = torch.empty((S, units, n), dtype=torch.uint8, device=dev)
        for u in range(k):
            rc.fill_splitmix64_cells(self.units[:, u], units * n, S, n, SEED, rank * 10_000_000 + u * S)
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, "rs" if name != "c4" else "xor"))
        self.enc = enc
        stride = units * n
        if name == "c1":
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n
            self.kernel = "gf_code_vec<3,2>"
            self.config = {"workload": f"rs-3-2-1024k encode, {S} stripes, device-resident (BASELINE configs[0] shape; "
                                       f"the reference runs it on the CPU)", "codec": "rs", "data_units": k,
                           "parity_units": p, "cell_bytes": n, "stripes": S}
            self._step = lambda: enc.encode_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n)
        elif name == "c2":
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n
            self.kernel = "gf_code_vec<6,3>"
            self.config = {"workload": f"rs-6-3-1024k encode, {S} stripes, device-resident (BASELINE configs[1])",
                           "codec": "rs", "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "layout": "stripe-major [stripe][unit][cell] in HBM"}
            self._step = lambda: enc.encode_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n)
        elif name == "c3":
            enc.encode_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n)
            self.dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
            self.erased = sorted(erased)
            present = [u for u in range(units) if u not in self.erased]
            self.out = torch.empty((S, 4, n), dtype=torch.uint8, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + len(self.erased)) * n
            self.kernel = "gf_code_vec<10,4>"
            pat = ",".join(map(str, self.erased))
            self.config = {"workload": f"rs-10-4-1024k decode, {S} stripes, 4 erased {{{pat}}}, device-resident",
                           "codec": "rs", "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S}
            self._step = lambda: self.dec.decode_batch(self.units, stride, n, present, self.erased, self.out, 4 * n,
                                                       n, S, n)
        elif name == "c3r":
            enc.encode_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n)
            self.dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
            self.erased = sorted(erased)
            present = [u for u in range(units) if u not in self.erased]
            self.stored = torch.empty((S, units, self.nwin), dtype=torch.int32, device=dev)
            ck.checksum_windows_batch(self.crc_type, self.units, n, S * units, n, self.bpc, self.stored)
            self.out = torch.empty((S, 4, n), dtype=torch.uint8, device=dev)
            self.out_crc = torch.empty((S, 4, self.nwin), dtype=torch.int32, device=dev)
            self.mism = torch.empty(S, dtype=torch.int32, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + 4) * n + S * (k + 4) * self.nwin * 4
            self.kernel = "encode_crc_g26<10,4> (reconstruct mode)"
            self.config = {"workload": "rs-10-4-1024k reconstruction: verify CRC32C of 10 read units + decode 4 + "
                                       f"CRC32C of rebuilt units {{{','.join(map(str, self.erased))}}}, 2048 stripes, "
                                       "fused, device-resident",
                           "codec": "rs", "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "bytes_per_checksum": self.bpc}
            self._step = lambda: self.dec.reconstruct_crc_batch(
                self.units, stride, n, present, self.erased, self.out, 4 * n, n, S, n, self.crc_type, self.bpc,
                self.out_crc, d_expected=self.stored, d_mismatch=self.mism)
        elif name in ("c4", "c5"):
            self.crcs = torch.empty((S, units, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n + S * units * self.nwin * 4
            self.kernel = f"encode_crc_g26<{k},{p}>"
            wl = ("xor-2-1-1024k + CRC32C/16 KiB, 16 block groups x 256 stripes" if name == "c4"
                  else "rs-6-3-1024k encode + CRC32C/16 KiB, 4096 stripes")
            self.config = {"workload": wl + ", fused, device-resident", "codec": "xor" if name == "c4" else "rs",
                           "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "bytes_per_checksum": self.bpc}
            self._step = lambda: enc.encode_crc_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n,
                                                      self.crc_type, self.bpc, self.crcs)
        else:  # e2e: pinned host -> HBM -> fused encode+CRC -> host, chunked over 2 streams
            self.crcs = torch.empty((S, units, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n
            self.kernel = "encode_crc_g26<6,3> (+H2D/D2H)"
            self.config = {"workload": "rs-6-3-1024k + CRC32C end-to-end from pinned host buffers", "stripes": S}
            self.streams = [torch.cuda.Stream(), torch.cuda.Stream()]
            self._step = self._e2e_step
        torch.cuda.synchronize()

    def _e2e_step(self):
        k, p, n, S = self.k, self.p, self.n, self.S
        stride = (k + p) * n
        chunk = 64
        for i, s0 in enumerate(range(0, S, chunk)):
            st = self.streams[i % 2]
            s1 = min(S, s0 + chunk)
            with torch.cuda.stream(st):
                self.units[s0:s1, :k].copy_(self.host_in[s0:s1], non_blocking=True)
                self.enc.encode_crc_batch(self.units[s0:], stride, n, self.units[s0:, k:], stride, n, s1 - s0, n,
                                          self.crc_type, self.bpc, self.crcs[s0:], stream=st)
                self.host_out[s0:s1].copy_(self.units[s0:s1, k:], non_blocking=True)
                self.host_crc[s0:s1].copy_(self.crcs[s0:s1], non_blocking=True)
        for st in self.streams:
            torch.cuda.current_stream().wait_stream(st)

    def step(self):
        self._step()


def pcie_ceiling(h2d_bytes, d2h_bytes, reps=5):
    """Plain pinned<->HBM DMA rates of the e2e byte volumes: H2D alone, D2H alone, and both at once on two
    streams (full duplex). The e2e/queue paths move 6 MiB in and 3 MiB out per rs-6-3 stripe, so the H2D rate
    under duplex traffic is the ceiling for their data GB/s."""
    dev = torch.device("cuda", torch.cuda.current_device())
    hin = torch.empty(h2d_bytes, dtype=torch.uint8).pin_memory()
    hout = torch.empty(d2h_bytes, dtype=torch.uint8).pin_memory()
    din = torch.empty(h2d_bytes, dtype=torch.uint8, device=dev)
    dout = torch.empty(d2h_bytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(h2d, d2h):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                with torch.cuda.stream(s1):
                    din.copy_(hin, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    hout.copy_(dout, non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    timed(True, True)
    t_h2d, t_d2h, t_both = timed(True, False), timed(False, True), timed(True, True)
    return {"h2d_GBps": round(reps * h2d_bytes / t_h2d / 1e9, 2), "d2h_GBps": round(reps * d2h_bytes / t_d2h / 1e9, 2),
            "duplex_h2d_GBps": round(reps * h2d_bytes / t_both / 1e9, 2),
            "duplex_d2h_GBps": round(reps * d2h_bytes / t_both / 1e9, 2),
            "bytes": {"h2d": h2d_bytes, "d2h": d2h_bytes},
            "note": "contiguous pinned DMA copies of the same volumes, one H2D and one D2H stream"}


# ------------------------------------------------------------------------------------------ CPU baseline


def cpu_baseline(workload, budget_s):
    """oracle/ (C restatement of the reference path, gcc -O3) timed on this host's cores on a bounded sample of
    the workload: T threads share one coder (RawErasureCoderBenchmark.java:201-206), each repeating one unit of
    work (a stripe, a decode, a cell's windows) until the wall budget is spent."""
    import oracle
    from synth import cells
    threads = min(16, os.cpu_count() or 1)
    n = MIB
    if workload == "c3":
        k, p, erased = 10, 4, [0, 1, 2, 3]
        d = cells(SEED, 900, k, n)
        units = d + oracle.rs_encode(k, p, d)
        ins = [None if u in erased else units[u] for u in range(k + p)]
        job, data_bytes = (lambda: oracle.rs_decode(k, p, ins, erased)), k * n
        what = "rs-10-4-1024k decodes of 4 erased units (oracle rs_decode: RSRawDecoder + RSUtil.encodeData)"
    elif workload in ("crc", "verify"):
        cell = cells(SEED, 900, 1, n)[0]
        job, data_bytes = (lambda: oracle.crc_windows(oracle.CRC32C, cell, 16384)), n
        what = "1 MiB cells checksummed as CRC32C/16 KiB windows (oracle crc_windows: CrcIntTable slice-by-8)"
    elif workload in ("c4", "c5", "c3r"):
        k, p = (2, 1) if workload == "c4" else (10, 4) if workload == "c3r" else (6, 3)
        d = cells(SEED, 900, k, n)

        def job():
            par = oracle.rs_encode(k, p, d) if workload != "c4" else [oracle.xor_encode(d)]
            for u in d + par:
                oracle.crc_windows(oracle.CRC32C, u, 16384)
        data_bytes = k * n
        what = {"c4": "xor-2-1-1024k stripes coded + CRC32C/16 KiB of all 3 units",
                "c5": "rs-6-3-1024k stripes coded + CRC32C/16 KiB of all 9 units",
                "c3r": "rs-10-4-1024k stripes, 10 units -> 4 rebuilt + CRC32C/16 KiB of all 14 units (the "
                       "reconstruction's work)"}[workload] + " (oracle coder + crc_windows)"
    else:
        k, p = (3, 2) if workload == "c1" else (6, 3)
        d = cells(SEED, 900, k, n)
        job, data_bytes = (lambda: oracle.rs_encode(k, p, d)), k * n
        what = f"rs-{k}-{p}-1024k stripes encoded (oracle rs_encode: C restatement of RSUtil.encodeData)"
    job()  # warm the tables
    done = [0] * threads
    stop = time.perf_counter() + budget_s

    def worker(i):
        while time.perf_counter() < stop:
            job()
            done[i] += 1

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    units = sum(done)
    return {"value": round(units * data_bytes / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{units} {what}, {threads} threads sharing one coder, {el:.1f} s wall (gcc -O3)"}


# ------------------------------------------------------------------------------------------ main


def main():
    args = parse()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OZEC_BENCH_SAME_DEVICE=1 + OZEC_DIST_BACKEND=gloo rehearse the N-rank path on a one-GPU box
    dev_idx = 0 if os.environ.get("OZEC_BENCH_SAME_DEVICE") == "1" else local
    torch.cuda.set_device(dev_idx)
    backend = os.environ.get("OZEC_DIST_BACKEND", "nccl")
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    if args.tune:
        from ozone_amd import _lib
        for kv in args.tune:
            key, val = kv.split("=", 1)
            if _lib.lib().ozec_set_tuning(key.encode(), int(val)) != 0:
                raise SystemExit(f"unknown tuning knob {kv}")
    erased = [int(e) for e in args.erased.split(",")]
    if len(erased) != 4 or len(set(erased)) != 4 or not all(0 <= e < 14 for e in erased):
        raise SystemExit("--erased: four distinct unit indexes of rs-10-4 (0..13)")
    wl = Workload(args.workload, rank, args.stripes, args.threads, erased)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        wl.step()
    barrier()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record()
        wl.step()
        b.record()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    from ozone_amd.shard import max_over_ranks
    elapsed = max_over_ranks(elapsed, dist, device="cuda" if backend == "nccl" else "cpu")
    value = wl.data_bytes * world * args.steps / elapsed / 1e9
    achieved = wl.alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    if os.path.exists(tf):
        with open(tf) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    result = {
        "metric": METRIC if args.workload == "c2" else f"{args.workload}: data GB/s",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 bytes generated in HBM)",
        "config": dict(wl.config, parallelism=f"stripe-sharded x{world} (independent stripes, no collective)"),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": wl.kernel, "kernel_ms": round(kern_ms, 4),
                     "alg_bytes_per_launch": wl.alg_bytes},
    }
    if args.workload in ("e2e", "queue", "queue_pageable"):
        # the kernel is not the bound here: report the PCIe ceiling beside the value (never the value itself)
        pc = pcie_ceiling(64 * 6 * MIB, 64 * 3 * MIB)
        pc["value_frac_of_duplex_h2d"] = round(value / world / pc["duplex_h2d_GBps"], 4)
        result["pcie"] = pc
        result["roofline"]["note"] = ("e2e: kernel_ms is the whole PCIe-inclusive step; the bound is the link "
                                      "(see pcie), not HBM")
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
