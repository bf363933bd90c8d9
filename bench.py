#!/usr/bin/env python3
"""Benchmark of the MI355X EC + checksum hot path (driver contract: one JSON line on rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|...]

Default workload = BASELINE.json configs[1]: rs-6-3-1024k encode of 4096 stripes per GPU, device-resident.
A "step" is one ozec_encode_batch over the GPU's 4096 stripes (24 GiB of data cells read, 12 GiB of parity
written).

Multi-GPU: one process per GPU.  Under torchrun the ranks come from the environment; with
`--gpus N` and no WORLD_SIZE this script starts the N rank processes itself (before anything touches a GPU) and
waits for them.  A global batch of 4096·N stripes is split into contiguous stripe ranges (ozone_amd.shard
.stripe_range), one per GPU, with no collective on the data path ("scaling": "weak": 4096 stripes per GPU).
torch.distributed only carries barriers and max-over-ranks reductions of the timings.

value        = data bytes of all ranks / max-over-ranks wall time of the K timed steps (GB = 1e9 B)
roofline     = algorithmic bytes per launch / mean kernel time from HIP events on the launch stream (max over
               ranks), against 8.0 TB/s; `traffic` = HBM bytes per launch of the same kernel measured by this run
               in two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, gfx950 correction), N = 1 only
e2e          = BASELINE configs[4] (C5) at the same N: one batch of 8192 rs-6-3-1024k stripes in shared host
               memory, each GPU encoding + CRC32C'ing its stripe range from NUMA-local pinned pages
               (ozec_encode_crc_host_batch), parity and CRCs back into the batch
cpu_baseline = (rank 0, N = 1) oracle/cpu_baseline.c compiled -march=native on this host and run on a bounded
               sample of the same work with T = the CPUs this process may use and with 1 thread
"""
import argparse
import ctypes
import json
import mmap
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tests"))
from devcopy import to_dev, to_host  # noqa: E402  (host <-> device through pinned staging, never a pageable DMA)

MIB = 1 << 20
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
SEED = 0x00EC5EED
METRIC = "EC encode GB/s (data bytes) rs-6-3-1024k @1/8 GPUs + % HBM roofline"
WORKLOADS = ["c1", "c2", "c3", "c3r", "c3r_host", "c4", "c4s", "c5", "c5dev", "crc", "verify", "host", "queue", "queue_pageable",
             "stream", "legs", "jni", "tail"]
# the device-resident legs of the default line, each timed like the headline (every kernel north_star
# names under the driver's clock): (workload, erased units) -- C5dev rs-6-3 encode + CRC32C, C3r with both erasure sets
# of BASELINE.md, C3 rs-10-4 decode with both sets (RSRawDecoder.java:87-101), CRC32C compute and verify per 16 KiB
# window (Checksum.java:157-200, :272-297), C4 xor-2-1 + CRC32C over block groups (XORRawEncoder.java:39-85)
LEGS = [("c5dev", None), ("c3r", (0, 1, 2, 3)), ("c3r", (1, 4, 10, 13)), ("c3", (0, 1, 2, 3)), ("c3", (1, 4, 10, 13)),
        ("crc", None), ("verify", None), ("c4", None)]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 20 untimed steps: short launches (the 1.4 ms CRC batch) run ~5 % slow until the clock has settled
    # (scripts/event_bracket.py: first timed launches 1.47 ms, settled 1.39 ms)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=WORKLOADS)
    ap.add_argument("--stripes", type=int, default=0, help="override the per-GPU stripe count (profiling only)")
    ap.add_argument("--erased", default="0,1,2,3",
                    help="c3/c3r: erased unit indexes of rs-10-4 (SURVEY 8(d): 0,1,2,3 all data; 1,4,10,13 mixed)")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="wall budget of each CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the C5 end-to-end leg of the default line")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 PMC traffic passes")
    ap.add_argument("--no-legs", action="store_true", help="skip the device-resident legs (LEGS) of the default line")
    ap.add_argument("--no-inproc", action="store_true",
                    help="skip the in-process multi-GPU C5 leg (one process, libozec's device list over all N GPUs)")
    ap.add_argument("--no-jni", action="store_true", help="skip the JNI per-call rows of the default line")
    ap.add_argument("--full-line", action="store_true",
                    help="print the whole record on stdout (default: a compact line, the record in gpurun_out/"
                         "bench_full.json or $OZEC_BENCH_FULL)")
    ap.add_argument("--e2e-stripes", type=int, default=8192, help="C5 batch size (all GPUs together)")
    ap.add_argument("--e2e-steps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=0, help="C5: stripes per pipelined chunk (0 = library default)")
    ap.add_argument("--threads", type=int, default=1, help="host workload: caller threads sharing one coder")
    ap.add_argument("--host-pinned", action="store_true",
                    help="host workload: every caller's cells in pinned memory (ozec_host_alloc): DMA in place")
    ap.add_argument("--queue-batch", type=int, default=32, help="queue workloads: stripes per GPU batch")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="ozec_set_tuning knob (A/B and profiling runs only; defaults are the measured best)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------ launch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker_specs(n, argv, environ, port):
    """(argv, env, keep_stdout) of each of the n rank processes launch_workers starts: the same command line, the
    torchrun variables of rank r (RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n, rendezvous on
    127.0.0.1:port), and only rank 0's stdout kept (it prints the one JSON line)."""
    specs = []
    for r in range(n):
        env = dict(environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        specs.append(([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env, r == 0))
    return specs


def launch_workers(args):
    """--gpus N without torchrun: start N rank processes (this process never touches a GPU) and wait."""
    same = os.environ.get("OZEC_BENCH_SAME_DEVICE") == "1"
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if not same and ndev < args.gpus:
        raise SystemExit(f"--gpus {args.gpus}: only {ndev} visible GPU(s)")
    procs = [subprocess.Popen(cmd, env=env, stdout=None if keep else subprocess.DEVNULL)
             for cmd, env, keep in worker_specs(args.gpus, sys.argv[1:], os.environ, _free_port())]
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def node_cpus(node):
    try:
        text = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in text.split(","):
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def bind_process_to_gpu_node(dev):
    """Run this rank on the CPUs of its GPU's NUMA node (the staging copies and DMA descriptors live there)."""
    from ozone_amd.stripe_queue import device_numa_node
    node = device_numa_node(dev)
    if node < 0:
        return node
    want = node_cpus(node) & os.sched_getaffinity(0)
    if want:
        os.sched_setaffinity(0, want)
    return node


def usable_cpus():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def host_info():
    info = {"cpus_usable": usable_cpus(), "cpus_online": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            key, _, val = line.partition(":")
            if key.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "NUMA node(s)"):
                info[key.strip()] = val.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


# ------------------------------------------------------------------------------------------ workloads


class Workload:
    """Allocates device-resident inputs once; step() launches one batch on the current stream."""

    def __init__(self, name, rank, world, stripes_override, threads=1, erased=(0, 1, 2, 3), queue_batch=32):
        from ozone_amd import checksum as ck
        from ozone_amd import rawcoder as rc
        from ozone_amd.shard import stripe_range
        self.name = name
        self.stream = torch.cuda.current_stream()
        dev = torch.device("cuda", torch.cuda.current_device())
        n = MIB
        self.n = n
        if name == "host":
            k, p, S = 6, 3, stripes_override or 64
            T = max(1, threads)
            rng = np.random.default_rng(rank)
            if HOST_PINNED:  # one pinned pool per caller, its cells at one stride (a writer's buffer pool)
                from ozone_amd.stripe_queue import host_alloc
                self._pools = [host_alloc((k + p) * n) for _ in range(T)]
                cellv = [[pl.array[i * n:(i + 1) * n] for i in range(k + p)] for pl in self._pools]
                for t in range(T):
                    for i in range(k):
                        cellv[t][i][:] = rng.integers(0, 256, n, dtype=np.uint8)
                self.hd = [cv[:k] for cv in cellv]
                self.hp = [cv[k:] for cv in cellv]
            else:
                self.hd = [[rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)] for _ in range(T)]
                self.hp = [[np.empty(n, np.uint8) for _ in range(p)] for _ in range(T)]
            self.k, self.p, self.S = k, p, S
            enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + p) * n
            self.kernel = "gf_code_vec<6,3> (+pageable->pinned staging, H2D, D2H, per stripe)"
            self.config = {"workload": f"rs-6-3-1024k encode through the host-pointer ABI (ozec_encode: the JNI "
                                       f"drop-in path), {S} single-stripe calls from {T} threads sharing one coder"
                                       + (", cells in pinned memory (DMA in place)" if HOST_PINNED else
                                          ", cells in pageable memory (staged)"),
                           "stripes": S, "threads": T, "pinned": HOST_PINNED}

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
        if name == "c3r_host":
            # reconstruction end to end from pinned host memory: the reconstruction coordinator's read buffers
            # (ECReconstructionCoordinator.java:240-352) -> H2D of the 10 units read -> fused verify + decode + CRC
            # -> D2H of the 4 rebuilt units, their CRCs and the per-stripe verdicts
            from ozone_amd.stripe_queue import host_alloc
            k, p, S = 10, 4, stripes_override or 512
            self.erased = sorted(erased)
            present = [u for u in range(k + p) if u not in self.erased]
            self.bpc, self.crc_type = 16384, ck.ChecksumType.CRC32C
            nwin = n // self.bpc
            dunits = torch.empty((S, k + p, n), dtype=torch.uint8, device=dev)
            for s0 in range(0, S, 64):  # data cells, then parity on the GPU (the stored stripes)
                c = min(64, S - s0)
                for i in range(c):
                    rc.fill_splitmix64_cells(dunits[s0 + i], n, k, n, SEED, (rank * S + s0 + i) * k)
            encr = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
            encr.encode_batch(dunits, (k + p) * n, n, dunits[:, k:], (k + p) * n, n, S, n)
            dstored = torch.empty((S, k + p, nwin), dtype=torch.int32, device=dev)
            ck.checksum_windows_batch(self.crc_type, dunits, n, S * (k + p), n, self.bpc, dstored)
            torch.cuda.synchronize()
            self._pool = [host_alloc(S * (k + p) * n), host_alloc(S * 4 * n), host_alloc(S * 4 * nwin * 4),
                          host_alloc(S * (k + p) * nwin * 4), host_alloc(S * 4)]
            hin, hout, hocrc, hexp, hmis = (pb.array for pb in self._pool)
            torch.from_numpy(hin).copy_(dunits.reshape(-1))
            torch.from_numpy(hexp).copy_(dstored.reshape(-1).view(torch.uint8))
            del dunits, dstored
            torch.cuda.empty_cache()
            self.k, self.p, self.S = k, p, S
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + 4) * n + S * (k + 4) * nwin * 4
            self.kernel = "encode_crc_nb<10,4> (+H2D of the 10 units read, D2H of the 4 rebuilt, pipelined)"
            self.config = {"workload": f"rs-10-4-1024k reconstruction end to end from pinned host memory: H2D of the 10 "
                                       f"units read, verify CRC32C + decode 4 + CRC32C of rebuilt units "
                                       f"{{{','.join(map(str, self.erased))}}}, D2H, {S} stripes",
                           "codec": "rs", "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "bytes_per_checksum": self.bpc}
            dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
            hexp32, hocrc32, hmis32 = hexp.view(np.uint32), hocrc.view(np.uint32), hmis.view(np.int32)

            def step():
                dec.reconstruct_crc_host_batch(hin, (k + p) * n, n, present, self.erased, hout, 4 * n, n, S, n,
                                               self.crc_type, self.bpc, hocrc32, h_expected=hexp32, h_mismatch=hmis32)
            self._step = step
            self._check = lambda: bool((hmis32 == -1).all())
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
            # a writer's cell pool: one allocation carved into per-stripe slabs of k data then p parity cells back to
            # back; stripes submitted in pool order coalesce into one 2D copy per direction and run of 8 stripes
            whole = buf(pool * (k + p) * n)
            slabs = [whole[i * (k + p) * n:(i + 1) * (k + p) * n] for i in range(pool)]
            self.qd = [[sl[j * n:(j + 1) * n] for j in range(k)] for sl in slabs]
            for st in self.qd:
                for a in st:
                    a[:] = rng.integers(0, 256, n, dtype=np.uint8)
            self.qp = [[sl[(k + r) * n:(k + r + 1) * n] for r in range(p)] for sl in slabs]
            self.qc = [buf((k + p) * nwin * 4, np.uint32) for _ in range(pool)]
            enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
            self.q = StripeQueue(enc, n, queue_batch, self.crc_type, self.bpc)
            self.k, self.p, self.S = k, p, S
            self.data_bytes = S * k * n
            self.alg_bytes = S * (k + p) * n
            self.kernel = "encode_crc_nb<6,3> via ozec_stripe_queue (+H2D/D2H 2D copies per run of stripes)"
            self.config = {"workload": f"rs-6-3-1024k + CRC32C/16 KiB through the stripe queue (SURVEY 8(f) row 3) "
                                       f"from {'pinned' if pinned else 'pageable'} host cells, {S} stripes, "
                                       f"batches of {queue_batch}", "stripes": S, "stripes_per_batch": queue_batch}

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
        elif name in ("c2", "c5dev"):
            k, p, S = 6, 3, stripes_override or 4096
        elif name in ("c3", "c3r"):
            k, p, S = 10, 4, stripes_override or 2048
        elif name in ("c4", "c4s"):
            k, p, S = 2, 1, stripes_override or 16 * 256
        else:  # crc / verify
            k, p, S = 1, 0, stripes_override or 8192
        self.k, self.p, self.S = k, p, S
        # this rank's share of the global batch (S stripes per GPU, contiguous ranges: SURVEY 8(e))
        self.lo, self.hi = stripe_range(S * world, rank, world)
        self.bpc = 16384
        self.nwin = n // self.bpc
        self.crc_type = ck.ChecksumType.CRC32C
        if name in ("crc", "verify"):
            self.data = torch.empty((S, n), dtype=torch.uint8, device=dev)
            rc.fill_splitmix64_cells(self.data, n, S, n, SEED, self.lo)
            self.crcs = torch.empty((S, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * n
            if name == "crc":
                self.alg_bytes = S * n + S * self.nwin * 4
                self.kernel = "crc_windows_g26s"
                self.config = {"workload": "CRC32C per 16 KiB window, device-resident", "cells": S, "cell_bytes": n,
                               "bytes_per_checksum": self.bpc}
                self._step = lambda: ck.checksum_windows_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs)
            else:
                ck.checksum_windows_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs)
                self.mism = torch.empty(S, dtype=torch.int32, device=dev)
                # every data byte and every stored CRC read, one first-failure index per cell written
                self.alg_bytes = S * n + S * self.nwin * 4 + S * 4
                self.kernel = "crc_windows_g26s"
                self.config = {"workload": "CRC32C verify per 16 KiB window against stored CRCs (datanode scanner, "
                                           "SURVEY 8(f) row 2), device-resident", "cells": S, "cell_bytes": n,
                               "bytes_per_checksum": self.bpc}
                self._step = lambda: ck.checksum_verify_batch(self.crc_type, self.data, n, S, n, self.bpc, self.crcs,
                                                              self.mism)
            torch.cuda.synchronize()
            return
        units = k + p
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, "rs" if k != 2 else "xor"))
        self.enc = enc
        if name == "c4":
            # block-major, as a datanode stores EC block groups: 16 groups of 2 data blocks + 1 parity block of
            # 256 MiB (one block file per unit), unit stride 256 MiB, stripe s of a group at offset s MiB
            G, B = S // 256, 256
            self.blocks = torch.empty((G, units, B * n), dtype=torch.uint8, device=dev)
            for u in range(k):
                rc.fill_splitmix64_cells(self.blocks[:, u], units * B * n, G, B * n, SEED, self.lo + u * G * 1000)
            self.crcs = torch.empty((G, B, units, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n + S * units * self.nwin * 4
            self.kernel = "encode_crc_g26<2,1>"
            self.config = {"workload": "xor-2-1-1024k + CRC32C/16 KiB over 256 MiB blocks, 16 block groups x 256 "
                                       "stripes, fused, device-resident", "codec": "xor", "data_units": k,
                           "parity_units": p, "cell_bytes": n, "stripes": S, "bytes_per_checksum": self.bpc,
                           "layout": "block-major: [group][unit][256 MiB block], unit stride 256 MiB"}
            us = B * n

            self._step = lambda: enc.encode_crc_block_groups(self.blocks, units * us, us, G, B, n, self.crc_type,
                                                             self.bpc, self.crcs)
            torch.cuda.synchronize()
            return
        # HBM layout: stripe-major, units contiguous: unit u of stripe s at s*(k+p)*n + u*n
        self.units = torch.empty((S, units, n), dtype=torch.uint8, device=dev)
        for u in range(k):
            rc.fill_splitmix64_cells(self.units[:, u], units * n, S, n, SEED, u * S * world + self.lo)
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
            self.config = {"workload": f"rs-6-3-1024k encode, {S} stripes per GPU, device-resident (BASELINE configs[1])",
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
            self.kernel = "encode_crc_nb<10,4> (nibble tables, fused.hip)"
            self.config = {"workload": "rs-10-4-1024k reconstruction: verify CRC32C of 10 read units + decode 4 + "
                                       f"CRC32C of rebuilt units {{{','.join(map(str, self.erased))}}}, {S} stripes, "
                                       "fused, device-resident",
                           "codec": "rs", "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "bytes_per_checksum": self.bpc}
            self._step = lambda: self.dec.reconstruct_crc_batch(
                self.units, stride, n, present, self.erased, self.out, 4 * n, n, S, n, self.crc_type, self.bpc,
                self.out_crc, d_expected=self.stored, d_mismatch=self.mism)
            self._check = lambda: bool((self.mism == -1).all().item())  # every stripe's read units verified
        else:  # c4s (xor-2-1 stripe-major) / c5dev (rs-6-3): fused encode + CRC, device-resident
            self.crcs = torch.empty((S, units, self.nwin), dtype=torch.int32, device=dev)
            self.data_bytes = S * k * n
            self.alg_bytes = S * units * n + S * units * self.nwin * 4
            self.kernel = "encode_crc_g26<2,1>" if k == 2 else f"encode_crc_nb<{k},{p}> (nibble tables, fused.hip)"
            wl = ("xor-2-1-1024k + CRC32C/16 KiB, stripe-major" if name == "c4s"
                  else "rs-6-3-1024k encode + CRC32C/16 KiB (the C5 kernel without PCIe)")
            self.config = {"workload": f"{wl}, {S} stripes, fused, device-resident", "codec": "xor" if k == 2 else "rs",
                           "data_units": k, "parity_units": p, "cell_bytes": n, "stripes": S,
                           "bytes_per_checksum": self.bpc}
            self._step = lambda: enc.encode_crc_batch(self.units, stride, n, self.units[:, k:], stride, n, S, n,
                                                      self.crc_type, self.bpc, self.crcs)
        torch.cuda.synchronize()

    def step(self):
        self._step()

    def free(self):
        for a in ("units", "blocks", "data", "crcs", "stored", "out", "out_crc", "mism"):
            if hasattr(self, a):
                delattr(self, a)
        torch.cuda.empty_cache()


# ------------------------------------------------------------------------------------------ C5 end to end


_KEEP_MAPPED = []  # host mappings held by ctypes views until the process exits


class HostBatch:
    """One batch of rs-6-3-1024k stripes in host memory shared by every rank ([stripe][9 units][1 MiB], then a
    CRC area with one page-aligned slot per rank), so the ranks really split ONE batch.  Each rank places its own
    stripe range on its GPU's NUMA node and pins it (ozec_host_register).  Falls back to a private mapping of
    the rank's own range when /dev/shm cannot hold the batch."""

    def __init__(self, S, rank, world, dist, dev, k=6, p=3, n=MIB, bpc=16384):
        from ozone_amd.shard import stripe_range
        from ozone_amd.stripe_queue import host_register
        self.k, self.p, self.n, self.S = k, p, n, S
        self.units, self.nwin = k + p, -(-n // bpc)
        self.stripe_bytes = self.units * n
        self.lo, self.hi = stripe_range(S, rank, world)
        per = -(-S // world)
        self.crc_slot = -(-(per * self.units * self.nwin * 4) // (2 * MIB)) * (2 * MIB)
        total = S * self.stripe_bytes + world * self.crc_slot
        name = None
        try:
            free = os.statvfs("/dev/shm").f_bavail * os.statvfs("/dev/shm").f_frsize
        except OSError:
            free = 0
        self.shared = free > total + (8 << 30)
        if self.shared:
            name = f"/dev/shm/ozec_c5_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}" if rank == 0 else None
            if dist is not None:
                obj = [name]
                dist.broadcast_object_list(obj, src=0)
                name = obj[0]
            if rank == 0:
                fd = os.open(name, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
                os.ftruncate(fd, total)
                os.close(fd)
            if dist is not None:
                dist.barrier()
            fd = os.open(name, os.O_RDWR)
            self.mm = mmap.mmap(fd, total, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
            os.close(fd)
            # every rank has it mapped: unlink now, so the memory goes away with the last mapping even if a rank dies
            if dist is not None:
                dist.barrier()
            if rank == 0:
                os.unlink(name)
            self.name = name
            self._anchor = ctypes.c_char.from_buffer(self.mm)
            self.base = ctypes.addressof(self._anchor)
            self.data_off = self.lo * self.stripe_bytes
            self.crc_off = S * self.stripe_bytes + rank * self.crc_slot
        else:
            self.name = None
            own = (self.hi - self.lo) * self.stripe_bytes + self.crc_slot
            self.mm = mmap.mmap(-1, max(own, mmap.PAGESIZE), mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            self._anchor = ctypes.c_char.from_buffer(self.mm)
            self.base = ctypes.addressof(self._anchor)
            self.data_off = 0
            self.crc_off = (self.hi - self.lo) * self.stripe_bytes
        self.rank, self.dev = rank, dev
        self.data_len = (self.hi - self.lo) * self.stripe_bytes
        self.registered = []
        t0 = time.perf_counter()
        for off, ln in ((self.data_off, self.data_len), (self.crc_off, self.crc_slot)):
            if ln:
                host_register(self.base + off, ln, dev)
                self.registered.append(self.base + off)
        self.register_s = time.perf_counter() - t0

    def fill(self, enc_dev):
        """Synthetic data cells (splitmix64, stream = global stripe id * k + unit) generated on the GPU and DMA'd
        into this rank's range; parity and CRC areas are left for the encode."""
        from ozone_amd import rawcoder as rc
        k, n, C = self.k, self.n, 64
        tmp = torch.zeros((C, self.units, n), dtype=torch.uint8, device=enc_dev)  # parity cells stay zero
        host = np.frombuffer((ctypes.c_uint8 * self.data_len).from_address(self.base + self.data_off), np.uint8)
        for s0 in range(self.lo, self.hi, C):
            c = min(C, self.hi - s0)
            for i in range(c):  # cell (stripe s, unit u) = splitmix64 stream s * k + u
                rc.fill_splitmix64_cells(tmp[i], n, k, n, SEED, (s0 + i) * k)
            v = host[(s0 - self.lo) * self.stripe_bytes:(s0 - self.lo + c) * self.stripe_bytes]
            torch.from_numpy(v).copy_(tmp[:c].reshape(-1))  # one DMA into the registered range
        torch.cuda.synchronize()
        del tmp

    def placement(self):
        """NUMA node of this rank's first and last data page (after the run)."""
        from ozone_amd.stripe_queue import page_node
        if not self.data_len:
            return []
        return [page_node(self.base + self.data_off), page_node(self.base + self.data_off + self.data_len - 1)]

    def close(self, dist):
        """Unregister; the mapping itself stays until the process exits (a ctypes view anchors it, and the bench ends
        right after); the shared-memory object was unlinked at creation, so its pages go with the last rank."""
        from ozone_amd.stripe_queue import host_unregister
        for a in self.registered:
            host_unregister(a)
        self.registered = []
        _KEEP_MAPPED.append((self.mm, self._anchor))
        if dist is not None:
            dist.barrier()


def e2e_leg(args, rank, world, dist, dev, backend, cpu_group=None):
    """BASELINE configs[4] (C5): rs-6-3-1024k encode + CRC32C of one 8192-stripe batch in pinned host memory,
    sharded across the GPUs by contiguous stripe ranges, end to end (H2D + fused kernel + D2H): one process per GPU.
    Then (unless --no-inproc) the same batch through ONE process driving all N GPUs (in_process_leg).  Returns
    (multi-process result, in-process result or None)."""
    from ozone_amd import checksum as ck
    from ozone_amd import rawcoder as rc
    from ozone_amd.shard import max_over_ranks
    S = args.e2e_stripes
    hb = HostBatch(S, rank, world, dist, dev)
    try:
        hb.fill(torch.device("cuda", dev))
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(6, 3))
        n, k, sb = hb.n, hb.k, hb.stripe_bytes
        mine = hb.hi - hb.lo
        d0 = hb.base + hb.data_off

        def step():
            if mine:
                enc.encode_crc_host_batch(d0, sb, n, d0 + k * n, sb, n, mine, n, ck.ChecksumType.CRC32C, 16384,
                                          hb.base + hb.crc_off, False, args.chunk)

        step()  # warm-up: device buffers of the pipeline, first-touch of nothing (pages are pinned)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.e2e_steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if dist is not None:
            dist.barrier()
        el_max = max_over_ranks(el, dist, device="cuda" if backend == "nccl" else "cpu")
        # a spot check of the last stripe this rank encoded, against the device coder on the same cells
        ok = True
        if mine:
            last = np.frombuffer((ctypes.c_uint8 * sb).from_address(d0 + (mine - 1) * sb), np.uint8).reshape(9, n)
            cells = to_dev(last[:k], f"cuda:{dev}").unsqueeze(0)
            par = enc.encode_stripes(cells)
            torch.cuda.synchronize()
            ok = bool((to_host(par[0]) == last[k:]).all())
        res = {"workload": "rs-6-3-1024k encode + CRC32C/16 KiB, one batch of %d stripes in shared host memory, "
                           "contiguous stripe range per GPU, pinned NUMA-local pages, H2D + fused kernel + D2H "
                           "(BASELINE configs[4])" % S,
               "value": round(S * k * n * args.e2e_steps / el_max / 1e9, 2), "unit": "GB/s (data bytes)",
               "ms_per_step": round(el_max / args.e2e_steps * 1e3, 2), "steps": args.e2e_steps,
               "stripes": S, "stripes_per_gpu": [mine], "shared_batch": hb.shared,
               "register_s": round(hb.register_s, 2), "parity_spot_check": ok,
               "numa": {"gpu_node": None, "data_page_nodes": hb.placement()}}
        from ozone_amd.stripe_queue import device_numa_node
        res["numa"]["gpu_node"] = device_numa_node(dev)
        res["per_rank"] = gather_per_rank({"elapsed_s": round(el, 4), "stripes": mine,
                                           "GBps": round(mine * k * n * args.e2e_steps / el / 1e9, 2),
                                           "register_s": round(hb.register_s, 3), "gpu_node": res["numa"]["gpu_node"],
                                           "data_page_nodes": res["numa"]["data_page_nodes"]}, dist)
        if dist is not None:
            allr = [None] * world
            dist.all_gather_object(allr, {"mine": mine, "numa": res["numa"], "ok": ok})
            res["stripes_per_gpu"] = [a["mine"] for a in allr]
            res["numa"] = [a["numa"] for a in allr]
            res["parity_spot_check"] = all(a["ok"] for a in allr)
        pc = pcie_ceiling(64 * 6 * MIB, 64 * 3 * MIB)
        res["pcie_per_gpu"] = pc
        res["frac_of_duplex_h2d_link"] = round(res["value"] / world / pc["duplex_h2d_GBps"], 4)
        inproc = None
        if not args.no_inproc:
            log("C5 end-to-end leg, one process over all GPUs")
            try:
                inproc = in_process_leg(args, hb, rank, world, dist, cpu_group, pc)
            except Exception as e:  # the multi-process figure stands on its own
                inproc = {"error": f"{type(e).__name__}: {e}"}
        return res, inproc
    finally:
        hb.close(dist)


def in_process_leg(args, hb, rank, world, dist, cpu_group, pc):
    """north_star: "a batch is partitioned across the 8 MI355X of one node as per-GPU streams" -- inside the drop-in
    process, as Ozone runs it (one JVM per datanode or client making a coder per stream, ECKeyOutputStream.java:117,
    ECReconstructionCoordinator.java:240-352).  Rank 0 alone sets libozec's device list to the node's N GPUs
    (ozec_set_devices) and runs the whole C5 batch through ONE ozec_encode_crc_host_batch call per step, which cuts it
    into N contiguous stripe ranges run by per-GPU pipelines on threads of their own (capi.cpp host_batch_split); the
    other ranks wait on a CPU barrier and leave their GPUs idle.  The batch is the one the ranks just encoded (each
    range's pages already on its GPU's NUMA node); rank 0 registers the other ranks' ranges in its own process."""
    from ozone_amd import _lib
    from ozone_amd import checksum as ck
    from ozone_amd import rawcoder as rc
    from ozone_amd.shard import stripe_range
    from ozone_amd.stripe_queue import device_numa_node, host_alloc, host_register, host_unregister, page_node

    def cpu_barrier():
        if dist is not None:
            dist.barrier(group=cpu_group)
    if world > 1 and not hb.shared:
        cpu_barrier()
        return {"error": "the batch is not in shared memory (/dev/shm too small): rank 0 cannot see every range"}
    if rank != 0:
        cpu_barrier()
        return None
    try:
        S, sb, n, k = hb.S, hb.stripe_bytes, hb.n, hb.k
        same = os.environ.get("OZEC_BENCH_SAME_DEVICE") == "1"
        devs = [0] * world if same else list(range(world))
        nwin = hb.nwin
        base = hb.base  # the shared mapping: stripe s at base + s * sb in every rank
        extra = []
        t0 = time.perf_counter()
        for r in range(1, world):  # the other ranks' ranges, one registration each (= libozec's part r)
            lo, hi = stripe_range(S, r, world)
            if hi > lo:
                host_register(base + lo * sb, (hi - lo) * sb, -1)  # pages already on GPU r's node: no move
                extra.append(base + lo * sb)
        reg_s = time.perf_counter() - t0
        crc = host_alloc(S * hb.units * nwin * 4, devs[0])
        saved_aff = os.sched_getaffinity(0)
        if ORIG_AFFINITY:
            os.sched_setaffinity(0, ORIG_AFFINITY)  # the per-GPU pipeline threads of both sockets
        L = _lib.lib()
        prev_policy = L.ozec_device_policy()
        try:
            rc.set_devices(devs)
            rc.set_device_policy("current")  # the coder on device 0, so part r (= rank r's range) runs on GPU r
            enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, hb.p))
            rc.set_device_policy(prev_policy)

            def step():
                enc.encode_crc_host_batch(base, sb, n, base + k * n, sb, n, S, n, ck.ChecksumType.CRC32C, 16384,
                                          crc.array.ctypes.data, False, args.chunk)
            step()  # warm-up: every GPU's pipeline buffers
            t0 = time.perf_counter()
            for _ in range(args.e2e_steps):
                step()
            el = time.perf_counter() - t0
            # spot check: the last stripe of every part against the device coder on GPU 0
            ok = True
            parts = []
            for i, d in enumerate(devs):
                lo, hi = stripe_range(S, i, len(devs))
                parts.append({"device": d, "stripes": hi - lo, "gpu_node": device_numa_node(d),
                              "data_page_nodes": [page_node(base + lo * sb), page_node(base + hi * sb - 1)]
                              if hi > lo else []})
                if hi > lo:
                    last = np.frombuffer((ctypes.c_uint8 * sb).from_address(base + (hi - 1) * sb), np.uint8).reshape(
                        hb.units, n)
                    cells = to_dev(last[:k], f"cuda:{d}").unsqueeze(0)
                    par = enc.encode_stripes(cells)
                    torch.cuda.synchronize()
                    ok = ok and bool((to_host(par[0]) == last[k:]).all())
        finally:
            rc.set_devices([devs[0]])
            L.ozec_set_device_policy(prev_policy)
            os.sched_setaffinity(0, saved_aff)
            for a in extra:
                host_unregister(a)
            crc.free()
        ndev = len(set(devs))
        value = S * k * n * args.e2e_steps / el / 1e9
        return {"workload": "rs-6-3-1024k encode + CRC32C/16 KiB, the same %d-stripe batch through ONE process: "
                            "ozec_set_devices(%s), one ozec_encode_crc_host_batch call per step split into contiguous "
                            "stripe ranges on per-GPU pipeline threads" % (S, devs),
                "value": round(value, 2), "unit": "GB/s (data bytes)",
                "ms_per_step": round(el / args.e2e_steps * 1e3, 2), "steps": args.e2e_steps, "n_gpus": ndev,
                "devices": devs, "parts": parts, "register_other_ranges_s": round(reg_s, 2),
                "parity_spot_check": ok,
                "frac_of_duplex_h2d_link": round(value / ndev / pc["duplex_h2d_GBps"], 4),
                "note": "per-GPU pipelines run concurrently inside one call; per-part times are not separated"}
    finally:
        cpu_barrier()


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
            "note": "contiguous pinned DMA copies of the same volumes, one H2D and one D2H stream"}


# ------------------------------------------------------------------------------------------ CPU baseline

_CPU_BASELINE_BIN = None


def _cpu_baseline_bin():
    """oracle/cpu_baseline.c + oracle/ozec_oracle.c built for THIS host (-march=native), falling back to the
    portable build from build()."""
    global _CPU_BASELINE_BIN
    if _CPU_BASELINE_BIN:
        return _CPU_BASELINE_BIN
    odir = os.path.join(ROOT, "oracle")
    out = os.path.join(tempfile.mkdtemp(prefix="ozec_cpub_"), "cpu_baseline")
    cmd = ["gcc", "-O3", "-march=native", "-std=gnu11", "-o", out, os.path.join(odir, "cpu_baseline.c"),
           os.path.join(odir, "ozec_oracle.c"), "-lz", "-lpthread"]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=120)
        _CPU_BASELINE_BIN = (out, "gcc -O3 -march=native")
    except (OSError, subprocess.SubprocessError):
        _CPU_BASELINE_BIN = (os.path.join(odir, "cpu_baseline"), "gcc -O3 -march=x86-64-v3 (prebuilt)")
    return _CPU_BASELINE_BIN


CPU_WHAT = {
    "c1": "rs-3-2-1024k stripes encoded (RSUtil.encodeData table loop, oracle restatement)",
    "c2": "rs-6-3-1024k stripes encoded (RSUtil.encodeData table loop, oracle restatement)",
    "c3": "rs-10-4-1024k stripes decoded, 4 erased (RSRawDecoder + RSUtil.encodeData)",
    "c3r": "rs-10-4-1024k reconstructions: CRC32C verify of 10 units + decode 4 + CRC32C of the 4 rebuilt",
    "c4": "xor-2-1-1024k stripes coded + CRC32C/16 KiB of all 3 units",
    "c5": "rs-6-3-1024k stripes encoded + CRC32C/16 KiB of all 9 units",
    "crc": "1 MiB cells checksummed as CRC32C/16 KiB windows (SSE4.2 crc32, 3 streams: the JDK CRC32C intrinsic)",
    "verify": "1 MiB cells verified against stored CRC32C/16 KiB windows (SSE4.2 crc32)",
}


def cpu_baseline(workload, budget_s):
    """The reference's CPU path timed on this host's cores (RawErasureCoderBenchmark.java:182-236 definitions:
    threads share one coder, data bytes counted): T = every CPU this process may use, and 1 thread."""
    wl = {"c4s": "c4", "c5dev": "c5", "host": "c2", "queue": "c5", "queue_pageable": "c5", "stream": "c2",
          "c3r_host": "c3r"}.get(
        workload, workload)
    exe, flags = _cpu_baseline_bin()
    T = usable_cpus()
    res = {}
    for t in (T, 1):
        out = subprocess.run([exe, wl, str(t), str(budget_s)], capture_output=True, text=True, timeout=budget_s + 120)
        if out.returncode != 0:
            raise RuntimeError(f"cpu_baseline {wl} failed: {out.stderr.strip()}")
        res[t] = json.loads(out.stdout)
    hi, one = res[T], res[1]
    info = host_info()
    return {"value": round(hi["GBps"], 3), "unit": "GB/s", "cores": T, "kind": "port",
            "value_1_thread": round(one["GBps"], 3),
            "sample": f"{hi['units']} {CPU_WHAT[wl]} in {hi['seconds']:.1f} s on {T} threads sharing one coder "
                      f"({one['units']} in {one['seconds']:.1f} s on 1 thread); oracle/cpu_baseline.c, {flags}",
            "host": info}


# ------------------------------------------------------------------------------------------ live PMC traffic

HOST_PINNED = False  # --host-pinned (host workload)
ORIG_AFFINITY = None  # the CPUs the process was started with, before each rank binds itself to its GPU's node
TUNE = []  # --tune KEY=VALUE knobs, also handed to the JNI harness (OZEC_TUNE)

KERNEL_PAT = {"c1": "gf_code_vec<3, 2", "c2": "gf_code_vec<6, 3", "c3": "gf_code_vec<10, 4",
              "c3r": ("encode_crc_nb<10, 4", "encode_crc_lv<10, 4", "encode_crc_g26<10, 4"), "c4": "encode_crc_g26<2, 1",
              "c4s": "encode_crc_g26<2, 1", "c5dev": ("encode_crc_nb<6, 3", "encode_crc_lv<6, 3", "encode_crc_g26<6, 3"),
              "crc": "crc_windows_g26s", "verify": "crc_windows_g26s"}


def _kernel_match(pat, name):
    """pat: a name fragment, or a tuple of fragments (the nibble-table, streamed-input or per-window fused kernel)."""
    return any(p in name for p in (pat if isinstance(pat, tuple) else (pat,)))


def log(msg):
    """progress on stderr (stdout carries only the one JSON line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _rocprof_passes(child, tag_opts, timeout=300):
    """Run the bench child command under rocprofv3 once per (tag, options) pass -- counters that do not fit one pass
    get passes of their own -- and return {tag: [csv files]} (the caller removes the parent directory)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        raise OSError("rocprofv3 not found")
    work = tempfile.mkdtemp(prefix="ozec_pmc_")
    env = dict(os.environ, TMPDIR="/tmp")
    env.pop("WORLD_SIZE", None)
    files = {"_dir": work}
    for tag, opts in tag_opts:
        d = os.path.join(work, tag)
        cmd = [prof] + opts + ["--kernel-trace", "--stats", "-d", d, "-o", "run", "--output-format", "csv", "--"] + child
        log(f"rocprofv3 pass {tag}: {' '.join(child[2:6])}")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
        if r.returncode != 0:
            raise OSError(f"rocprofv3 {tag} pass rc={r.returncode}: {r.stderr.strip()[-300:]}")
        files[tag] = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs]
    return files


_PMC_PASSES = (("FETCH_SIZE", ["--pmc", "FETCH_SIZE"]), ("WRITE_SIZE", ["--pmc", "WRITE_SIZE"]), ("stats", []))


FILL_KERNEL = "fill_splitmix64"  # every Workload starts by filling its synthetic cells with it


def _leg_segments(rows, name_key, order_key):
    """The dispatches in launch order cut into one segment per leg: each Workload's set-up starts with a run of
    synthetic-data fill launches, and everything from there to the next leg's fills is that leg's (set-up, warm-up and
    timed steps, with whatever else a step launches: the reconstruction's mismatch finisher, the runtime's memset that
    zeroes a new WorkQueue slot)."""
    rows = sorted(rows, key=lambda r: int(r[order_key]))
    segs = []
    prev_fill = False
    for r in rows:
        fill = FILL_KERNEL in r[name_key]
        if fill and not prev_fill:
            segs.append([])
        if segs:
            segs[-1].append(r)
        prev_fill = fill
    return segs


def _leg_rows(rows, name_key, order_key, pat, leg, steps):
    """The timed dispatches of leg number `leg` of the child run: the last `steps` dispatches of its segment whose
    kernel matches `pat` (set-up launches of the same kernel -- the encode before a decode leg -- come before them)."""
    mine = [r for r in _leg_segments(rows, name_key, order_key)[leg] if _kernel_match(pat, r[name_key])]
    if len(mine) < steps:
        raise IndexError(f"leg {leg}: {len(mine)} dispatches of {pat}, {steps} expected")
    return mine[-steps:]


def _leg_stats(files, pat, leg, steps, alg_bytes):
    """One leg's numbers from the three passes (the child runs the legs in order; `leg` is this one's index)."""
    import csv
    out = {}
    st = [f for f in files["stats"] if f.endswith("kernel_stats.csv")]
    tr = [f for f in files["stats"] if f.endswith("kernel_trace.csv")]
    timed = _leg_rows(list(csv.DictReader(open(tr[0]))), "Kernel_Name", "Start_Timestamp", pat, leg, steps)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    out["rocprof_kernel"] = timed[-1]["Kernel_Name"]
    out["rocprof_avg_ms"] = round(float(np.mean(dur)), 4)
    out["rocprof_min_ms"] = round(float(np.min(dur)), 4)
    out["rocprof_timed_dispatches"] = len(dur)
    out["kernel_vgpr"] = int(timed[-1].get("VGPR_Count") or 0)
    out["kernel_lds_bytes"] = int(timed[-1].get("LDS_Block_Size") or 0)
    out["kernel_scratch_bytes"] = int(timed[-1].get("Scratch_Size") or 0)
    rows = [row for row in csv.DictReader(open(st[0])) if row["Name"] == out["rocprof_kernel"]]
    if rows:
        out["rocprof_stats_avg_all_calls_ms"] = round(float(rows[0]["AverageNs"]) / 1e6, 4)
    for tag in ("FETCH_SIZE", "WRITE_SIZE"):
        cc = [f for f in files[tag] if f.endswith("counter_collection.csv")]
        vals = [float(r["Counter_Value"]) for r in _leg_rows([r for r in csv.DictReader(open(cc[0]))
                                                              if r["Counter_Name"] == tag], "Kernel_Name", "Dispatch_Id",
                                                             pat, leg, steps)]
        if not vals:
            raise KeyError(f"no {tag} rows for kernel {pat}")
        out[tag + "_KiB"] = sum(vals) / len(vals)
        out[tag + "_dispatches"] = len(vals)
    hbm = int(round((2 * out["FETCH_SIZE_KiB"] + out["WRITE_SIZE_KiB"]) * 1024))
    out["hbm_bytes_per_launch"] = hbm
    out["traffic_over_algorithmic"] = round(hbm / alg_bytes, 5)
    out["correction"] = "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1 KiB (gfx950 FETCH_SIZE counts half of wide reads)"
    out["frac_rocprof_avg"] = round(alg_bytes / (out["rocprof_avg_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
    return hbm, out


def _child_base(args, workload):
    base = [sys.executable, os.path.abspath(__file__), "--workload", workload, "--steps", str(args.steps),
            "--warmup", str(args.warmup), "--no-cpu", "--no-e2e", "--no-pmc", "--no-legs", "--no-inproc", "--no-jni",
            "--erased", args.erased] + \
        (["--stripes", str(args.stripes)] if args.stripes else [])
    for kv in args.tune:
        base += ["--tune", kv]
    return base


def pmc_traffic(args, alg_bytes):
    """HBM bytes per launch of the workload's dominant kernel, measured now: the same bench command as a CHILD
    process under rocprofv3, one --pmc pass per counter (FETCH_SIZE, WRITE_SIZE: they do not fit one pass), plus
    a --kernel-trace --stats pass for the rocprof average duration.  gfx950: FETCH_SIZE reports half of wide
    streaming reads (MI355X_MICROARCH.md, HBM) -> bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024."""
    pat = KERNEL_PAT.get(args.workload)
    if not pat:
        return None, {"error": "no kernel pattern for this workload"}
    # the child runs exactly the main run's warm-up and timed steps, so the rocprof durations of the timed dispatches
    # are taken at the same clock state as the HIP events (a 3-step child ran 11-20 % slow)
    files = {}
    try:
        files = _rocprof_passes(_child_base(args, args.workload), _PMC_PASSES)
        return _leg_stats(files, pat, 0, args.steps, alg_bytes)
    except (OSError, subprocess.SubprocessError, IndexError, KeyError, ValueError) as e:
        return None, {"error": f"{type(e).__name__}: {e}"}
    finally:
        if files.get("_dir"):
            shutil.rmtree(files["_dir"], ignore_errors=True)


def time_workload(wl, steps, warmup, dist):
    """W untimed steps, then K steps bracketed by a barrier + synchronize, each step between HIP events on the launch
    stream: (wall seconds, mean event ms per step)"""
    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
    for _ in range(warmup):
        wl.step()
    barrier()
    st = torch.cuda.current_stream()  # every device-resident workload launches on it (rawcoder._stream_ptr)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(st)
        wl.step()
        b.record(st)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    return elapsed, float(np.mean([a.elapsed_time(b) for a, b in ev]))


def device_legs(args, rank, world, dist, red_dev):
    """The device-resident legs (LEGS): the fused kernels of C5 (rs-6-3 encode + CRC32C) and of reconstruction (rs-10-4
    verify + decode + CRC32C, both erasure sets), the rs-10-4 decode (both sets), CRC32C compute and verify, and C4,
    each timed like the headline and reduced max over ranks: the kernel's roofline fraction from HIP events, and at
    N = 1 the rocprofv3 average and PMC traffic of the same timed dispatches from one child run of all legs (3
    passes)."""
    from ozone_amd.shard import max_over_ranks
    legs = []
    for name, erased in LEGS:
        log(f"leg {name} {erased or ''}")
        wl = Workload(name, rank, world, args.stripes, erased=list(erased or (0, 1, 2, 3)))
        elapsed, kern_ms = time_workload(wl, args.steps, args.warmup, dist)
        elapsed = max_over_ranks(elapsed, dist, device=red_dev)
        kern_ms = max_over_ranks(kern_ms, dist, device=red_dev)
        leg = {"leg": name + (f" {{{','.join(map(str, erased))}}}" if erased else ""),
               "workload": wl.config["workload"], "kernel": wl.kernel, "stripes_per_gpu": wl.S,
               "value": round(wl.data_bytes * world * args.steps / elapsed / 1e9, 2), "unit": "GB/s (data bytes)",
               "ms_per_step": round(elapsed / args.steps * 1e3, 4), "kernel_ms": round(kern_ms, 4),
               "alg_bytes_per_launch": wl.alg_bytes,
               "frac": round(wl.alg_bytes / (kern_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
        if hasattr(wl, "_check"):
            leg["verified"] = wl._check()
        legs.append(leg)
        wl.free()
        del wl
    if rank == 0 and world == 1 and not args.no_pmc:
        files = {}
        try:
            files = _rocprof_passes(_child_base(args, "legs"), _PMC_PASSES, timeout=600)
            for i, (name, _) in enumerate(LEGS):
                traffic, detail = _leg_stats(files, KERNEL_PAT[name], i, args.steps, legs[i]["alg_bytes_per_launch"])
                legs[i]["traffic"] = traffic
                legs[i]["pmc"] = detail
                legs[i]["rocprof_avg_ms"] = detail["rocprof_avg_ms"]
                legs[i]["frac_rocprof_avg"] = detail["frac_rocprof_avg"]
        except (OSError, subprocess.SubprocessError, IndexError, KeyError, ValueError) as e:
            legs.append({"pmc_error": f"{type(e).__name__}: {e}"})
        finally:
            if files.get("_dir"):
                shutil.rmtree(files["_dir"], ignore_errors=True)
    return legs


# ------------------------------------------------------------------------------------------ per-call latency


def stream_latency(args):
    """In-situ per-call cost of the drop-in entry points (one call = what one Java call does), through the C ABI
    from one thread: ozec_encode of one rs-6-3 stripe (RawErasureEncoder.encode, ECKeyOutputStream.java:304) and
    ozec_crc_update (ChecksumByteBuffer.update, Checksum.java:157-200), beside the CPU doing the same call
    (oracle/cpu_baseline.c percall_*: the rs_java table loop; the SSE4.2 crc32 the JDK's CRC32C uses).  The ctypes
    call overhead of the Python harness is measured on a no-op entry point and reported, not subtracted."""
    from ozone_amd import _lib
    from ozone_amd import rawcoder as rc
    n, k, p = MIB, 6, 3
    rng = np.random.default_rng(1)
    L = _lib.lib()

    def per_call(fn, min_s=0.3):
        fn()
        calls, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < min_s:
            fn()
            calls += 1
        return (time.perf_counter() - t0) / calls * 1e6

    exe, flags = _cpu_baseline_bin()

    def cpu(kind, nbytes):
        out = subprocess.run([exe, kind, str(nbytes), "0.3"], capture_output=True, text=True, timeout=60)
        return json.loads(out.stdout)["us_per_call"]

    rows = {"ctypes_call_overhead_us": round(per_call(lambda: L.ozec_version(), 0.1), 2)}
    for cell in (64 << 10, MIB):
        d = [rng.integers(0, 256, cell, dtype=np.uint8) for _ in range(k)]
        o = [np.empty(cell, np.uint8) for _ in range(p)]
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
        rows[f"encode_stripe_{cell >> 10}KiB_cells"] = {"gpu_us": round(per_call(lambda: enc.encode(d, o)), 1),
                                                       "cpu_us": round(cpu("percall_encode", cell), 1)}
        # the same call with every cell in pinned memory (ozec_host_alloc; Java: allocatePinned): DMA in place,
        # no staging copy
        from ozone_amd.stripe_queue import host_alloc
        pool = host_alloc((k + p) * cell)
        dp = [pool.array[i * cell:(i + 1) * cell] for i in range(k + p)]
        for i in range(k):
            dp[i][:] = d[i]
        us = per_call(lambda: enc.encode(dp[:k], dp[k:]))
        rows[f"encode_stripe_{cell >> 10}KiB_cells_pinned"] = {"gpu_us": round(us, 1),
                                                              "GBps": round(k * cell / us / 1e3, 2)}
        del dp
        pool.free()
    buf = rng.integers(0, 256, 16 << 20, dtype=np.uint8)
    st = ctypes.c_uint32(0xFFFFFFFF)
    cross = None
    for nb in (1, 512, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20):
        g = per_call(lambda: L.ozec_crc_update(3, ctypes.byref(st), buf.ctypes.data, nb), 0.2)
        c = cpu("percall_crc32c", nb)
        rows[f"crc_update_{nb}B"] = {"gpu_us": round(g, 2), "cpu_us": round(c, 2)}
        if cross is None and g < c:
            cross = nb
    rows["crc_update_gpu_wins_from_bytes"] = cross
    # Checksum.computeChecksum of one host buffer (Checksum.java:157-179) through ozec_checksum_windows, the batch
    # entry the Java hook would call: CRC32C per 16 KiB window, from 1 and from T threads (each its own buffer),
    # beside the CPU doing the same per-window CRC32C (SSE4.2, what the JDK's CRC32C intrinsic does)
    T = usable_cpus()
    bpc = 16384
    cross = {}
    for nb in (16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
        for th in (1, T):
            bufs = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(th)]
            outs = [np.empty(nb // bpc, np.uint32) for _ in range(th)]

            def one(i):
                rc_ = L.ozec_checksum_windows(3, bufs[i].ctypes.data, nb, bpc, outs[i].ctypes.data, 0)
                assert rc_ == 0

            one(0)
            counts = [0] * th
            t_end = time.perf_counter() + 0.3

            def loop(i):
                while time.perf_counter() < t_end:
                    one(i)
                    counts[i] += 1

            t0 = time.perf_counter()
            if th == 1:
                loop(0)
            else:
                ts = [threading.Thread(target=loop, args=(i,)) for i in range(th)]
                for x in ts:
                    x.start()
                for x in ts:
                    x.join()
            el = time.perf_counter() - t0
            calls = sum(counts)
            out = subprocess.run([exe, "percall_windows", str(nb), "0.3", str(th)], capture_output=True, text=True,
                                 timeout=60)
            c = json.loads(out.stdout)
            g_gbps = calls * nb / el / 1e9
            rows[f"checksum_windows_{nb >> 10}KiB_{th}thr"] = {
                "gpu_us": round(el / (calls / th) * 1e6, 1), "gpu_GBps": round(g_gbps, 2),
                "cpu_us": round(c["us_per_call"], 1), "cpu_GBps": round(c["GBps"], 2)}
            if g_gbps > c["GBps"] and th not in cross:
                cross[th] = nb
    rows["checksum_windows_gpu_wins_from_bytes"] = {f"{th}thr": cross.get(th) for th in (1, T)}
    rows["cpu"] = (f"oracle/cpu_baseline.c percall_* (1 thread; checksum_windows rows: per-window CRC32C on 1 / {T} "
                   f"threads, each its own buffer), {flags}")
    return rows


# ------------------------------------------------------------------------------------------ JNI per-call path

_JNI_BIN = None


def _jni_percall_bin():
    """tests/native/jni_percall.c + jni/ozec_jni.c + jni/ozec_marshal.c against the JNI test double, linked to the
    in-tree libozec.so (built here at run time, as the CPU baseline is)."""
    global _JNI_BIN
    if _JNI_BIN:
        return _JNI_BIN
    lib = os.path.join(ROOT, "ozone_amd", "lib")
    out = os.path.join(tempfile.mkdtemp(prefix="ozec_jni_"), "jni_percall")
    mock = os.path.join(ROOT, "tests", "native", "mockjni")
    subprocess.run(["gcc", "-O2", "-I", mock, "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "jni", "ozec_jni.c"),
                    os.path.join(ROOT, "jni", "ozec_marshal.c"), os.path.join(mock, "mockjni.c"),
                    os.path.join(ROOT, "tests", "native", "jni_percall.c"), "-L", lib, "-lozec", "-lpthread",
                    "-Wl,--wrap=ozec_encode,--wrap=ozec_decode,--wrap=ozec_crc_update,--wrap=ozec_checksum_windows,"
                    "--wrap=ozec_encode_cb,--wrap=ozec_decode_cb,"
                    "--wrap=ozec_host_alloc,--wrap=ozec_host_free", f"-Wl,-rpath,{lib}", "-o", out],
                   check=True, capture_output=True, timeout=120)
    _JNI_BIN = out
    return out


def jni_percall(specs, seconds, dev=0):
    """Run the JNI harness over `specs` ("encode:6:3:65536:4", ...) in one child process pinned to GPU `dev`
    (OZEC_DEVICES), one JSON row per spec."""
    env = dict(os.environ, OZEC_DEVICES=str(dev), OZEC_TUNE=",".join(TUNE))
    r = subprocess.run([_jni_percall_bin(), str(seconds)] + list(specs), capture_output=True, text=True,
                       timeout=120 + 4 * seconds * len(specs), env=env)
    if r.returncode != 0:
        raise RuntimeError(f"jni_percall rc={r.returncode}: {r.stderr.strip()[-400:]}")
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def _cpu_percall_encode(nbytes, seconds=0.3):
    exe, flags = _cpu_baseline_bin()
    out = subprocess.run([exe, "percall_encode", str(nbytes), str(seconds)], capture_output=True, text=True, timeout=60)
    return json.loads(out.stdout)["us_per_call"], flags


def jni_rows(args, threads=(1, 4, 16), cells=(64 << 10, MIB), seconds=0.5):
    """The Java drop-in's per-call production path: OzecNative.encodeArrays / decodeArrays on heap
    byte[] -- what ECKeyOutputStream (one stripe per call, ECKeyOutputStream.java:304, heap buffers :701) and the
    reconstruction coordinator (ECReconstructionCoordinator.java:283) call -- through jni/ozec_jni.c compiled
    against the JNI test double: GetByteArrayRegion into a pooled pinned arena, in-place DMA + kernel,
    SetByteArrayRegion back.  rs-6-3, T threads sharing one coder (RawErasureCoderBenchmark.java:201-206), beside
    the CPU doing one stripe per call on one thread (oracle/cpu_baseline.c percall_encode: the RSUtil table loop)."""
    specs = [f"{mode}:6:3:{c}:{t}" for mode in ("encode", "decode") for c in cells for t in threads]
    # a writer whose buffer pool is pinned (OzecNative.allocatePinned): encodeDirect on pinned direct buffers
    specs += [f"encodedirect:6:3:{c}:{t}" for c in cells for t in threads]
    rows = jni_percall(specs, seconds)
    cpu = {}
    for c in cells:
        cpu[c], flags = _cpu_percall_encode(c)
    for r in rows:
        if r["mode"] == "encode":
            r["cpu_1thread_us_per_stripe"] = round(cpu[r["cell_bytes"]], 1)
    return {"path": "jni/ozec_jni.c encodeArrays / decodeArrays (heap byte[]) and encodeDirect (pinned direct buffers, "
                    "encodedirect rows) via the JNI test double, rs-6-3, decode of 3 erased {0,1,2}", "rows": rows,
            "cpu": f"oracle/cpu_baseline.c percall_encode (1 thread, one stripe per call), {flags}"}


def tail_rows(args, lens=(1007, 1008, 50000, 50001, 700000, 700001), seconds=0.4):
    """The last, partial stripe of every key (parityCellSize = dataBuffers[0].position(), ECKeyOutputStream.java:276):
    cells of any length.  (a) one stripe per call through the JNI path (encodeArrays, 1 and 16
    threads); (b) the fused encode + CRC32C of one stripe per call from pinned host memory
    (ozec_encode_crc_host_batch); (c) device-resident fused encode + CRC32C batches of such cells (unit stride
    padded to 4 KiB, and packed), kernel time per launch -- since round 5 every length runs on the nibble kernel (the
    last 1-15 bytes of a unit in nb_tail; until then a length that was not a multiple of 16 B took the unfused path:
    encode, then one CRC pass per unit, profiles/r05/tail/bench_tail_after.json)."""
    from ozone_amd import checksum as ck
    from ozone_amd import rawcoder as rc
    from ozone_amd.stripe_queue import host_alloc
    k, p, bpc = 6, 3, 16384
    out = {"lens": list(lens)}
    specs = [f"encode:{k}:{p}:{n}:{t}" for n in lens for t in (1, 16)]
    out["jni_encode"] = jni_percall(specs, seconds)
    enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    dev = torch.device("cuda", torch.cuda.current_device())
    host, dev_rows, cpu = [], [], {}
    for n in lens:
        cpu[n], flags = _cpu_percall_encode(n, 0.2)
        nwin = -(-n // bpc)
        pb = host_alloc((k + p) * n + (k + p) * nwin * 4)
        a = pb.array
        a[:k * n] = np.random.default_rng(n).integers(0, 256, k * n, dtype=np.uint8)
        crc_addr = a.ctypes.data + (k + p) * n

        def one():
            enc.encode_crc_host_batch(a.ctypes.data, (k + p) * n, n, a.ctypes.data + k * n, (k + p) * n, n, 1, n,
                                      ck.ChecksumType.CRC32C, bpc, crc_addr)
        one()
        calls, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            one()
            calls += 1
        us = (time.perf_counter() - t0) / calls * 1e6
        host.append({"cell_bytes": n, "us_per_stripe": round(us, 1), "GBps": round(k * n / us / 1e3, 3),
                     "cpu_1thread_encode_only_us": round(cpu[n], 1)})
        pb.free()
        # device-resident batches of such stripes, about 2 GiB of data cells: unit stride padded to 4 KiB, and packed
        # (unit stride = n: units at odd byte offsets when n is odd)
        S = max(64, min(65536, (2 << 30) // (k * n)))
        for layout in ("pitch 4 KiB", "packed"):
            us_ = -(-n // 4096) * 4096 if layout == "pitch 4 KiB" else n
            units = torch.zeros((S, k + p, us_), dtype=torch.uint8, device=dev)
            for u in range(k):
                rc.fill_splitmix64_cells(units[:, u], (k + p) * us_, S, n, SEED, u * S)
            crcs = torch.empty((S, k + p, nwin), dtype=torch.int32, device=dev)

            def launch():
                enc.encode_crc_batch(units, (k + p) * us_, us_, units[:, k:], (k + p) * us_, us_, S, n,
                                     ck.ChecksumType.CRC32C, bpc, crcs)
            for _ in range(3):
                launch()
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record(st)
            for _ in range(reps):
                launch()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            alg = S * (k + p) * n + S * (k + p) * nwin * 4
            dev_rows.append({"cell_bytes": n, "layout": layout, "unit_stride": us_, "stripes": S,
                             "ms_per_launch": round(ms, 4), "GBps_data": round(S * k * n / ms / 1e6, 1),
                             "frac_hbm": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                             "path": "fused (nibble kernel" + (f", last {n % 16} B per unit in nb_tail)" if n % 16
                                                              else ")")})
            if layout == "packed":
                # the same packed stripes through the coding-only and checksum-only entry points (units at odd
                # offsets when n is odd: gf_code_vec through buffer descriptors and crc_windows_g26 with align-1 loads
                # since round 5; gf_code_bytes / crc_windows_bytes before)
                def ms_of(fn):
                    for _ in range(2):
                        fn()
                    e0.record(st)
                    for _ in range(reps):
                        fn()
                    e1.record(st)
                    torch.cuda.synchronize()
                    return e0.elapsed_time(e1) / reps
                ms_code = ms_of(lambda: enc.encode_batch(units, (k + p) * us_, us_, units[:, k:], (k + p) * us_, us_,
                                                         S, n))
                ms_crc = ms_of(lambda: ck.checksum_windows_batch(ck.ChecksumType.CRC32C, units, us_, S * (k + p), n,
                                                                 bpc, crcs))
                dev_rows[-1]["encode_only_ms"] = round(ms_code, 4)
                dev_rows[-1]["encode_only_frac_hbm"] = round(S * (k + p) * n / (ms_code * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                dev_rows[-1]["checksum_only_ms"] = round(ms_crc, 4)
                dev_rows[-1]["checksum_only_frac_hbm"] = round(S * (k + p) * (n + nwin * 4) / (ms_crc * 1e-3) / 1e9 /
                                                               PEAK_HBM_GBS, 4)
            del units, crcs
            torch.cuda.empty_cache()
    out["fused_host_one_stripe_per_call"] = host
    out["fused_device_batch"] = dev_rows
    out["cpu"] = f"oracle/cpu_baseline.c percall_encode (1 thread, encode only), {flags}"
    return out


# ------------------------------------------------------------------------------------------ main


_JSON_FD = None


def _quiet_stdout():
    """Keep stdout for the one JSON line: libraries print to fd 1 from C++ (gloo's "Rank 0 is connected to 1 peer
    ranks"), so fd 1 is pointed at stderr for the whole run and the result goes to a saved copy of it."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def gather_per_rank(rec, dist):
    """{key: [value of rank 0, 1, ...]} of one record per rank (the max-over-ranks figures hide which rank, NUMA node
    or link is the straggler of an N-GPU run)."""
    recs = [rec]
    if dist is not None:
        recs = [None] * dist.get_world_size()
        dist.all_gather_object(recs, rec)
    return {k: [r[k] for r in recs] for k in rec}


def _r(v, nd=4):
    return round(v, nd) if isinstance(v, float) else v


def compact_line(full, full_path):
    """The stdout line of the default run, kept well under the driver's 9 KB tail: every leg as
    one short object (leg, erasure set, kernel, kernel_ms, frac, rocprof_avg_ms, traffic over algorithmic bytes), the
    headline roofline without its PMC detail, the C5 legs, JNI per-call rows as us per stripe, the CPU baseline without
    its host block.  The full record (PMC blocks, per-rank detail, every JNI row) goes to `full_path`."""
    out = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "n_ranks", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    cfg = full.get("config", {})
    out["config"] = {k: cfg[k] for k in ("workload", "cell_bytes", "stripes", "global_stripes", "parallelism") if k in cfg}
    rf = full.get("roofline", {})
    out["roofline"] = {k: _r(rf[k]) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                             "kernel_ms", "alg_bytes_per_launch", "rocprof_avg_ms", "frac_rocprof_avg")
                       if k in rf}
    if isinstance(rf.get("pmc"), dict) and "traffic_over_algorithmic" in rf["pmc"]:
        out["roofline"]["traffic_over_algorithmic"] = rf["pmc"]["traffic_over_algorithmic"]
    if "per_rank" in full:
        out["per_rank"] = {k: full["per_rank"][k] for k in ("elapsed_s", "kernel_ms", "numa_node") if k in full["per_rank"]}
    legs = []
    for lg in full.get("legs", []):
        if "leg" not in lg:
            legs.append({k: str(v)[:200] for k, v in lg.items()})
            continue
        c = {"leg": lg["leg"], "kernel": lg.get("kernel", "").split(" (")[0], "value": lg.get("value"),
             "kernel_ms": lg.get("kernel_ms"), "frac": lg.get("frac"), "rocprof_avg_ms": lg.get("rocprof_avg_ms"),
             "frac_rocprof_avg": lg.get("frac_rocprof_avg")}
        pm = lg.get("pmc")
        if isinstance(pm, dict) and "traffic_over_algorithmic" in pm:
            c["traffic_over_algorithmic"] = pm["traffic_over_algorithmic"]
        for k in ("verified", "error"):
            if k in lg:
                c[k] = lg[k]
        legs.append(c)
    if legs:
        out["legs"] = legs
    for key in ("e2e", "e2e_in_process"):
        e = full.get(key)
        if isinstance(e, dict):
            c = {k: e[k] for k in ("value", "unit", "ms_per_step", "frac_of_duplex_h2d_link", "parity_spot_check",
                                   "error") if k in e}
            if isinstance(e.get("cpu_baseline"), dict):
                c["cpu_baseline_GBps"] = e["cpu_baseline"].get("value")
            out[key] = c
    jp = full.get("jni_percall")
    if isinstance(jp, dict) and "rows" in jp:
        out["jni_percall_us"] = {f"{r['mode']} {r['cell_bytes'] >> 10}K x{r['threads']}": r["us_per_stripe"]
                                 for r in jp["rows"]}
        out["jni_percall_ok"] = all(r.get("round_trip_ok", True) for r in jp["rows"])
    elif jp is not None:
        out["jni_percall"] = str(jp)[:300]
    cb = full.get("cpu_baseline")
    if isinstance(cb, dict):
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "value_1_thread", "sample") if k in cb}
    if "verified" in full:
        out["verified"] = full["verified"]
    out["full_record"] = full_path
    return out


def emit_default(result):
    """rank 0 of the default (c2) run: the full record to a file, the compact line to stdout."""
    path = os.environ.get("OZEC_BENCH_FULL", os.path.join(ROOT, "gpurun_out", "bench_full.json"))
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(result, f, indent=1)
    except OSError as e:
        path = f"(not written: {e})"
    emit(compact_line(result, os.path.relpath(path, ROOT) if os.path.isabs(path) else path))


def emit(obj):
    line = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_workers(args)
    _quiet_stdout()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OZEC_BENCH_SAME_DEVICE=1 + OZEC_DIST_BACKEND=gloo rehearse the N-rank path on a one-GPU box
    dev_idx = 0 if os.environ.get("OZEC_BENCH_SAME_DEVICE") == "1" else local
    torch.cuda.set_device(dev_idx)
    # one process per GPU here: this rank's coders, host batches and staging use its own GPU only (libozec's default
    # would spread one process's coders over every visible GPU, ozec_set_devices)
    from ozone_amd import rawcoder as _rc
    _rc.set_devices([dev_idx])
    global ORIG_AFFINITY
    ORIG_AFFINITY = os.sched_getaffinity(0)
    numa_node = bind_process_to_gpu_node(dev_idx)
    backend = os.environ.get("OZEC_DIST_BACKEND", "nccl")
    dist = None
    cpu_group = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
            # waits that must not occupy a GPU (an RCCL barrier spins a kernel on each waiting rank's GPU, which the
            # in-process leg is using): a gloo group over the same ranks
            cpu_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(backend)
    TUNE[:] = args.tune
    if args.tune:
        from ozone_amd import _lib
        for kv in args.tune:
            key, val = kv.split("=", 1)
            if _lib.lib().ozec_set_tuning(key.encode(), int(val)) != 0:
                raise SystemExit(f"unknown tuning knob {kv}")
    erased = [int(e) for e in args.erased.split(",")]
    if len(erased) != 4 or len(set(erased)) != 4 or not all(0 <= e < 14 for e in erased):
        raise SystemExit("--erased: four distinct unit indexes of rs-10-4 (0..13)")
    from ozone_amd.shard import max_over_ranks
    red_dev = "cuda" if backend == "nccl" else "cpu"
    pci = torch.cuda.get_device_properties(dev_idx)
    dev_id = (f"{getattr(pci, 'pci_domain_id', '')}:{getattr(pci, 'pci_bus_id', '')}:{getattr(pci, 'pci_device_id', '')}"
              f":{getattr(pci, 'uuid', '')}")
    devices = [dev_id]
    if dist is not None:
        devices = [None] * world
        dist.all_gather_object(devices, dev_id)
    n_gpus = len(set(devices))

    if args.workload == "c5":
        res, inproc = e2e_leg(args, rank, world, dist, dev_idx, backend, cpu_group)
        result = {"metric": "C5 e2e: rs-6-3-1024k encode + CRC32C GB/s (data bytes) from pinned host memory",
                  "value": res["value"], "unit": "GB/s", "n_gpus": n_gpus, "n_ranks": world,
                  "steps": args.e2e_steps, "warmup": 1, "ms_per_step": res["ms_per_step"], "higher_is_better": True,
                  "scaling": "strong", "vs_baseline": None, "dtype": "u8",
                  "data": "synthetic (splitmix64 bytes generated on the GPU, copied into the host batch)",
                  "config": {"workload": res["workload"], "stripes": args.e2e_stripes,
                             "parallelism": f"stripe-range sharded x{world} (one shared batch, no collective)"},
                  "e2e": res, "e2e_in_process": inproc}
        if rank == 0 and world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline("c5", args.cpu_seconds)
        if rank == 0:
            emit(result)
        if dist is not None:
            dist.destroy_process_group()
        return 0

    if args.workload == "legs":  # the device-resident legs alone (the rocprofv3 child of the default line)
        legs = device_legs(args, rank, world, dist, red_dev)
        if rank == 0:
            emit({"metric": "device-resident legs", "value": None, "legs": legs})
        if dist is not None:
            dist.destroy_process_group()
        return 0

    if args.workload in ("jni", "tail"):
        if rank == 0:
            rows = jni_rows(args) if args.workload == "jni" else tail_rows(args)
            emit({"metric": f"{args.workload}: per-call rows", "value": None, "n_gpus": n_gpus, "dtype": "u8",
                  "config": {"workload": args.workload}, "rows": rows})
        return 0

    if args.workload == "stream":
        if rank == 0:
            emit({"metric": "per-call latency of the drop-in entry points (us)", "value": None,
                  "n_gpus": n_gpus, "dtype": "u8", "config": {"workload": "stream"},
                  "calls": stream_latency(args)})
        return 0

    global HOST_PINNED
    HOST_PINNED = bool(args.host_pinned)
    log(f"workload {args.workload}: setting up")
    wl = Workload(args.workload, rank, world, args.stripes, args.threads, erased, args.queue_batch)
    log(f"workload {args.workload}: {args.warmup} warm-up + {args.steps} timed steps")
    elapsed, kern_ms = time_workload(wl, args.steps, args.warmup, dist)
    per_rank = gather_per_rank({"elapsed_s": round(elapsed, 5), "kernel_ms": round(kern_ms, 4), "numa_node": numa_node,
                                "device": dev_id, "cpus": len(os.sched_getaffinity(0))}, dist)
    elapsed = max_over_ranks(elapsed, dist, device=red_dev)
    kern_ms = max_over_ranks(kern_ms, dist, device=red_dev)
    value = wl.data_bytes * world * args.steps / elapsed / 1e9
    achieved = wl.alg_bytes / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC if args.workload == "c2" else f"{args.workload}: data GB/s",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": n_gpus,
        "n_ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 bytes generated in HBM)",
        "config": dict(wl.config, global_stripes=wl.S * world,
                       parallelism=f"stripe-range sharded x{world}: rank r encodes stripes [r*{wl.S}, (r+1)*{wl.S}) "
                                   f"of one global batch on its own GPU (no collective)"),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None,
                     "kernel": wl.kernel, "kernel_ms": round(kern_ms, 4), "kernel_ms_reduction": "max over ranks",
                     "alg_bytes_per_launch": wl.alg_bytes, "numa_node": numa_node},
        "per_rank": per_rank,
    }
    if args.workload in ("host", "queue", "queue_pageable", "c3r_host"):
        pc = pcie_ceiling(64 * 10 * MIB, 64 * 4 * MIB) if args.workload == "c3r_host" else \
            pcie_ceiling(64 * 6 * MIB, 64 * 3 * MIB)
        pc["value_frac_of_duplex_h2d"] = round(value / world / pc["duplex_h2d_GBps"], 4)
        result["pcie"] = pc
        result["roofline"]["note"] = "kernel_ms is the whole PCIe-inclusive step; the bound is the link, not HBM"
    if hasattr(wl, "_check"):
        result["verified"] = wl._check()
    wl.free()
    del wl
    if args.workload == "c2" and not args.no_legs:
        try:
            result["legs"] = device_legs(args, rank, world, dist, red_dev)
        except Exception as e:  # the headline stands on its own
            result["legs"] = [{"error": f"{type(e).__name__}: {e}"}]
    if args.workload == "c2" and not args.no_e2e:
        log("C5 end-to-end leg")
        try:
            result["e2e"], result["e2e_in_process"] = e2e_leg(args, rank, world, dist, dev_idx, backend, cpu_group)
        except Exception as e:  # the device-resident line stands on its own
            result["e2e"] = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0 and world == 1:
        if not args.no_pmc and args.workload in KERNEL_PAT:
            log("PMC traffic passes of the headline kernel")
            traffic, detail = pmc_traffic(args, result["roofline"]["alg_bytes_per_launch"])
            result["roofline"]["traffic"] = traffic
            result["roofline"]["pmc"] = detail
            if "rocprof_avg_ms" in detail:
                rf = result["roofline"]
                alg = rf["alg_bytes_per_launch"]
                rf["rocprof_avg_ms"] = detail["rocprof_avg_ms"]
                rf["rocprof_min_ms"] = detail["rocprof_min_ms"]
                rf["frac_rocprof_avg"] = round(alg / (detail["rocprof_avg_ms"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                rf["rocprof_avg_over_events"] = round(detail["rocprof_avg_ms"] / rf["kernel_ms"], 4)
                rf["clocks"] = ("kernel_ms: HIP events around each timed step on the launch stream (mean of the timed "
                                "steps); rocprof_avg_ms: rocprofv3 durations of the same kernel's timed dispatches in a "
                                "child run with the same warm-up and steps; frac uses kernel_ms")
        if args.workload == "c2" and not args.no_jni:
            log("JNI per-call rows")
            try:
                result["jni_percall"] = jni_rows(args)
            except Exception as e:  # the device-resident line stands on its own
                result["jni_percall"] = {"error": f"{type(e).__name__}: {e}"}
        if not args.no_cpu:
            log("CPU baseline")
            result["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds)
            if "e2e" in result and "value" in result["e2e"]:
                result["e2e"]["cpu_baseline"] = cpu_baseline("c5", args.cpu_seconds)
    if rank == 0:
        if args.workload == "c2" and not args.full_line:
            emit_default(result)
        else:
            emit(result)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
