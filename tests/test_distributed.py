"""world_size-2 gloo run of the multi-GPU path's host logic on CPU: each rank takes its stripe range, encodes it
(oracle stands in for the GPU here), the union of the shards equals the single-process encode, and the
max-over-ranks reduction bench.py uses picks the slowest rank."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from ozone_amd.shard import max_over_ranks, stripe_range


def test_stripe_range_partitions():
    for S in (1, 7, 4096, 8192, 8191):
        for G in (1, 2, 3, 4, 8):
            ranges = [stripe_range(S, g, G) for g in range(G)]
            covered = [i for lo, hi in ranges for i in range(lo, hi)]
            assert covered == list(range(S))
            assert max(hi - lo for lo, hi in ranges) - min(hi - lo for lo, hi in ranges) <= (S + G - 1) // G
    with pytest.raises(ValueError):
        stripe_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, S, k, p, n, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle
    from synth import SEED, cells
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = stripe_range(S, rank, world)
    digests = {}
    for s in range(lo, hi):
        par = oracle.rs_encode(k, p, cells(SEED, s * k, k, n))
        digests[s] = int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint64)))
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    slowest = max_over_ranks(1.0 + rank, dist)
    import bench
    per_rank = bench.gather_per_rank({"elapsed_s": 1.0 + rank, "numa_node": rank % 2, "stripes": hi - lo}, dist)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        q.put((gathered, slowest, per_rank))


def test_two_rank_gloo_sharded_encode():
    S, k, p, n, world = 6, 6, 3, 4096, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, k, p, n, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    gathered, slowest, per_rank = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    import oracle
    from synth import SEED, cells
    merged = {}
    for d in gathered:
        assert not set(d) & set(merged)  # disjoint shards
        merged.update(d)
    assert sorted(merged) == list(range(S))
    for s in range(S):
        par = oracle.rs_encode(k, p, cells(SEED, s * k, k, n))
        assert merged[s] == int(np.bitwise_xor.reduce(np.concatenate(par).view(np.uint64)))
    assert slowest == 2.0
    # bench.py's per-rank arrays beside the max: rank order, one entry per rank
    assert per_rank == {"elapsed_s": [1.0, 2.0], "numa_node": [0, 1],
                        "stripes": [hi - lo for lo, hi in (stripe_range(S, r, world) for r in range(world))]}


def test_launch_workers_environment_and_argv():
    """bench.py --gpus N without torchrun: N children with the same argv, torchrun's variables for their rank, a
    rendezvous on 127.0.0.1, only rank 0's stdout kept (the one JSON line)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    argv = ["--gpus", "4", "--steps", "5", "--workload", "c2"]
    specs = bench.worker_specs(4, argv, {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29555)
    assert len(specs) == 4
    for r, (cmd, env, keep) in enumerate(specs):
        assert cmd[0] == sys.executable and cmd[1] == "-u" and cmd[2].endswith("bench.py") and cmd[3:] == argv
        assert (env["RANK"], env["LOCAL_RANK"], env["WORLD_SIZE"], env["LOCAL_WORLD_SIZE"]) == (str(r), str(r), "4", "4")
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/usr/bin"  # the caller's env is kept
        assert keep == (r == 0)


def test_bench_stdout_holds_only_the_json_line():
    """bench.py's contract is ONE JSON line on stdout: anything a library writes to fd 1 from native code (gloo's
    "Rank 0 is connected to 1 peer ranks") goes to stderr instead."""
    import json
    import subprocess
    import sys
    code = ("import os, sys; sys.path.insert(0, %r); import bench; bench._quiet_stdout(); "
            "os.write(1, b'[Gloo] Rank 0 is connected\\n'); print('python noise'); bench.emit({'metric': 'x', 'value': 1})"
            % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "x", "value": 1}, r.stdout
    assert "Gloo" in r.stderr and "python noise" in r.stderr
