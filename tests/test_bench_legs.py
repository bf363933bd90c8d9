"""bench.py's selection of each leg's timed dispatches in the rocprofv3 child run (every leg of the
default line gets its rocprof average and PMC traffic).  The child runs the legs in order; each leg's set-up starts
with the synthetic-data fill kernel, and its steps may launch other kernels between the measured ones (the
reconstruction's mismatch finisher, the runtime's memset of a new WorkQueue slot).  Synthetic trace rows, CPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pytest  # noqa: E402

import bench  # noqa: E402


def _trace(seq):
    """seq: kernel names in launch order -> kernel-trace rows with increasing timestamps"""
    return [{"Kernel_Name": k, "Start_Timestamp": str(1000 * i), "End_Timestamp": str(1000 * i + 500 + i)}
            for i, k in enumerate(seq)]


def _legs_sequence(W, K):
    """the dispatch sequence of the default line's child: LEGS in order, with their set-up launches"""
    seq = []
    nb104, nb63, gf104, crc, ver, x21, fill = ("encode_crc_nb<10, 4, 2>", "encode_crc_nb<6, 3, 2>",
                                               "gf_code_vec<10, 4, true>", "crc_windows_g26s<4, 2, false>",
                                               "crc_windows_g26s<4, 2, true>", "encode_crc_g26<2, 1, 2>",
                                               "fill_splitmix64")
    for name, _ in bench.LEGS:
        if name == "c5dev":  # the persistent kernel's first launches each zero a new WorkQueue slot (a memset kernel)
            ms = "__amd_rocclr_fillBufferAligned"
            seq += [fill] * 6 + [nb63, ms, nb63, ms, nb63] + [nb63, ms] * 5 + [nb63] * (W + K - 8)
        elif name == "c3r":
            seq += [fill] * 10 + [gf104, crc] + [nb104, "finish_mismatch"] * (W + K)
        elif name == "c3":
            seq += [fill] * 10 + [gf104] + [gf104] * (W + K)  # the set-up encode runs into the decode steps
        elif name == "crc":
            seq += [fill] + [crc] * (W + K)
        elif name == "verify":
            seq += [fill] + [crc] + [ver] * (W + K)
        elif name == "c4":
            seq += [fill] * 2 + [x21] * (W + K)
    return seq


def test_each_leg_gets_its_own_timed_dispatches():
    W, K = 5, 20
    rows = _trace(_legs_sequence(W, K))
    seen = set()
    last_end = -1
    for i, (name, _) in enumerate(bench.LEGS):
        pat = bench.KERNEL_PAT[name]
        got = bench._leg_rows(rows, "Kernel_Name", "Start_Timestamp", pat, i, K)
        assert len(got) == K
        assert len({r["Kernel_Name"] for r in got}) == 1 and bench._kernel_match(pat, got[0]["Kernel_Name"])
        ts = [int(r["Start_Timestamp"]) for r in got]
        assert ts == sorted(ts) and ts[0] > last_end  # legs in order, none sharing a dispatch
        assert not seen & set(ts)
        seen |= set(ts)
        last_end = ts[-1]
    # the verify leg's timed dispatches are the verify kernel's, not the set-up CRC launch before them
    i = [n for n, _ in bench.LEGS].index("verify")
    got = bench._leg_rows(rows, "Kernel_Name", "Start_Timestamp", bench.KERNEL_PAT["verify"], i, K)
    assert all(r["Kernel_Name"].endswith("true>") for r in got)
    # c3: the set-up encode of the same kernel precedes the decode steps and is not among them
    i = [n for n, _ in bench.LEGS].index("c3")
    seg = bench._leg_segments(rows, "Kernel_Name", "Start_Timestamp")[i]
    first_gf = min(int(r["Start_Timestamp"]) for r in seg if r["Kernel_Name"].startswith("gf_code_vec"))
    got = bench._leg_rows(rows, "Kernel_Name", "Start_Timestamp", bench.KERNEL_PAT["c3"], i, K)
    assert int(got[0]["Start_Timestamp"]) > first_gf


def test_pmc_rows_order_by_dispatch_id():
    """counter rows carry Dispatch_Id, not timestamps, and come in any order; too few dispatches is an error"""
    W, K = 2, 3
    seq = ["fill_splitmix64"] + ["a<1>"] * (W + K) + ["fill_splitmix64"] * 2 + ["a<1>", "b"] * (W + K + 1)
    rows = [{"Kernel_Name": k, "Dispatch_Id": str(i + 1), "Counter_Value": str(i)} for i, k in enumerate(seq)]
    rows = rows[::-1]
    first = bench._leg_rows(rows, "Kernel_Name", "Dispatch_Id", "a<", 0, K)
    second = bench._leg_rows(rows, "Kernel_Name", "Dispatch_Id", "a<", 1, K)
    assert [int(r["Dispatch_Id"]) for r in first] == [4, 5, 6]
    assert [int(r["Dispatch_Id"]) for r in second] == [15, 17, 19]
    with pytest.raises(IndexError):
        bench._leg_rows(rows, "Kernel_Name", "Dispatch_Id", "a<", 0, W + K + 1)


def test_compact_line_keeps_every_leg_under_the_drivers_tail():
    """the default run prints one line under the driver's 9 KB stdout tail that still carries the
    contract keys, the headline roofline, every leg (kernel time, fraction, rocprof average, traffic), both C5 legs, the
    JNI per-call rows and the CPU baseline -- checked on a full record of this round's default run."""
    full_path = os.path.join(ROOT, "profiles", "r06", "final_a", "bench_full.json")
    full = json.load(open(full_path))
    line = json.dumps(bench.compact_line(full, "gpurun_out/bench_full.json"))
    assert len(line) < 9000
    out = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert out["value"] == full["value"] and out["roofline"]["frac"] == full["roofline"]["frac"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in out["roofline"], k
    assert [lg["leg"] for lg in out["legs"]] == [lg["leg"] for lg in full["legs"]]
    for lg in out["legs"]:
        assert {"kernel_ms", "frac", "rocprof_avg_ms", "traffic_over_algorithmic"} <= set(lg), lg
    assert out["e2e"]["value"] == full["e2e"]["value"] and "e2e_in_process" in out
    assert len(out["jni_percall_us"]) == len(full["jni_percall"]["rows"])
    assert {"value", "unit", "cores", "kind", "sample"} <= set(out["cpu_baseline"])
