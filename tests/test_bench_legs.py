"""bench.py's selection of each leg's timed dispatches in the rocprofv3 child run (every leg of the
default line gets its rocprof average and PMC traffic).  The child runs the legs in order; a leg's warm-up and timed
steps are one unbroken run of its kernel, its set-up launches other kernels first.  Synthetic trace rows, CPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

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
        if name == "c5dev":
            seq += [fill] * 6 + [nb63] * (W + K)
        elif name == "c3r":
            seq += [fill] * 10 + [gf104, crc] + [nb104] * (W + K)
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
    for i, (name, _) in enumerate(bench.LEGS):
        pat = bench.KERNEL_PAT[name]
        occ = sum(1 for nm, _ in bench.LEGS[:i] if bench.KERNEL_PAT[nm] == pat)
        got = bench._leg_rows(rows, "Kernel_Name", "Start_Timestamp", pat, occ, W, K)
        assert len(got) == K
        assert len({r["Kernel_Name"] for r in got}) == 1 and bench._kernel_match(pat, got[0]["Kernel_Name"])
        ts = [int(r["Start_Timestamp"]) for r in got]
        assert ts == sorted(ts) and ts[-1] - ts[0] == 1000 * (K - 1)  # consecutive dispatches
        assert not seen & set(ts)  # no two legs share a dispatch
        seen |= set(ts)
    # the verify leg is the second run of crc_windows_g26s: the verify kernel, not the compute one
    i = [n for n, _ in bench.LEGS].index("verify")
    got = bench._leg_rows(rows, "Kernel_Name", "Start_Timestamp", bench.KERNEL_PAT["verify"], 1, W, K)
    assert got[0]["Kernel_Name"].endswith("true>") and i > [n for n, _ in bench.LEGS].index("crc")


def test_pmc_rows_order_by_dispatch_id():
    """counter rows carry Dispatch_Id, not timestamps; the same runs come out"""
    W, K = 2, 3
    seq = ["fill"] + ["a<1>"] * (W + K) + ["fill"] + ["a<1>"] * (W + K + 1)
    rows = [{"Kernel_Name": k, "Dispatch_Id": str(i + 1), "Counter_Value": str(i)} for i, k in enumerate(seq)]
    rows = rows[::-1]  # file order does not matter
    first = bench._leg_rows(rows, "Kernel_Name", "Dispatch_Id", "a<", 0, W, K)
    second = bench._leg_rows(rows, "Kernel_Name", "Dispatch_Id", "a<", 1, W, K)
    assert [int(r["Dispatch_Id"]) for r in first] == [4, 5, 6]
    assert [int(r["Dispatch_Id"]) for r in second] == [11, 12, 13]
