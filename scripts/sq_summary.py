"""Summarise rocprofv3 --pmc SQ passes (gpurun_out/sqpmc/<w>_p<i>/run_counter_collection.csv) for the dominant
kernel of each workload: per-dispatch means and the derived issue / LDS / wait ratios."""
import csv
import glob
import json
import sys
from collections import defaultdict

PAT = {"c5dev": "encode_crc_g26<6, 3", "c3r": "encode_crc_g26<10, 4", "c2": "gf_code_vec<6, 3",
       "crc": "crc_windows_g26s", "c4s": "encode_crc_g26<2, 1"}
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sqpmc"
out = {}
for w, pat in PAT.items():
    vals = defaultdict(list)
    for f in glob.glob(f"{root}/{w}_p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not vals:
        continue
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    d = {}
    g = m.get("GRBM_GUI_ACTIVE")
    if g:
        d["kernel_cycles(GRBM_GUI_ACTIVE)"] = g
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m:
        d["valu_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
    if "SQ_INSTS_LDS" in m and "SQ_WAVES" in m:
        d["lds_per_wave"] = m["SQ_INSTS_LDS"] / m["SQ_WAVES"]
    # busy fractions, normalised per SIMD (1024) / per CU (256) over the kernel's cycles
    if g:
        if "SQ_ACTIVE_INST_VALU" in m:
            d["valu_issue_busy_per_simd"] = m["SQ_ACTIVE_INST_VALU"] / (g * 1024)
        if "SQ_LDS_IDX_ACTIVE" in m:
            d["lds_idx_active_per_cu"] = m["SQ_LDS_IDX_ACTIVE"] / (g * 256)
        if "SQ_BUSY_CYCLES" in m:
            d["sq_busy"] = m["SQ_BUSY_CYCLES"] / (g * 32)
    if "SQ_WAVE_CYCLES" in m:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
            if k in m:
                d[k + "/WAVE_CYCLES"] = m[k] / m["SQ_WAVE_CYCLES"]
    out[w] = {"counters": m, "derived": d}
print(json.dumps(out, indent=1))
