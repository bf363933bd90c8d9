"""Summarise the SQ counter passes of scripts/gpu_final_r4.sh phase c / scripts/gpu_r5.sh step sq (<dir>/sq_<workload>_p<1|2>/run_counter_collection.csv)
for each workload's dominant kernel: per-dispatch means and the derived LDS / VALU busy fractions.  The counters of one
XCD are reported (x8 for the chip): LDS busy per CU = SQ_LDS_IDX_ACTIVE x 8 / (GRBM_GUI_ACTIVE x 256 CUs), VALU issue per
SIMD = SQ_ACTIVE_INST_VALU x 8 / (GRBM_GUI_ACTIVE x 1024 SIMDs).
usage: python scripts/final_sq_summary.py <dir>   (writes <dir>/sq_summary.json)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PAT = {"c3r": "encode_crc_nb", "c5dev": "encode_crc_nb", "c4": "encode_crc_g26", "c2": "gf_code_vec",
       "c3": "gf_code_vec", "crc": "crc_windows_g26s", "verify": "crc_windows_g26s"}
root = sys.argv[1]
out = {}
for w, pat in PAT.items():
    m = {}
    for p in (1, 2):
        vals = defaultdict(list)
        for f in glob.glob(f"{root}/sq_{w}_p{p}/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if pat in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            m[k if p == 1 or k not in m else k + "_p2"] = sum(v) / len(v)
    if not m:
        continue
    g1, g2 = m.get("GRBM_GUI_ACTIVE"), m.get("GRBM_GUI_ACTIVE_p2", m.get("GRBM_GUI_ACTIVE"))
    d = {}
    if g1 and "SQ_LDS_IDX_ACTIVE" in m:
        d["lds_busy_per_cu(x8xcd)"] = round(m["SQ_LDS_IDX_ACTIVE"] * 8 / (g1 * 256), 4)
    if g2 and "SQ_ACTIVE_INST_VALU" in m:
        d["valu_issue_per_simd(x8xcd)"] = round(m["SQ_ACTIVE_INST_VALU"] * 8 / (g2 * 1024), 4)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_cycles/lds_cycles"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    if m.get("SQ_WAVES"):
        d["valu_per_wave"] = m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVES"]
        d["lds_per_wave"] = m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"]
    if m.get("SQ_WAVE_CYCLES_p2"):
        d["wait_any/wave_cycles"] = round(m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES_p2"], 4)
    if m.get("SQ_WAVE_CYCLES"):
        d["wait_inst_lds/wave_cycles"] = round(m.get("SQ_WAIT_INST_LDS", 0) / m["SQ_WAVE_CYCLES"], 4)
    out[w] = {"kernel_pattern": pat, "counters_per_dispatch": m, "derived": d}
json.dump(out, open(os.path.join(root, "sq_summary.json"), "w"), indent=1)
for w, v in out.items():
    print(w, v["derived"])
