"""Summarise gpurun_out/nbsq/<wl>_v<variant>_p<pass>/ counter CSVs: per-dispatch means of the fused kernel and the
derived LDS / VALU utilisation (per CU / per SIMD over GRBM_GUI_ACTIVE cycles)."""
import csv, glob, json, os, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/nbsq"
res = {}
for d in sorted(glob.glob(f"{root}/*_v*_p1")):
    tag = os.path.basename(d)[:-3]
    vals = defaultdict(list)
    for p in (1, 2):
        for f in glob.glob(f"{root}/{tag}_p{p}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "encode_crc" in r["Kernel_Name"]:
                    vals[(p, r["Counter_Name"])].append(float(r["Counter_Value"]))
    m = {f"{c}@{p}": sum(v) / len(v) for (p, c), v in vals.items()}
    if not m:
        continue
    g1, g2 = m.get("GRBM_GUI_ACTIVE@1"), m.get("GRBM_GUI_ACTIVE@2")
    w = m.get("SQ_WAVES@1", 1)
    dd = {"gui_cycles": g1,
          "valu_per_wave": m.get("SQ_INSTS_VALU@1", 0) / w, "lds_per_wave": m.get("SQ_INSTS_LDS@1", 0) / w,
          "lds_idx_active_per_cu": m.get("SQ_LDS_IDX_ACTIVE@1", 0) / (g1 * 256) if g1 else None,
          "lds_bank_conflict_per_cu": m.get("SQ_LDS_BANK_CONFLICT@1", 0) / (g1 * 256) if g1 else None,
          "wait_inst_lds/wave_cycles": m.get("SQ_WAIT_INST_LDS@1", 0) / m.get("SQ_WAVE_CYCLES@1", 1),
          "active_inst_lds/wave_cycles": m.get("SQ_ACTIVE_INST_LDS@1", 0) / m.get("SQ_WAVE_CYCLES@1", 1),
          "valu_busy_per_simd": m.get("SQ_ACTIVE_INST_VALU@2", 0) / (g2 * 1024) if g2 else None,
          "wait_inst_any/wave_cycles": m.get("SQ_WAIT_INST_ANY@2", 0) / m.get("SQ_WAVE_CYCLES@2", 1),
          "wait_any/wave_cycles": m.get("SQ_WAIT_ANY@2", 0) / m.get("SQ_WAVE_CYCLES@2", 1),
          "waves_per_simd": m.get("SQ_WAVE_CYCLES@2", 0) / (g2 * 1024) if g2 else None}
    res[tag] = {"derived": dd, "counters": m}
print(json.dumps(res, indent=1))
