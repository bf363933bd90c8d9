"""Copy the last gpu_check.sh outputs from gpurun_out/ into profiles/<tag>/ and refresh profiles/traffic_c2.json."""
import csv, json, os, shutil, sys
tag = sys.argv[1]
G, P = "gpurun_out", os.path.join("profiles", tag)
os.makedirs(P, exist_ok=True)
for w in ("c2", "c3", "c3r", "c4", "c5", "crc", "e2e"):
    if os.path.exists(f"{G}/bench_{w}.json"):
        shutil.copy(f"{G}/bench_{w}.json", f"{P}/bench_{w}.json")
shutil.copy(f"{G}/prof_c2/run_kernel_stats.csv", f"{P}/c2_kernel_stats.csv")
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    shutil.copy(f"{G}/pmc_c2_{c}/run_counter_collection.csv", f"{P}/c2_pmc_{c}.csv")
shutil.copy(f"{G}/pytest_gpu.log", f"{P}/pytest_gpu.log")
def mean(path, ctr):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if "gf_code_vec" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
    return sum(v) / len(v)
f, w = mean(f"{P}/c2_pmc_FETCH_SIZE.csv", "FETCH_SIZE"), mean(f"{P}/c2_pmc_WRITE_SIZE.csv", "WRITE_SIZE")
kname = [r["Name"] for r in csv.DictReader(open(f"{P}/c2_kernel_stats.csv")) if "gf_code_vec" in r["Name"]][0]
avg = [float(r["AverageNs"]) for r in csv.DictReader(open(f"{P}/c2_kernel_stats.csv")) if "gf_code_vec" in r["Name"]][0]
out = {"workload": "c2", "kernel": kname, "rocprof_average_ns": avg, "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
       "correction": "gfx950 FETCH_SIZE reports 1/2 of wide coalesced streaming reads (MI355X_MICROARCH.md HBM): bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
       "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
       "source": f"profiles/{tag}/c2_pmc_{{FETCH,WRITE}}_SIZE.csv (rocprofv3 --pmc, separate passes, bench.py --steps 3)"}
json.dump(out, open("profiles/traffic_c2.json", "w"), indent=1)
print(json.dumps(out))
