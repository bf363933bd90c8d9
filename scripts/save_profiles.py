"""Copy a scripts/gpu_full.sh session from gpurun_out/full/ into profiles/<tag>/ and refresh
profiles/traffic_<workload>.json (HBM bytes per launch of each workload's dominant kernel, from PMC)."""
import csv, json, os, shutil, sys

tag = sys.argv[1]
G, P = os.path.join("gpurun_out", "full"), os.path.join("profiles", tag)
os.makedirs(P, exist_ok=True)
KERNEL = {"c2": "gf_code_vec", "c3": "gf_code_vec", "c3r": "encode_crc_g26", "c4": "encode_crc_g26",
          "c5": "encode_crc_g26", "crc": "crc_windows_g26", "verify": "crc_windows_g26"}
for w in ("c2", "c3", "c3r", "c4", "c5", "crc", "verify", "e2e", "host"):
    if os.path.exists(f"{G}/bench_{w}.json"):
        shutil.copy(f"{G}/bench_{w}.json", f"{P}/bench_{w}.json")
shutil.copy(f"{G}/pytest_gpu.log", f"{P}/pytest_gpu.log")


def rows(path):
    return list(csv.DictReader(open(path)))


for w, pat in KERNEL.items():
    stats = f"{G}/prof_{w}/run_kernel_stats.csv"
    if not os.path.exists(stats):
        continue
    shutil.copy(stats, f"{P}/{w}_kernel_stats.csv")
    ctr = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        src = f"{G}/pmc_{w}_{c}/run_counter_collection.csv"
        shutil.copy(src, f"{P}/{w}_pmc_{c}.csv")
        v = [float(r["Counter_Value"]) for r in rows(src) if pat in r["Kernel_Name"] and r["Counter_Name"] == c]
        ctr[c] = sum(v) / len(v)
    k = [r for r in rows(stats) if pat in r["Name"]][0]
    bench = json.loads(open(f"{P}/bench_{w}.json").read().strip().splitlines()[-1])
    out = {"workload": w, "kernel": k["Name"], "rocprof_average_ns": float(k["AverageNs"]),
           "bench_kernel_ms": bench["roofline"]["kernel_ms"], "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"],
           "FETCH_SIZE_KiB": ctr["FETCH_SIZE"], "WRITE_SIZE_KiB": ctr["WRITE_SIZE"],
           "correction": "gfx950 FETCH_SIZE reports 1/2 of wide coalesced streaming reads (MI355X_MICROARCH.md HBM): "
                         "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
           "hbm_bytes_per_launch": int(round((2 * ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024)),
           "source": f"profiles/{tag}/{w}_pmc_{{FETCH,WRITE}}_SIZE.csv (rocprofv3 --pmc, separate passes)"}
    json.dump(out, open(f"profiles/traffic_{w}.json", "w"), indent=1)
    print(json.dumps({x: out[x] for x in ("workload", "rocprof_average_ns", "bench_kernel_ms", "alg_bytes_per_launch", "hbm_bytes_per_launch")}))
