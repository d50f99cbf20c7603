"""Summarise rocprofv3 outputs of tools/gpu_round.sh into profiles/ (committed evidence).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE from
separate --pmc passes, in KiB; on gfx950 FETCH_SIZE reports half of a wide coalesced
stream, so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (the kernel's HBM reads are the
16-B-per-lane state loads; the node records are L2-resident).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
chains = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
chain_steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
src = os.path.join(ROOT, "gpurun_out")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, f"prof_{tag}", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [r for r in csv.DictReader(open(os.path.join(src, f"pmc_{c}_{tag}", "pmc_counter_collection.csv")))
            if "flip" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"]]
    kname = rows[0]["Kernel_Name"] if rows else None
    vals[c] = [float(r["Counter_Value"]) for r in rows]
fetch = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
hbm = (2 * fetch + write) * 1024
summary = {"round": tag, "kernel": kname, "chains": chains, "chain_steps": chain_steps,
           "FETCH_SIZE_KiB_per_launch": fetch, "WRITE_SIZE_KiB_per_launch": write,
           "launches": {k: len(v) for k, v in vals.items()},
           "hbm_bytes_per_launch": hbm,
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM section)"}
json.dump(summary, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
json.dump(summary, open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
