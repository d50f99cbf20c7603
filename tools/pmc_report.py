"""Summarise gpurun_out/sq/* PMC passes: per-kernel-dispatch averages of each counter."""
import csv, glob, os, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
for d in sorted(glob.glob(os.path.join(root, "b*_g*"))):
    f = os.path.join(d, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "flip" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: f"{sum(v[1:]) / max(1, len(v) - 1):.4g}" for k, v in sorted(acc.items())})
