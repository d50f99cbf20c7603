"""Summarise tools/gpu_profile.sh outputs (gpurun_out/prof_<tag>/) into profiles/<tag>_*:

  <tag>_bench.json          the bench line of the run
  <tag>_kernel_stats.csv    rocprofv3 --kernel-trace --stats of `bench.py --steps 5 --warmup 1`
  <tag>_kernel_stats_full.csv  ... of the full-diagnostics leg (`--full-diag-steps 3`)
  <tag>_pmc_traffic.json    HBM bytes per launch of the flip kernel (also profiles/pmc_traffic.json,
                            which bench.py reads into roofline.traffic)
  <tag>_lds_issue.json      LDS / issue counters per dispatch
  <tag>_roofline_check.json the bench line's roofline recomputed from the rocprofv3 durations
  <tag>_side_c{3,4,5}.json  the k > 2 side-config bench lines

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come from separate --pmc
passes, in KiB; on gfx950 FETCH_SIZE reports half of a wide coalesced stream (the kernel's HBM
reads are the 16-B-per-lane state loads), so hbm = (2 FETCH_SIZE + WRITE_SIZE) x 1024.
Usage: python tools/profile_summary.py TAG"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)


def flip_rows(path):
    return [r for r in csv.DictReader(open(path)) if "flip2_kernel" in r["Kernel_Name"] or
            "flip_kernel" in r["Kernel_Name"]]


bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
json.dump(bench, open(os.path.join(dst, f"{tag}_bench.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
if os.path.exists(os.path.join(src, "trace_full", "run_kernel_stats.csv")):  # full-diagnostics leg
    shutil.copy(os.path.join(src, "trace_full", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats_full.csv"))

# per-launch durations of the headline kernel in the traced bench (steps 5, warmup 1)
# (exactly the bench line's instance: other flip kernels of the run -- e.g. a reference-sweep side
# line's full-diagnostics instance -- are not the headline's launches)
KNAME = bench["roofline"]["kernel"]
trace = [r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv")))
         if KNAME + "(" in r["Kernel_Name"]]
durs = [(float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-6 for r in trace]
timed = durs[1:]  # drop the warmup launch
rl = bench["roofline"]
# the bound level's algorithmic bytes (roofline.levels, round 4) -- the bytes achieved is priced on
lvl = rl.get("levels", {}).get(rl["bound"]) if isinstance(rl.get("levels"), dict) else None
alg = lvl["bytes"] if lvl else rl["alg_bytes_per_launch"]
check = {"round": tag, "kernel": trace[0]["Kernel_Name"] if trace else None,
         "rocprof_launch_ms": durs, "rocprof_timed_mean_ms": statistics.mean(timed),
         "rocprof_timed_median_ms": statistics.median(timed),
         "bench_hip_event_kernel_ms": rl["kernel_ms"], "alg_bytes_per_launch": alg,
         "achieved_gbs_from_rocprof": alg / (statistics.mean(timed) * 1e-3) / 1e9,
         "achieved_gbs_bench": rl["achieved"], "peak_gbs": rl["peak"], "bound": rl["bound"]}
check["rel_diff"] = check["achieved_gbs_from_rocprof"] / check["achieved_gbs_bench"] - 1.0
check["frac_from_rocprof"] = check["achieved_gbs_from_rocprof"] / rl["peak"]

vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [r for r in flip_rows(os.path.join(src, f"pmc_{c}", "pmc_counter_collection.csv"))
            if KNAME + "(" in r["Kernel_Name"]]
    vals[c] = [float(r["Counter_Value"]) for r in rows][1:]  # timed launches
fetch = statistics.mean(vals["FETCH_SIZE"])
write = statistics.mean(vals["WRITE_SIZE"])
traffic = {"round": tag, "kernel": check["kernel"], "chains": bench["config"]["chains_per_gpu"],
           "chain_steps": bench["config"]["chain_steps_per_launch"], "workload": bench["config"]["graph"],
           "FETCH_SIZE_KiB_per_launch": fetch, "WRITE_SIZE_KiB_per_launch": write,
           "launches": {k: len(v) for k, v in vals.items()},
           "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
           "build_id": bench.get("build_id"),  # the library the counters measured (bench.measured_traffic)
           "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM section)"}
json.dump(traffic, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
json.dump(traffic, open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w"), indent=1)
check["hbm_bytes_per_launch"] = traffic["hbm_bytes_per_launch"]
check["hbm_gbs_measured"] = traffic["hbm_bytes_per_launch"] / (statistics.mean(timed) * 1e-3) / 1e9

def lds_issue(path, kname):
    """Per-dispatch LDS / issue counters of the kernels named like `kname` (warmup dropped)."""
    by = defaultdict(dict)
    names = {}
    for r in flip_rows(path):
        if kname not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        by[d][r["Counter_Name"]] = float(r["Counter_Value"])
        by[d]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    ids = sorted(by)[1:] or sorted(by)
    avg = {k: statistics.mean(by[i][k] for i in ids) for k in by[ids[0]]}
    t = avg["_ns"] * 1e-9
    clk = avg["GRBM_GUI_ACTIVE"] / 8 / t
    cyc = clk * t
    return {"round": tag, "kernel": names[ids[0]], "dispatches": len(ids), "kernel_ms": t * 1e3,
           "counters_per_dispatch": {k: v for k, v in avg.items() if not k.startswith("_")},
           "effective_clock_ghz": clk / 1e9,
           "lds_array_busy_frac": avg["SQ_LDS_IDX_ACTIVE"] / (256 * cyc),
           "lds_bytes_upper_bound_gbs": avg["SQ_LDS_IDX_ACTIVE"] * 256 / t / 1e9,
           "lds_bank_conflict_frac_of_active": avg["SQ_LDS_BANK_CONFLICT"] / max(avg["SQ_LDS_IDX_ACTIVE"], 1),
           "valu_insts_per_simd_cycle": avg["SQ_INSTS_VALU"] / (1024 * cyc),
           "salu_insts_per_cu_cycle": avg["SQ_INSTS_SALU"] / (256 * cyc),
           "lds_insts_per_wave": avg["SQ_INSTS_LDS"] / max(avg["SQ_WAVES"], 1),
           "valu_insts_per_wave": avg["SQ_INSTS_VALU"] / max(avg["SQ_WAVES"], 1),
           "note": "SQ_LDS_IDX_ACTIVE counts LDS-array cycles (incl. bank-conflict cycles) summed over CUs; "
                   "x 256 B/clk/CU bounds the LDS bytes moved from above"}


lds = lds_issue(os.path.join(src, "pmc_lds", "pmc_counter_collection.csv"), KNAME + "(")
json.dump(lds, open(os.path.join(dst, f"{tag}_lds_issue.json"), "w"), indent=1)
check["lds_array_busy_frac"] = lds["lds_array_busy_frac"]
json.dump(check, open(os.path.join(dst, f"{tag}_roofline_check.json"), "w"), indent=1)
for w in ("c3", "c4", "c5"):
    p = os.path.join(src, f"side_{w}.json")
    if os.path.exists(p):
        line = json.loads(open(p).read().strip().splitlines()[-1])
        json.dump(line, open(os.path.join(dst, f"{tag}_side_{w}.json"), "w"), indent=1)
for w in ("c3", "c4", "c5"):  # counters of the k > 2 instances
    d = os.path.join(src, f"side_pmc_{w}_lds", "pmc_counter_collection.csv")
    if not os.path.exists(d):
        continue
    side = lds_issue(d, "fc::flip_kernel")
    # the run they come from (tools/gpu_profile.sh: 20,000-step launches of the side line's
    # resident chains), which bench.py matches before it reports them as the line's traffic
    side["chain_steps"] = 20000
    p = os.path.join(src, f"side_{w}.json")
    if os.path.exists(p):
        line = json.loads(open(p).read().strip().splitlines()[-1])
        side["chains"] = line["config"]["chains_per_gpu"]
        side["build_id"] = line.get("build_id")
    hb = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in flip_rows(os.path.join(src, f"side_pmc_{w}_{c}", "pmc_counter_collection.csv"))
                if "fc::flip_kernel" in r["Kernel_Name"]]
        hb[c] = statistics.mean([float(r["Counter_Value"]) for r in rows][1:] or [float(r["Counter_Value"]) for r in rows])
    side["FETCH_SIZE_KiB_per_launch"] = hb["FETCH_SIZE"]
    side["WRITE_SIZE_KiB_per_launch"] = hb["WRITE_SIZE"]
    side["hbm_bytes_per_launch"] = (2 * hb["FETCH_SIZE"] + hb["WRITE_SIZE"]) * 1024
    side["hbm_gbs_measured"] = side["hbm_bytes_per_launch"] / (side["kernel_ms"] * 1e-3) / 1e9
    side["workload"] = w
    json.dump(side, open(os.path.join(dst, f"{tag}_side_pmc_{w}.json"), "w"), indent=1)
print(json.dumps(check, indent=1))
