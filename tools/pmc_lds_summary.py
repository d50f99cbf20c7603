"""Summarise the LDS / issue PMC pass of tools/pmc_lds.sh into profiles/<tag>_lds_issue.json.

Per flip-kernel dispatch (the warmup dispatch dropped): raw counter sums as rocprofv3 reports
them (summed over the chip), plus derived rates with the kernel time of the same dispatch:
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / time (MI355X_MICROARCH.md, DVFS note); LDS array
busy fraction = SQ_LDS_IDX_ACTIVE / (256 CUs x cycles) and the LDS bytes that many array cycles
can move at 256 B per CU-cycle (an upper bound on the achieved LDS bandwidth); VALU / SALU
instructions per SIMD-cycle (1024 SIMDs)."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
f = os.path.join(ROOT, "gpurun_out", f"pmc_lds_{tag}", "pmc_counter_collection.csv")
rows = [r for r in csv.DictReader(open(f)) if "flip" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"]]
by = defaultdict(dict)
for r in rows:
    by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    by[int(r["Dispatch_Id"])]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    by[int(r["Dispatch_Id"])]["_name"] = r["Kernel_Name"]
ids = sorted(by)[1:] or sorted(by)
avg = {k: sum(by[i][k] for i in ids) / len(ids) for k in by[ids[0]] if not k.startswith("_name")}
t = avg["_ns"] * 1e-9
clk = avg["GRBM_GUI_ACTIVE"] / 8 / t
cycles = clk * t
out = {"round": tag, "kernel": by[ids[0]]["_name"], "dispatches": len(ids), "kernel_ms": t * 1e3,
       "counters_per_dispatch": {k: v for k, v in avg.items() if not k.startswith("_")},
       "effective_clock_ghz": clk / 1e9,
       "lds_array_busy_frac": avg["SQ_LDS_IDX_ACTIVE"] / (256 * cycles),
       "lds_bytes_upper_bound_gbs": avg["SQ_LDS_IDX_ACTIVE"] * 256 / t / 1e9,
       "lds_bank_conflict_frac_of_active": avg["SQ_LDS_BANK_CONFLICT"] / max(avg["SQ_LDS_IDX_ACTIVE"], 1),
       "valu_insts_per_simd_cycle": avg["SQ_INSTS_VALU"] / (1024 * cycles),
       "salu_insts_per_cu_cycle": avg["SQ_INSTS_SALU"] / (256 * cycles),
       "lds_insts_per_wave": avg["SQ_INSTS_LDS"] / max(avg["SQ_WAVES"], 1),
       "valu_insts_per_wave": avg["SQ_INSTS_VALU"] / max(avg["SQ_WAVES"], 1)}
dst = os.path.join(ROOT, "profiles", f"{tag}_lds_issue.json")
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
