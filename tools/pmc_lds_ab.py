"""Per-library LDS / issue counters of tools/pmc_lds_ab.sh: the flip-kernel dispatches after the
first (warm-up) one, averaged; each variant's difference to the first library (the base).  A
variant that issues one LDS access kind twice (tools/patches/lds_dup_attribution.patch, -DFC_EXP_DUP=k) adds that kind's own
instructions, array cycles and bank-conflict cycles once more, so its difference attributes them."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out_dir, libs = sys.argv[1], sys.argv[2:]
res = {}
for L in libs:
    n = os.path.basename(L)[:-3]
    f = glob.glob(os.path.join(out_dir, n, "**", "*counter_collection.csv"), recursive=True)
    by = defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        if "flip2_kernel" not in r["Kernel_Name"]:
            continue
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)[1:] or sorted(by)
    res[n] = {k: sum(by[i][k] for i in ids) / len(ids) for k in by[ids[0]]}
base = libs[0] and os.path.basename(libs[0])[:-3]
b = res[base]
table = {}
for n, c in res.items():
    row = {"lds_insts_per_wave": c["SQ_INSTS_LDS"] / c["SQ_WAVES"],
           "lds_active": c["SQ_LDS_IDX_ACTIVE"], "bank_conflict": c["SQ_LDS_BANK_CONFLICT"],
           "conflict_frac_of_active": c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)}
    if n != base:
        dl = c["SQ_INSTS_LDS"] - b["SQ_INSTS_LDS"]
        row["delta_lds_insts_per_wave"] = dl / c["SQ_WAVES"]
        row["delta_bank_conflict"] = c["SQ_LDS_BANK_CONFLICT"] - b["SQ_LDS_BANK_CONFLICT"]
        row["delta_conflict_share_of_base"] = row["delta_bank_conflict"] / max(b["SQ_LDS_BANK_CONFLICT"], 1)
        row["delta_active_share_of_base"] = (c["SQ_LDS_IDX_ACTIVE"] - b["SQ_LDS_IDX_ACTIVE"]) / max(b["SQ_LDS_IDX_ACTIVE"], 1)
        row["conflict_cycles_per_added_inst"] = row["delta_bank_conflict"] / max(dl, 1)
    table[n] = row
print(json.dumps(table, indent=1))
json.dump({"counters": res, "table": table}, open(os.path.join(out_dir, "summary.json"), "w"), indent=1)
