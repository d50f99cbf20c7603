#!/bin/bash
# Full-diagnostics instance variants on the C2 probe (diag 31 = waits, histograms, cut_times,
# flips, event log; 4096 chains x 100,000 steps, 3 launches) under rocprofv3 --kernel-trace
# --stats: flip kernel and tally_reduce means per library.
#   bash tools/archive/ab_full_trace.sh <tag> abl/x.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp FC_PROBE_DIAG=${DIAG:-31} FC_PROBE_EVCAP=100001
TAG=$1; shift
mkdir -p "$R/gpurun_out/abft_$TAG"
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so); O=$R/gpurun_out/abft_$TAG/${n}_$rep
    export FC_LIB_PATH=$R/$L
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- python3 tools/probe_c2.py 4096 100000 -1 3 > "$O.log" 2>&1 || { echo "$n failed"; tail -20 "$O.log"; exit 1; }
    python3 - "$O" "$n" "$rep" <<'PY'
import csv, sys
o, n, rep = sys.argv[1:]
d = {r["Name"]: float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(o + "/run_kernel_stats.csv"))}
fk = [v for k, v in d.items() if "flip2_kernel" in k]
tr = [v for k, v in d.items() if "tally_reduce" in k]
print(f"{n} rep {rep}: flip {fk[0] if fk else 0:.2f} ms  reduce {tr[0] if tr else 0:.2f} ms")
PY
  done
done
