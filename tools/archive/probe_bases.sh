#!/bin/bash
# Per-base C2 throughput (timing only), then SQ counter passes over the mixed-base workload.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/probe; mkdir -p "$OUT"
for b in -1 0 1 2 3 4 5 6 7 8 9; do
  timeout -k 10 120 python3 tools/probe_c2.py 4096 10000 $b 3 >> "$OUT/bases.log" 2>&1 || { echo "probe $b failed"; tail -20 "$OUT/bases.log"; exit 1; }
done
cat "$OUT/bases.log"
if [ -n "$PMC" ]; then BASES=-1 bash tools/pmc_probe.sh || exit 1; python3 tools/pmc_report.py gpurun_out/sq > "$OUT/pmc.txt" 2>&1; cat "$OUT/pmc.txt"; fi
