#!/bin/bash
# r05g: rocprofv3 kernel stats of the full-diagnostics C2 probe (flip kernel + tally reduce)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r05g; mkdir -p "$OUT"
for L in ${LIBS:-abl/tlog.so}; do
  n=$(basename $L .so)
  FC_PROBE_DIAG=${DIAG:-15} FC_LIB_PATH=$R/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$n" -o run --output-format csv -- python3 tools/probe_c2.py 4096 100000 -1 3 > "$OUT/tr_$n.log" 2>&1 || { echo "trace $n failed"; tail -20 "$OUT/tr_$n.log"; exit 1; }
  echo "== $n"; tail -1 "$OUT/tr_$n.log"; cat "$OUT"/tr_$n/*kernel_stats.csv | cut -c1-200
done
echo R05G_OK
