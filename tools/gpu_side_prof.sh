#!/bin/bash
# Phase cycles of the k > 2 kernel per base (FC_PHASE_PROF build, abl/prof.so or LIB=..., built
# in-tree beforehand): tools/probe_side.py runs, then tools/prof_side_report.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/sideprof_${1:-x}; mkdir -p "$OUT"
for w in ${WL:-c4 c5}; do
  rm -f "$OUT/prof_$w.bin"
  FC_LIB_PATH=${LIB:-$R/abl/prof.so} FC_PROF_OUT="$OUT/prof_$w.bin" timeout -k 10 200 python3 tools/probe_side.py $w 0 ${STEPS:-20000} 2 > "$OUT/probe_$w.log" 2>&1 || { echo "probe $w failed"; tail -20 "$OUT/probe_$w.log"; exit 1; }
  cat "$OUT/probe_$w.log"
  C=$(grep -o "C=[0-9]*" "$OUT/probe_$w.log" | head -1 | cut -d= -f2)
  python3 tools/prof_side_report.py "$OUT/prof_$w.bin" $C 3 | tee "$OUT/report_$w.txt"
done
