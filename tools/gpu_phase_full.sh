#!/bin/bash
# Phase profile (FC_PHASE_PROF build) of the C2 probe, lean instance against the
# full-diagnostics instance (FC_PROBE_DIAG = waits + histograms + cut_times + flips).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/phase_full; mkdir -p "$OUT"
for D in 1 15; do
  rm -f "$OUT/prof_$D.bin"
  FC_PROBE_DIAG=$D FC_LIB_VARIANT=prof FC_PROF_OUT="$OUT/prof_$D.bin" timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-20000} -1 2 > "$OUT/probe_$D.log" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe_$D.log"; exit 1; }
  echo "== diag $D"; cat "$OUT/probe_$D.log"
  python3 tools/prof_report.py "$OUT/prof_$D.bin" 4096 10 > "$OUT/report_$D.txt" && head -12 "$OUT/report_$D.txt"
done
