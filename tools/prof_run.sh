#!/bin/bash
# Phase-cycle profile (FC_PHASE_PROF build) of the C2 probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/phase${FC_STREAM:+_$FC_STREAM}; mkdir -p "$OUT"
for b in ${PB:--1}; do
  rm -f "$OUT/prof_$b.bin"
  FC_LIB_VARIANT=${VAR:-prof} FC_PROF_OUT="$OUT/prof_$b.bin" timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-10000} $b 2 > "$OUT/probe_$b.log" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe_$b.log"; exit 1; }
  cat "$OUT/probe_$b.log"
  python3 tools/prof_report.py "$OUT/prof_$b.bin" 4096 10
done
