#!/bin/bash
# Chain dealing on / off under the FC_PHASE_PROF build: per-SIMD composition and chain times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/deal; mkdir -p "$OUT"
for T in "deal=-1" ""; do
  tag=${T:-deal_on}
  rm -f "$OUT/prof_$tag.bin"
  FC_TUNE=$T FC_LIB_VARIANT=prof FC_PROF_OUT="$OUT/prof_$tag.bin" timeout -k 10 120 python3 tools/probe_c2.py 4096 100000 -1 3 > "$OUT/probe_$tag.log" 2>&1 || { echo "probe failed"; tail -20 "$OUT/probe_$tag.log"; exit 1; }
  echo "== $tag"; tail -1 "$OUT/probe_$tag.log"
  python3 tools/deal_report.py "$OUT/prof_$tag.bin" 4096 10
done
