#!/bin/bash
# A/B of prebuilt library variants on the C2 probe (full 100,000-step launches):
#   bash tools/archive/ab_libs.sh <tag> lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/ab_$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 > "$OUT/${n}_$rep.log" 2>&1 || { echo "probe $n failed"; tail -20 "$OUT/${n}_$rep.log"; exit 1; }
    echo "$n rep $rep: $(tail -1 $OUT/${n}_$rep.log)"
  done
done
