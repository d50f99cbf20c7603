#!/bin/bash
# A/B of prebuilt library variants on a side workload (tools/probe_side.py):
#   WL=c4 bash tools/archive/ab_side.sh <tag> lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/abs_$TAG; mkdir -p "$OUT"
for w in ${WL:-c4 c5}; do
  for rep in 1 2; do
    for L in "$@"; do
      n=$(basename $L .so)
      FC_LIB_PATH=$R/$L timeout -k 10 150 python3 tools/probe_side.py $w 0 ${STEPS:-20000} 3 > "$OUT/${w}_${n}_$rep.log" 2>&1 || { echo "probe $w $n failed"; tail -20 "$OUT/${w}_${n}_$rep.log"; exit 1; }
      echo "$w $n rep $rep: $(tail -1 $OUT/${w}_${n}_$rep.log | cut -c1-110)"
    done
  done
done
