#!/bin/bash
# Round 6: A/B of abl/ variant libraries on the k > 2 side configurations (tools/probe_side.py,
# resident chains, 20,000 steps per launch, 3 launches), two repetitions interleaved.
# Usage: WL="c3 c4 c5" bash tools/gpu_r06_kgt2_ab.sh TAG libA libB ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/kab_$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for w in ${WL:-c3 c4 c5}; do
    for lib in "$@"; do
      echo "[$lib rep$rep $w]" >> "$OUT/ab.txt"
      FC_LIB_PATH=$R/abl/$lib.so timeout -k 10 150 python3 tools/probe_side.py $w 0 20000 3 >> "$OUT/ab.txt" 2>> "$OUT/ab.err" || { echo "probe failed $lib $w"; tail -20 "$OUT/ab.err"; exit 1; }
    done
  done
done
cat "$OUT/ab.txt"
echo KAB_OK
