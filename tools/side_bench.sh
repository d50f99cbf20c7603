#!/bin/bash
# Side measurements of the non-headline BASELINE configs (c3, c4, c5) on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
for W in c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $W --steps 3 --warmup 1 --chain-steps ${CHAIN_STEPS:-5000} --no-cpu-baseline --full-diag-steps 0 > "$OUT/side_${W}_$TAG.json" 2> "$OUT/side_${W}_$TAG.err" || { echo "side $W failed"; tail -30 "$OUT/side_${W}_$TAG.err"; exit 1; }
  cat "$OUT/side_${W}_$TAG.json"
done
echo SIDE_OK
