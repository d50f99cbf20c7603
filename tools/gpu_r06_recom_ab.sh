#!/bin/bash
# ReCom A/B of abl/ variant libraries (bench.py --workload recom), 2 reps each.  Usage: TAG libA libB ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/recom_ab_$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    FC_LIB_PATH=$R/abl/$lib.so timeout -k 10 200 python3 bench.py --workload recom --steps 3 --warmup 1 --no-cpu-baseline --allow-variant > "$OUT/$lib.$rep.json" 2> "$OUT/$lib.$rep.err" || { echo "recom $lib failed"; tail -20 "$OUT/$lib.$rep.err"; exit 1; }
    python3 -c "import json; j=json.loads(open('$OUT/$lib.$rep.json').read().strip().splitlines()[-1]); print('$lib rep$rep', '%.4e' % j['value'], round(j['kernel_ms'], 2), round(j['trees_per_step'], 4))"
  done
done
echo RECOM_AB_OK
