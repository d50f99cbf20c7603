#!/bin/bash
# k > 2 side configs under alternative launch tuning (TUNES="wl:tune ..."), one bench line each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/side_tune; mkdir -p "$OUT"
for wt in ${TUNES}; do
  w=${wt%%:*}; t=${wt#*:}
  timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0 --tune "$t" > "$OUT/$w.json" 2> "$OUT/$w.err" || { echo "side $w $t failed"; tail -20 "$OUT/$w.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/$w.json')); print('$w', '$t', d['value'], d['ms_per_step'], d['roofline']['kernel'])"
done
