#!/bin/bash
# Round 6: the GPU suite, then the k > 2 side lines (C3 / C4 / C5) on the product library, with
# window variants (tune nsub) of C3.  Usage: bash tools/gpu_r06_side.sh TAG [skip_tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1
OUT=$R/gpurun_out/side_$TAG; mkdir -p "$OUT"
if [ -z "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
SB="--steps 5 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0"
for w in c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --workload $w $SB > "$OUT/side_$w.json" 2> "$OUT/side_$w.err" || { echo "side $w failed"; tail -20 "$OUT/side_$w.err"; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('$OUT/side_$w.json').read().strip().splitlines()[-1]); print('$w', '%.3e' % j['value'], j['roofline']['kernel_ms'], j['roofline']['kernel'], 'draws/prop', round(j['draws_per_proposal'],2))"
done
for t in nsub=2 nsub=1; do
  timeout -k 10 300 python3 bench.py --workload c3 $SB --tune $t > "$OUT/side_c3_$t.json" 2> "$OUT/side_c3_$t.err" || { echo "side c3 $t failed"; tail -20 "$OUT/side_c3_$t.err"; exit 1; }
  python3 -c "import json,sys; j=json.loads(open('$OUT/side_c3_$t.json').read().strip().splitlines()[-1]); print('c3 $t', '%.3e' % j['value'], j['roofline']['kernel_ms'])"
done
echo SIDE_DONE
