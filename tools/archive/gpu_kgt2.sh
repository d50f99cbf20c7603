#!/bin/bash
# k > 2 kernel change check: the k > 2 GPU parity tests, then the side-config bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_pair_gpu.py tests/test_series_gpu.py tests/test_corrected_stats_gpu.py \
  tests/test_checkpoint_gpu.py -x -q -m gpu --timeout 400 --timeout-method thread > "$OUT/pytest_kgt2.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_kgt2.log"; [ $rc -eq 0 ] || exit $rc
for w in ${WL:-c3 c4 c5}; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 5 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0 > "$OUT/side_$w.json" 2> "$OUT/side_$w.err" || { echo "side $w failed"; tail -20 "$OUT/side_$w.err"; exit 1; }
  python3 -c "import json; d = json.load(open('$OUT/side_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel'])"
done
