#!/bin/bash
# r05h: whole -m gpu suite, then the bench line with the full-diagnostics leg under rocprofv3
# --stats (flip kernels, tally reduce, frame series kernels), then the plain bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r05h; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "suite failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_full" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --full-diag-steps 3 --sweep-replicas 0 > "$OUT/trace_full.log" 2>&1 || { echo "trace full failed"; tail -20 "$OUT/trace_full.log"; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace_full/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,3), round(float(r['MinNs'])/1e6,3), round(float(r['MaxNs'])/1e6,3))
"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-diag-steps 3 --sweep-replicas 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/bench.json')); f=j['full_diagnostics']; print('c2', j['value'], j['roofline']['kernel_ms'], 'full', f['value'], f['kernel_ms'], f['value_with_frame_series_on_host'], f['frame_series']['ms_per_launch'], 'sweeps', j['reference_sweeps']['wall_s'])"
echo R05H_OK
