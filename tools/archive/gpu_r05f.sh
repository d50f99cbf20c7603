#!/bin/bash
# r05f: tally log -- the k = 2 diagnostic parity tests, the whole suite, then A/B against the
# round-4 library on the full-diagnostics instance, and the bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r05f; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "suite failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
DIAG="15 31" REP=2 bash tools/archive/ab_diag.sh abl/base.so abl/tlog.so > "$OUT/ab.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.txt"; exit 1; }
cat "$OUT/ab.txt"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-diag-steps 3 --sweep-replicas 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/bench.json')); f=j['full_diagnostics']; print('c2', j['value'], j['roofline']['kernel_ms'], 'full', f['value'], f['kernel_ms'], f['value_with_frame_series_on_host'], f['frame_series']['ms_per_launch'], 'sweeps', j['reference_sweeps']['wall_s'])"
echo R05F_OK
