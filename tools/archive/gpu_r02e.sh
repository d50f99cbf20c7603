#!/bin/bash
# Corrected-statistics GPU tests, then the phase profile of the k = 2 kernel at bases mu and 10.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_corrected_stats_gpu.py tests/test_checkpoint_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest_r02e.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_r02e.log"; [ $rc -eq 0 ] || exit $rc
PB="6 9" bash tools/prof_run.sh > "$OUT/phase_r02e.txt" 2>&1 || { tail -20 "$OUT/phase_r02e.txt"; exit 1; }
cat "$OUT/phase_r02e.txt"
