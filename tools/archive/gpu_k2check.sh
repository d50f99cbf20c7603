#!/bin/bash
# k = 2 kernel change check: the k = 2 parity tests, then an A/B of prebuilt libraries
# (LIBS, PB, REP, STEPS as tools/archive/ab.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_corrected_stats_gpu.py tests/test_chain_gpu.py \
  tests/test_variants_gpu.py tests/test_checkpoint_gpu.py tests/test_node_tape_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_k2.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_k2.log"; [ $rc -eq 0 ] || exit $rc
bash tools/archive/ab.sh
