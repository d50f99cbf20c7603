#!/bin/bash
# Round-2 check: the new parity / replay / pin tests, then the side-config probes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_pair_gpu.py tests/test_series_gpu.py tests/test_node_tape_gpu.py \
  tests/test_distribution_gpu.py tests/test_reference_pin_gpu.py tests/test_parity_gpu.py::test_c1_grid10 \
  -x -v -s -m gpu --timeout 400 --timeout-method thread > "$OUT/pytest_gpu_r02c.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu_r02c.log"; [ $rc -eq 0 ] || exit $rc
for w in c3 c4 c5; do
  timeout -k 10 120 python tools/probe_side.py $w 0 2000 2 > "$OUT/side_$w.log" 2>&1 || { tail "$OUT/side_$w.log"; exit 1; }
  cat "$OUT/side_$w.log"
done
