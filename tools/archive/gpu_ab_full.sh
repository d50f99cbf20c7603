#!/bin/bash
# k = 2 full-diagnostics change check: the k = 2 diagnostic parity tests, then an A/B of
# prebuilt libraries (LIBS) on the C2 probe, lean (diag 1) and full (diag 15) instances.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_corrected_stats_gpu.py tests/test_chain_gpu.py \
  tests/test_checkpoint_gpu.py tests/test_series_gpu.py tests/test_slope_gpu.py tests/test_variants_gpu.py tests/test_node_tape_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_k2full.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_k2full.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for D in ${DIAGS:-15 1}; do
    for L in ${LIBS:-flipcomplexityempirical_amd/libflipchain.so}; do
      echo "[$(basename $L) diag $D rep $rep] $(FC_PROBE_DIAG=$D FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-20000} -1 3 2>&1 | tail -1)" || exit 1
    done
  done
done
