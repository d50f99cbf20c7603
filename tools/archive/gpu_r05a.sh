#!/bin/bash
# r05a: the new k > 2 native-RNG replay / KS tests and the RCCL branch, then the whole -m gpu suite and smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_node_tape_gpu.py tests/test_distribution_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest_r05a_new.log" 2>&1 || { echo "new tests failed"; tail -60 "$OUT/pytest_r05a_new.log"; exit 1; }
tail -3 "$OUT/pytest_r05a_new.log"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_r05a_all.log" 2>&1 || { echo "suite failed"; tail -60 "$OUT/pytest_r05a_all.log"; exit 1; }
tail -3 "$OUT/pytest_r05a_all.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_r05a.log" 2>&1 || { echo "smoke failed"; tail -40 "$OUT/smoke_r05a.log"; exit 1; }
tail -2 "$OUT/smoke_r05a.log"
echo ALL_OK
