#!/bin/bash
# Round-4 session F: exact multi-flip marks (C3) -- parity tests, A/B against the hashed marks,
# draw rounds per batch, C3 phase cycles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r04f; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_production_gpu.py tests/test_pair_gpu.py > "$OUT/pytest.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
  for t in "" multi_flip=2 nsub=4 "nsub=4,multi_flip=2" nsub=1; do
    echo "c3 [$t] rep $rep: $(FC_TUNE=$t timeout -k 10 150 python3 tools/probe_side.py c3 0 20000 3 2>&1 | tail -1 | cut -c1-140)" || exit 1
  done
done
for w in c4 c5; do
  for t in "" nsub=4 nsub=1; do
    echo "$w [$t]: $(FC_TUNE=$t timeout -k 10 150 python3 tools/probe_side.py $w 0 20000 3 2>&1 | tail -1 | cut -c1-140)" || exit 1
  done
done
WL=c3 STEPS=20000 bash tools/gpu_side_prof.sh r04f || exit 1
echo R04F_OK
