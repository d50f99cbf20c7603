#!/bin/bash
# One GPU-box session: the whole -m gpu suite, smoke(), the bench line.  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r02}
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -40 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed"; tail -40 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
echo ALL_OK
