#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats and PMC passes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -3 "$OUT/pytest_gpu_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -40 "$OUT/smoke_$TAG.log"; exit 1; }
tail -2 "$OUT/smoke_$TAG.log"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed"; tail -40 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-diag-steps 0 > "$OUT/prof_$TAG.log" 2>&1 || { echo "rocprof failed"; tail -40 "$OUT/prof_$TAG.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d "$OUT/pmc_${C}_$TAG" -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --full-diag-steps 0 > "$OUT/pmc_${C}_$TAG.log" 2>&1 || { echo "pmc $C failed"; tail -40 "$OUT/pmc_${C}_$TAG.log"; exit 1; }
done
echo ALL_OK
