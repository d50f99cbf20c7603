#!/bin/bash
# Round-4 session A: the new GPU tests first, the whole -m gpu suite, smoke, then the N-rank
# bench rehearsals on one GPU (bench.py --gpus 2 launching its own ranks, gloo, both on device
# 0) against one rank holding the same global chains.  Each GPU step has its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r04a}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_sweep_gpu.py tests/test_production_gpu.py > "$OUT/pytest_new_$TAG.log" 2>&1 || { echo "new tests failed"; tail -60 "$OUT/pytest_new_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_new_$TAG.log"
timeout -k 10 900 $T tests -m gpu > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo "pytest failed"; tail -60 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_gpu_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -40 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B --chains 4096 > "$OUT/reh_c2_n1_$TAG.json" 2> "$OUT/reh_c2_n1_$TAG.err" || { echo "c2 n1 failed"; tail -30 "$OUT/reh_c2_n1_$TAG.err"; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 300 $B --gpus 2 --chains 2048 > "$OUT/reh_c2_n2_$TAG.json" 2> "$OUT/reh_c2_n2_$TAG.err" || { echo "c2 n2 failed"; tail -30 "$OUT/reh_c2_n2_$TAG.err"; exit 1; }
timeout -k 10 300 $B --workload c3 --chain-steps 20000 --chains 16384 > "$OUT/reh_c3_n1_$TAG.json" 2> "$OUT/reh_c3_n1_$TAG.err" || { echo "c3 n1 failed"; tail -30 "$OUT/reh_c3_n1_$TAG.err"; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 300 $B --workload c3 --chain-steps 20000 --gpus 2 --chains 8192 > "$OUT/reh_c3_n2_$TAG.json" 2> "$OUT/reh_c3_n2_$TAG.err" || { echo "c3 n2 failed"; tail -30 "$OUT/reh_c3_n2_$TAG.err"; exit 1; }
python tools/rehearsal_check.py "$OUT/reh_c2_n1_$TAG.json" "$OUT/reh_c2_n2_$TAG.json" "$OUT/reh_c3_n1_$TAG.json" "$OUT/reh_c3_n2_$TAG.json" | tee "$OUT/reh_check_$TAG.txt"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { echo "bench failed"; tail -40 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
echo ALL_OK
