#!/bin/bash
# Two-rank rehearsals on one GPU (bench.py --gpus 2 launching its own ranks, gloo, both on
# device 0) against one rank holding the same global chains: C2 and C3, reduced statistics
# compared by tools/rehearsal_check.py.  (The rehearsal steps of tools/archive/gpu_r04a.sh.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p "$OUT"
TAG=${1:-reh}
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B --chains 4096 > "$OUT/reh_c2_n1_$TAG.json" 2> "$OUT/reh_c2_n1_$TAG.err" || { echo "c2 n1 failed"; tail -30 "$OUT/reh_c2_n1_$TAG.err"; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 300 $B --gpus 2 --chains 2048 > "$OUT/reh_c2_n2_$TAG.json" 2> "$OUT/reh_c2_n2_$TAG.err" || { echo "c2 n2 failed"; tail -30 "$OUT/reh_c2_n2_$TAG.err"; exit 1; }
timeout -k 10 300 $B --workload c3 --chain-steps 20000 --chains 16384 > "$OUT/reh_c3_n1_$TAG.json" 2> "$OUT/reh_c3_n1_$TAG.err" || { echo "c3 n1 failed"; tail -30 "$OUT/reh_c3_n1_$TAG.err"; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 300 $B --workload c3 --chain-steps 20000 --gpus 2 --chains 8192 > "$OUT/reh_c3_n2_$TAG.json" 2> "$OUT/reh_c3_n2_$TAG.err" || { echo "c3 n2 failed"; tail -30 "$OUT/reh_c3_n2_$TAG.err"; exit 1; }
python tools/rehearsal_check.py "$OUT/reh_c2_n1_$TAG.json" "$OUT/reh_c2_n2_$TAG.json" "$OUT/reh_c3_n1_$TAG.json" "$OUT/reh_c3_n2_$TAG.json" | tee "$OUT/reh_check_$TAG.txt"
echo REHEARSAL_OK
