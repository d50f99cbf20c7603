#!/bin/bash
# Profile evidence for one round (committed under profiles/ by tools/profile_summary.py):
#   bench line (headline C2), rocprofv3 --kernel-trace --stats of the same bench, separate
#   --pmc passes (FETCH_SIZE, WRITE_SIZE, LDS / issue counters), and the k > 2 side configs.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_$TAG; mkdir -p "$OUT"
BENCH="bench.py --steps 5 --warmup 1 --no-cpu-baseline --full-diag-steps 0 --sweep-replicas 0"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
# the full-diagnostics leg (the reference loop body's tallies) in its own traced run
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_full" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --full-diag-steps 3 --sweep-replicas 0 > "$OUT/trace_full.log" 2>&1 || { echo "trace full failed"; tail -20 "$OUT/trace_full.log"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d "$OUT/pmc_$C" -o pmc --output-format csv -- python3 $BENCH > "$OUT/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; tail -20 "$OUT/pmc_$C.log"; exit 1; }
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_lds" -o pmc --output-format csv -- python3 $BENCH > "$OUT/pmc_lds.log" 2>&1 || { echo "pmc lds failed"; tail -20 "$OUT/pmc_lds.log"; exit 1; }
for w in c3 c4 c5; do
  # C4 also runs its diagnostics leg (event log, hitting time, autocorrelation; BASELINE config 4)
  FD=0; [ $w = c4 ] && FD=2
  timeout -k 10 300 python3 bench.py --workload $w --steps 5 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps $FD > "$OUT/side_$w.json" 2> "$OUT/side_$w.err" || { echo "side $w failed"; tail -20 "$OUT/side_$w.err"; exit 1; }
  cat "$OUT/side_$w.json"
done
# counters of the k > 2 instances (C3 flip_kernel<8,2,3,false,2>, C4 flip_kernel<8,2,3,false,1>,
# C5 flip_kernel<16,4,3,false,1>)
for w in ${SIDE_PMC:-c3 c4 c5}; do
  SB="bench.py --workload $w --steps 2 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C -d "$OUT/side_pmc_${w}_$C" -o pmc --output-format csv -- python3 $SB > "$OUT/side_pmc_${w}_$C.log" 2>&1 || { echo "side pmc $w $C failed"; tail -20 "$OUT/side_pmc_${w}_$C.log"; exit 1; }
  done
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/side_pmc_${w}_lds" -o pmc --output-format csv -- python3 $SB > "$OUT/side_pmc_${w}_lds.log" 2>&1 || { echo "side pmc lds $w failed"; tail -20 "$OUT/side_pmc_${w}_lds.log"; exit 1; }
done
echo PROFILE_OK
