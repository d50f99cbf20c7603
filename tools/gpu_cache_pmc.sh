#!/bin/bash
# Where the bytes come from: L1 (TCP), L2 (TCC) and wave-state counters of
# one workload's flip kernel, one rocprofv3 --pmc pass per block (each within its slot limits:
# 4 TCP, 4 TCC, 8 SQ), then tools/cache_pmc_summary.py -> profiles/<tag>_<wl>_l1l2.json.
#   bash tools/gpu_cache_pmc.sh <tag> [c2 c3 c5]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
for w in "${@:-c2}"; do
  OUT=$R/gpurun_out/cache_${TAG}_$w; mkdir -p "$OUT"
  if [ $w = c2 ]; then
    B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --full-diag-steps 0 --sweep-replicas 0"
  else
    B="bench.py --workload $w --steps 2 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0"
  fi
  timeout -k 10 300 python3 $B > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench $w failed"; tail -20 "$OUT/bench.err"; exit 1; }
  i=0
  for P in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_WRITE_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_FLAT"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P -d "$OUT/pmc$i" -o pmc --output-format csv -- python3 $B > "$OUT/pmc$i.log" 2>&1 || { echo "pmc pass $i ($w) failed"; tail -20 "$OUT/pmc$i.log"; exit 1; }
  done
  python3 tools/cache_pmc_summary.py "$TAG" "$w" | tail -25
done
echo CACHE_PMC_OK
