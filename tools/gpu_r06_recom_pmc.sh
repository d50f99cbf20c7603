#!/bin/bash
# Round 6: instruction mix of the ReCom kernel (rocprofv3 --pmc, one pass, SQ counters only;
# bench.py --workload recom, one timed launch).  Usage: bash tools/gpu_r06_recom_pmc.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/recom_pmc_$1; mkdir -p "$OUT"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES \
  -d "$OUT" -o pmc --output-format csv -- python3 bench.py --workload recom --steps 1 --warmup 1 --no-cpu-baseline \
  > "$OUT/log.txt" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/log.txt"; exit 1; }
find "$OUT" -name "*counter_collection.csv" | head -3
echo PMC_OK
