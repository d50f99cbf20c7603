#!/bin/bash
# SQ counter passes over single-base probe runs (one rocprofv3 --pmc pass per counter group).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/sq; mkdir -p "$OUT"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM"
G2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
for b in ${BASES:-5 0 9}; do
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/b${b}_g$i" -o pmc --output-format csv -- python3 tools/probe_c2.py 4096 10000 $b 3 > "$OUT/b${b}_g$i.log" 2>&1 || { echo "pmc b$b g$i failed"; tail -20 "$OUT/b${b}_g$i.log"; exit 1; }
  done
done
echo PMC_OK
