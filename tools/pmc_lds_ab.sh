#!/bin/bash
# LDS / issue counters of prebuilt library variants on the C2 probe (one rocprofv3 --pmc pass per
# library, 4096 chains x 100,000 steps, 2 launches), summarised by tools/pmc_lds_ab.py:
#   bash tools/pmc_lds_ab.sh <tag> abl/base.so abl/x.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/pmcab_$TAG; mkdir -p "$OUT"
for L in "$@"; do
  n=$(basename $L .so)
  export FC_LIB_PATH=$R/$L
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/$n" -o pmc --output-format csv -- python3 tools/probe_c2.py 4096 100000 -1 2 > "$OUT/$n.log" 2>&1 || { echo "pmc $n failed"; tail -20 "$OUT/$n.log"; exit 1; }
  echo "$n: $(tail -1 $OUT/$n.log)"
done
python3 tools/pmc_lds_ab.py "$OUT" "$@"
