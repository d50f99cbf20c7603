#!/bin/bash
# LDS / issue counters of the headline kernel (one rocprofv3 --pmc pass), summarised into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=${1:-r01}
OUT=$R/gpurun_out/pmc_lds_$TAG
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT" -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT.log" 2>&1 || { echo "pmc lds failed"; tail -20 "$OUT.log"; exit 1; }
python3 tools/pmc_lds_summary.py "$TAG"
