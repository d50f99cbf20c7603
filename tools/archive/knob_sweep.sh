#!/bin/bash
# Launch-tuning sweep of the headline kernel on the full C2 launch (4096 chains, 100,000 steps):
# KNOBS="par_min=2 prio_th=0.9:1:1.1 ..." (each item: a space-free fc_params.tune_* list,
# key=value[,key=value], passed to tools/probe_c2.py as FC_TUNE).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-1}); do
  for K in base ${KNOBS}; do
    T=""; [ "$K" != base ] && T="$K"
    echo "[$K rep $rep] $(FC_TUNE="$T" timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 2>&1 | tail -1)" || exit 1
  done
done
