#!/bin/bash
# Env-knob sweep of the headline kernel on the full C2 launch (4096 chains, 100,000 steps):
# KNOBS="FC_PAR_MIN=2 FC_PRIO_TH=0.9,1,1.1 ..." (each item: space-free VAR=value[+VAR=value]).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-1}); do
  for K in base ${KNOBS}; do
    ENVS=""; [ "$K" != base ] && ENVS=$(echo "$K" | tr '+' ' ')
    echo "[$K rep $rep] $(env $ENVS timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 2>&1 | tail -1)" || exit 1
  done
done
