#!/bin/bash
# C2 probe (lean build, no stamps) over env settings x bases: PM="k=v,k=v ..." PB="bases"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/probe; mkdir -p "$OUT"
for cfg in ${PM:-"X=0"}; do
  for b in ${PB:--1 5 9}; do
    echo "[$cfg] $(env ${cfg//,/ } timeout -k 10 120 python3 tools/probe_c2.py 4096 10000 $b 3 2>&1 | tail -1)" || exit 1
  done
done
