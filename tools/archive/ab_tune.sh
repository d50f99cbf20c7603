#!/bin/bash
# A/B of launch tunings on one library (C2 probe, 4096 chains x 100,000 steps):
#   LIB=abl/x.so REP=2 bash tools/archive/ab_tune.sh "" "nsub=8" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-2}); do
  for T in "$@"; do
    echo "[$(basename ${LIB:-lib}) tune '$T' rep $rep] $(FC_TUNE="$T" FC_LIB_PATH=$R/${LIB:-flipcomplexityempirical_amd/libflipchain.so} timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} ${BASE:--1} 3 2>&1 | tail -1)" || exit 1
  done
done
