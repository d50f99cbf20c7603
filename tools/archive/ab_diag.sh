#!/bin/bash
# A/B of prebuilt libraries (abl/*.so) on the C2 probe with a given diagnostics mask:
#   DIAG=15 REP=2 bash tools/archive/ab_diag.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-2}); do
  for D in ${DIAG:-15}; do
    for L in "$@"; do
      echo "[$(basename $L) diag $D rep $rep] $(FC_PROBE_DIAG=$D FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 2>&1 | tail -1)" || exit 1
    done
  done
done
