#!/bin/bash
# A/B timing of prebuilt libraries on one box: LIBS="path ..." PB="base indices" REP=n
# (each library runs the C2 probe per base, interleaved over REP repetitions).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-2}); do
  for L in ${LIBS:-flipcomplexityempirical_amd/libflipchain.so}; do
    for b in ${PB:--1}; do
      echo "[$(basename $L) rep $rep] $(FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-10000} $b 3 2>&1 | tail -1)" || exit 1
    done
  done
done
