#!/bin/bash
# A/B of prebuilt libraries on the full C2 launch (4096 chains, 100,000 steps per launch):
# LIBS="path ..." REP=n; EXTRA="VAR=value" adds one run of the first library under that env.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in $(seq 1 ${REP:-2}); do
  for L in ${LIBS}; do
    echo "[$(basename $L) rep $rep] $(FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 2>&1 | tail -1)" || exit 1
  done
done
if [ -n "$EXTRA" ]; then
  L=$(echo $LIBS | cut -d' ' -f1)
  echo "[$(basename $L) $EXTRA] $(env $EXTRA FC_LIB_PATH=$R/$L timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-100000} -1 3 2>&1 | tail -1)" || exit 1
fi
