#!/bin/bash
# k > 2 side configs (C3 / C4 / C5) over launch-tuning variants: TUNES="nsub=1 nsub=2 ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for w in ${WORKLOADS:-c3 c4 c5}; do
  for T in ${TUNES:-nsub=1}; do
    echo "[$w $T] $(FC_TUNE="$T" timeout -k 10 120 python3 tools/probe_side.py $w 0 ${STEPS:-2000} 3 2>&1 | tail -1)" || exit 1
  done
done
