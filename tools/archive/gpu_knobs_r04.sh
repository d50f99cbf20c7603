#!/bin/bash
# Round-4 scheduling knobs on the faster k = 2 kernel: chain dealing and issue priorities,
# full C2 launches (tools/probe_c2.py, 4096 chains x 100,000 steps), two reps each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for rep in 1 2; do
  for t in ${KNOBS:-"" "deal=1" "prio_div=-1" "prio_div=2:4:8" "prio_div=3:6:12" "prio_th=-1" "prio_div=1:2:5"}; do
    echo "[$t] rep $rep: $(FC_TUNE=$t timeout -k 10 120 python3 tools/probe_c2.py 4096 100000 -1 3 2>&1 | tail -1)" || exit 1
  done
done
