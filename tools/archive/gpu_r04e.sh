#!/bin/bash
# Round-4 session E: k > 2 draw rounds per batch with the multi-flip commit (scheduling only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for w in c3 c4 c5; do
  for t in nsub=1 nsub=2 nsub=4 hit_stop=16 hit_stop=48; do
    echo "$w $t: $(FC_TUNE=$t timeout -k 10 150 python3 tools/probe_side.py $w 0 20000 3 2>&1 | tail -1 | cut -c1-120)" || exit 1
  done
done
echo R04E_OK
