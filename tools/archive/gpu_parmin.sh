#!/bin/bash
# Per-base segment-parallel threshold probe: C2 chains of one base (PB base indices), par_min values (PM).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for b in ${PB:-4 7}; do
  for pm in ${PM:-2 3 4 6 64}; do
    echo "[base_idx $b par_min $pm] $(FC_TUNE=par_min=$pm timeout -k 10 120 python3 tools/probe_c2.py 4096 20000 $b 3 2>&1 | tail -1)" || exit 1
  done
done
