#!/bin/bash
# Round-4 session B: C3 phase cycles (FC_PHASE_PROF build, built in-tree beforehand) and the
# gfx950 counter list (which TCP / TCC counters exist for the L1 / L2 pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r04b; mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "rocprofv3 -L rc $?"
grep -o "TC[CP]_[A-Za-z0-9_]*" "$OUT/counters_list.txt" | sort -u > "$OUT/tc_counters.txt" || true
wc -l "$OUT/tc_counters.txt"
WL=c3 STEPS=20000 bash tools/gpu_side_prof.sh r04b || exit 1
echo R04B_OK
