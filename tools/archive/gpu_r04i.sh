#!/bin/bash
# Round-4 session I: compiler scheduling strategies on the C2 launch (A/B, prebuilt in ablibs/),
# and the two-rank sweep rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
LIBS="flipcomplexityempirical_amd/libflipchain.so ablibs/libflipchain_max-ilp.so ablibs/libflipchain_max-memory-clause.so ablibs/libflipchain_o2.so" REP=2 bash tools/archive/ab_full.sh | tee gpurun_out/ab_r04i.txt || exit 1
WL="c3 c4" STEPS=20000 bash tools/archive/ab_side.sh r04i flipcomplexityempirical_amd/libflipchain.so ablibs/libflipchain_max-ilp.so ablibs/libflipchain_max-memory-clause.so | tee -a gpurun_out/ab_r04i.txt || exit 1
bash tools/sweep_rehearsal.sh | tee gpurun_out/sweep_rehearsal_r04i.txt || exit 1
echo R04I_OK
