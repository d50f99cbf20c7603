#!/bin/bash
# Round-4 session D: C2 phase cycles per base (FC_PHASE_PROF build) at the bench's launch shape,
# and the C4 L1 / L2 counter passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
STEPS=100000 PB=-1 bash tools/prof_run.sh | tee gpurun_out/phase_r04d.txt || exit 1
bash tools/gpu_cache_pmc.sh r04d c4 > gpurun_out/cache_r04d.txt 2>&1 || { tail -20 gpurun_out/cache_r04d.txt; exit 1; }
echo R04D_OK
