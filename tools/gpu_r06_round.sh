#!/bin/bash
# Round 6 evidence run: GPU suite, then the profile set (tools/gpu_profile.sh: bench line, kernel
# trace, PMC traffic / LDS counters, k > 2 side lines and their counters), the L1 / L2 counters of
# C2 and C3 (tools/gpu_cache_pmc.sh), the ReCom side line and the smoke.  Usage: TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
bash tools/gpu_profile.sh $TAG || exit 1
echo ROUND_OK
