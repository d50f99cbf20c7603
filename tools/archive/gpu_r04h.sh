#!/bin/bash
# Round-4 session H: the whole -m gpu suite, smoke, the default bench line (reference-sweep side
# line included), then the profile set (rocprofv3 stats, PMC passes, side configs) and the
# L1 / L2 passes of the new C3 instance.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r04h}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu_$TAG.log"; exit 1; }
tail -2 "$OUT/pytest_gpu_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -40 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
bash tools/gpu_profile.sh $TAG || exit 1
bash tools/gpu_cache_pmc.sh $TAG c3 > "$OUT/cache_$TAG.txt" 2>&1 || { tail -20 "$OUT/cache_$TAG.txt"; exit 1; }
echo R04H_OK
