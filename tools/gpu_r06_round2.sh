#!/bin/bash
# Round 6 evidence, second part: L1 / L2 counters of C2 and C3, the ReCom side line with its
# kernel trace, and the cooperative-search probe.  Usage: TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out
bash tools/gpu_cache_pmc.sh $TAG c2 c3 || exit 1
timeout -k 10 300 python3 bench.py --workload recom --steps 3 --warmup 1 > gpurun_out/${TAG}_side_recom.json 2> gpurun_out/${TAG}_side_recom.err || { echo "recom failed"; tail -20 gpurun_out/${TAG}_side_recom.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_recom_trace -o run --output-format csv -- python3 bench.py --workload recom --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_recom_trace.log 2>&1 || { echo "recom trace failed"; tail -20 gpurun_out/${TAG}_recom_trace.log; exit 1; }
cat gpurun_out/${TAG}_side_recom.json
timeout -k 10 400 python3 tools/probe_coop.py 1000 > gpurun_out/${TAG}_coop_probe.txt 2>&1 || { echo "coop probe failed"; tail -20 gpurun_out/${TAG}_coop_probe.txt; exit 1; }
cat gpurun_out/${TAG}_coop_probe.txt
echo ROUND2_OK
