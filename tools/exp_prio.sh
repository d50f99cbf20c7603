#!/bin/bash
# Issue-priority sweep of the k = 2 kernel on the C2 bench (FC_PRIO_DIV / FC_PRIO_TH).
set -o pipefail
for P in ${PRIOS:-"2,5,10 -1,0,0"}; do
  export FC_PRIO_DIV=${P%|*} FC_PRIO_TH=${P#*|}
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/prio.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/prio.json'));print('$P', '%.4e'%d['value'], d['ms_per_step'])"
done
