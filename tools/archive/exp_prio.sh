#!/bin/bash
# Issue-priority sweep of the k = 2 kernel on the C2 bench (fc_params tune_prio_div / tune_prio_th).
set -o pipefail
for P in ${PRIOS:-"prio_div=2:5:10 prio_div=-1:0:0"}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --tune "$P" > gpurun_out/prio.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/prio.json'));print('$P', '%.4e'%d['value'], d['ms_per_step'])"
done
