#!/bin/bash
# N > 1 rehearsal on one GPU: two gloo ranks on device 0 (2048 chains each) against one rank with
# 4096 chains; the reduced full-diagnostics checksums must be identical.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/rehearsal; mkdir -p "$OUT"
A="--steps 3 --warmup 1 --no-cpu-baseline --full-diag-steps 1"
timeout -k 10 400 python3 bench.py $A > "$OUT/n1.json" 2> "$OUT/n1.err" || { echo "n1 failed"; tail -20 "$OUT/n1.err"; exit 1; }
FC_BENCH_BACKEND=gloo FC_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --chains 2048 $A > "$OUT/n2.json" 2> "$OUT/n2.err" || { echo "n2 failed"; tail -20 "$OUT/n2.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
a = json.loads(open(o + "/n1.json").read().strip().splitlines()[-1])
b = json.loads(open(o + "/n2.json").read().strip().splitlines()[-1])
ra, rb = a["full_diagnostics"]["reduced"], b["full_diagnostics"]["reduced"]
print("n1", ra["ranks"], ra["yields"], ra["checksums"])
print("n2", rb["ranks"], rb["yields"], rb["checksums"])
print("IDENTICAL" if ra["checksums"] == rb["checksums"] and ra["yields"] == rb["yields"] else "DIFFERENT")
PY
