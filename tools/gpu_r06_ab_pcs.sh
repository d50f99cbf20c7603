#!/bin/bash
# Round 6: A/B of abl/ variant libraries on the C2 probe (mix, base-6.96 chains one per SIMD,
# base-10 chains four per SIMD), then a PC-sampling profile of the product kernel on base-6.96
# chains alone (the slowest chain's serial path).  Usage: bash tools/gpu_r06_ab_pcs.sh TAG libA libB ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
TAG=$1; shift
OUT=$R/gpurun_out/ab_$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    for cfg in "4096 100000 -1 3" "1024 100000 8 3" "4096 100000 9 3"; do
      echo "[$lib rep$rep $cfg]" >> "$OUT/ab.txt"
      FC_LIB_PATH=$R/abl/$lib.so timeout -k 10 120 python3 tools/probe_c2.py $cfg >> "$OUT/ab.txt" 2>> "$OUT/ab.err" || { echo "probe failed $lib $cfg"; tail -20 "$OUT/ab.err"; exit 1; }
    done
  done
done
cat "$OUT/ab.txt"
if [ -n "$PCS" ]; then
  rc=0
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval 65536 -d "$OUT/pcs" -o pcs --output-format csv -- python3 tools/probe_c2.py 1024 20000 8 2 \
    > "$OUT/pcs.log" 2>&1 || rc=$?
  echo "stochastic rc=$rc"; tail -5 "$OUT/pcs.log"
  if [ $rc -eq 1 ] || [ $rc -eq 2 ]; then
    timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
      --pc-sampling-interval 1 -d "$OUT/pch" -o pch --output-format csv -- python3 tools/probe_c2.py 1024 20000 8 2 \
      > "$OUT/pch.log" 2>&1 || { echo "host_trap failed"; tail -20 "$OUT/pch.log"; exit 1; }
    echo host_trap ok
  fi
  find "$OUT" -name "*.csv" | head
fi
echo AB_DONE
