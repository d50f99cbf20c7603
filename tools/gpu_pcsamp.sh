#!/bin/bash
# PC sampling of the headline kernel (rocprofv3 beta): where the lean C2 kernel's issue time goes,
# per instruction.  One short launch (20,000 steps per chain).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/pcsamp_${1:-x}; mkdir -p "$OUT"
B="bench.py --steps 1 --warmup 1 --chain-steps 20000 --no-cpu-baseline --full-diag-steps 0 --sweep-replicas 0"
M=${2:-host_trap}
U=${3:-time}
I=${4:-1000}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U --pc-sampling-interval $I -d "$OUT/pc" -o pc --output-format csv -- python3 $B > "$OUT/pc.log" 2>&1 || { echo "pc sampling failed"; tail -30 "$OUT/pc.log"; exit 1; }
ls -la "$OUT/pc"/* | head
for f in "$OUT"/pc/*.csv; do echo "== $f"; head -3 "$f"; wc -l "$f"; done
echo PCSAMP_OK
