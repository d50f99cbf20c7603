#!/bin/bash
# Per-base A/B of launch knobs: PB="base indices" KNOBS="k=v[,k=v] ..." STEPS (default 10000);
# every chain of a run on one base (tools/probe_c2.py), then the phase profile of the last knob.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
for b in ${PB:-6 9}; do
  for K in base ${KNOBS}; do
    T=""; [ "$K" != base ] && T="$K"
    echo "[b$b $K] $(FC_TUNE="$T" timeout -k 10 120 python3 tools/probe_c2.py 4096 ${STEPS:-10000} $b 3 2>&1 | tail -1)" || exit 1
  done
done
if [ -n "$PROF_KNOB" ]; then
  for b in ${PB:-6 9}; do
    FC_TUNE="$PROF_KNOB" FC_LIB_VARIANT=prof FC_PROF_OUT=/tmp/p_$b.bin timeout -k 10 120 python3 tools/probe_c2.py 4096 10000 $b 2 > /tmp/pp.log 2>&1 || { tail /tmp/pp.log; exit 1; }
    echo "[prof b$b $PROF_KNOB]"; python3 tools/prof_report.py /tmp/p_$b.bin 4096 1
  done
fi
