#!/bin/bash
# Experiment builds (timing-only A/B, never the product): the other sources compiled once, then
# one library per variant with extra -D flags on fc_flip2.hip (or the file given by VFILE):
#   bash tools/build_variants.sh name1 "-DFC_EXP_A" name2 "-DFC_EXP_B" ...  -> abl/<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/flipcomplexityempirical_amd/csrc
OBJ=/tmp/fc_varobj; mkdir -p "$OBJ" "$R/abl"
VFILE=${VFILE:-fc_flip2.hip}
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DFC_VARIANT_BUILD"
pids=()
for s in fc_flip2.hip fc_deal.hip fc_kernels.hip fc_series.hip fc_recom.hip fc_capi.cpp fc_graph.cpp; do
  [ "$s" = "$VFILE" ] && continue
  o=$OBJ/${s%.*}.o
  if [ ! -f "$o" ] || [ "$CS/$s" -nt "$o" ] || [ -n "$(find $CS -name '*.h' -newer $o)" ]; then
    eval /opt/rocm/bin/hipcc $F -c -o "$o" "$CS/$s" & pids+=($!)
  fi
done
while [ $# -ge 2 ]; do
  n=$1; fl=$2; shift 2
  ( eval /opt/rocm/bin/hipcc $F $fl -c -o "$OBJ/v_$n.o" "$CS/$VFILE" ) & pids+=($!)
  names+=($n)
done
for p in "${pids[@]}"; do wait $p; done
for n in "${names[@]}"; do
  objs=""
  for s in fc_flip2.hip fc_deal.hip fc_kernels.hip fc_series.hip fc_recom.hip fc_capi.cpp fc_graph.cpp; do
    if [ "$s" = "$VFILE" ]; then objs="$objs $OBJ/v_$n.o"; else objs="$objs $OBJ/${s%.*}.o"; fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o "$R/abl/$n.so" $objs
  echo "built abl/$n.so"
done
