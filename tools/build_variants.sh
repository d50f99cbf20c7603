#!/bin/bash
# Experiment builds (timing-only A/B, never the product): the other sources compiled once, then
# one library per variant with extra -D flags on fc_flip2.hip (or the file given by VFILE):
#   bash tools/build_variants.sh name1 "-DFC_EXP_A" name2 "-DFC_EXP_B" ...  -> abl/<name>.so
#   e.g. the LDS bank-conflict attribution builds (profiles/r05l_lds_conflict_attribution.json):
#   PATCH=tools/patches/lds_dup_attribution.patch bash tools/build_variants.sh base "" dup1 "-DFC_EXP_DUP=1" ...
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
# PATCH=<file>: the variants compile a patched copy of VFILE (tools/patches/; timing-only code
# stays out of the product sources)
SRC=$CS/$VFILE
if [ -n "$PATCH" ]; then
  SRC=$OBJ/patched_$VFILE
  cp "$CS/$VFILE" "$SRC"
  patch -s "$SRC" < "$PATCH"
  F="$F -I$CS"
fi
while [ $# -ge 2 ]; do
  n=$1; fl=$2; shift 2
  ( eval /opt/rocm/bin/hipcc $F $fl -c -o "$OBJ/v_$n.o" "$SRC" ) & pids+=($!)
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
