#!/bin/bash
# Round-4 session C: k > 2 occupancy A/B (FC_K_WAVES8 = 4 (product) / 5 / 6 / 8 waves per SIMD,
# prebuilt under ablibs/) on C3 and C4, then the L1 / L2 / wave-state counter passes of C2, C3, C5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
WL="c3 c4" STEPS=20000 bash tools/archive/ab_side.sh r04c flipcomplexityempirical_amd/libflipchain.so ablibs/libflipchain_w5.so ablibs/libflipchain_w6.so ablibs/libflipchain_w8.so || exit 1
bash tools/gpu_cache_pmc.sh r04c c2 c3 c5 || exit 1
echo R04C_OK
