#!/bin/bash
# main-kernel phase accounting on the closing round-5 source: VALU / SALU / LDS per site of
# timing-only ablation builds (tools/ablate.py), then their C4 kernel times (tools/ab_libs.sh)
set -o pipefail
O=gpurun_out/r05phases; mkdir -p $O
bash tools/sq_variants.sh r5c a_nonet a_nofold a_nofin a_nominor a_nodecide a_keyonly > $O/valu.txt 2>&1 || { cat $O/valu.txt; exit 1; }
cat $O/valu.txt
bash tools/ab_libs.sh $O/t r5c a_nonet a_nofold a_nofin a_nominor a_nodecide a_keyonly > /dev/null 2>&1 || exit 1
cat $O/t/ab.txt
