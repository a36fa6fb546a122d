#!/bin/bash
# are the main kernel's loads the limit? C4 kernel time of the closing source (r5c), with reads
# synthesised in registers (a_noload), the key build alone (a_keyonly) and the key build alone
# without loads (a_keyonly_noload); timing-only ablations (tools/ablate.py)
set -o pipefail
O=gpurun_out/r05noload; mkdir -p $O
bash tools/ab_libs.sh $O r5c a_noload a_keyonly a_keyonly_noload > /dev/null 2>&1 || exit 1
cat $O/ab.txt
