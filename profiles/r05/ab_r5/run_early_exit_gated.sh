#!/bin/bash
# early exit with a batch-level gate (ee72g): C4 A/B (4 runs each) and C2 against r5a
set -o pipefail
O=gpurun_out/ee72g; mkdir -p $O
bash tools/ab_libs.sh $O/c4a r5a ee72g || exit 1
bash tools/ab_libs.sh $O/c4b ee72g r5a || exit 1
bash tools/ab_cfgs.sh $O/cfg "r5a ee72g" "30:30:67108864" || exit 1
