#!/bin/bash
# the drop-in CLI end to end on the round-5 library: 50 Mb in 8 contigs at 30x/30x, reference CLI vs
# the native streaming walk and contig groups (outputs compared byte for byte)
set -o pipefail
mkdir -p gpurun_out/r05cli
timeout -k 10 1000 bash tools/e2e_groups.sh 50000000 30 30 8 > gpurun_out/r05cli/e2e_groups_50Mb_8contigs.json 2> gpurun_out/r05cli/e2e.err || { tail -20 gpurun_out/r05cli/e2e.err; exit 1; }
cat gpurun_out/r05cli/e2e_groups_50Mb_8contigs.json
