#!/bin/bash
# round-5 closing measurements, part 2: C2 / C3 / C5 / 1200x1000 bench lines + rocprofv3 summaries
set -o pipefail
bash tools/profile_configs.sh r05cfg4
