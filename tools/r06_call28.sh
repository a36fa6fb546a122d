#!/bin/bash
# Round 6: staged list appends + deep triage keys/8 loads in flight: probe,
# parity, benches, per-kernel times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_call24.sh && K="near_exit or synthetic_parity or deep_parity or group or mixed or misaligned or routing" bash tools/r06_call23.sh && bash tools/r06_call26.sh
