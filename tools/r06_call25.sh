#!/bin/bash
# Round 6: the deep triage after the round-count fix -- probe (debug-sync
# build), parity, then C5 / 1200x / C4 bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_call24.sh || exit $?
bash tools/r06_call23.sh
