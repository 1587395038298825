#!/bin/bash
# Round-3 profile set and bench lines (scripts/profile_round.sh, scripts/round_bench.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=r03 bash scripts/profile_round.sh || exit $?
ROUND=r03 bash scripts/round_bench.sh || exit $?
