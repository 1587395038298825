#!/bin/bash
# One GPU call for a round's measurements: the profile set
# (scripts/profile_round.sh), the bench lines (scripts/round_bench.sh) and the
# 8-way shard times of cover and table at 4K (scripts/shard_times.py).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
export ROUND=${ROUND:-r05}
bash scripts/profile_round.sh > gpurun_out/${ROUND}_profset.log 2>&1 || { echo "profile set failed"; exit 1; }
echo "profile set ok"
bash scripts/round_bench.sh > gpurun_out/${ROUND}_bench.log 2>&1 || { echo "bench lines failed"; exit 1; }
echo "bench lines ok"
{ SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py cover 3840 2160 &&
  SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py table 3840 2160; } > gpurun_out/${ROUND}_shard_times.txt 2>&1 || { echo "shard times failed"; exit 1; }
echo "all ok"
