#!/bin/bash
# Round-3 final evidence on HEAD: profile set (rocprofv3 stats + PMC), bench lines, 8-shard times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROUND=r03 bash scripts/profile_round.sh || exit $?
ROUND=r03 bash scripts/round_bench.sh || exit $?
for sc in "cover 3840 2160 1,2,4,8" "table 3840 2160 1,2,4,8" "reflect_refract 1920 1080 1,4"; do
  set -- $sc
  SHARD_COUNTS=$4 timeout -k 10 180 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r03_shard_times.txt || exit 1
done
