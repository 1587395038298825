#!/bin/bash
# (historical: RTC_POOL_GRID was measured, rejected and removed from the tree)
# Pool kernel grid below the resident one (RTC_POOL_GRID) on 8-way shards and whole frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
for envs in "X=0" "RTC_POOL_GRID=1280" "RTC_POOL_GRID=1024" "RTC_POOL_GRID=768"; do
  for sc in "cover 3840 2160 1,8" "table 3840 2160 1,8" "reflect_refract 1920 1080 1,4"; do
    set -- $sc
    echo "$envs :: $(env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' | tr '\n' ' ')"
  done
done
