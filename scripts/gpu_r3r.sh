#!/bin/bash
# Shard floor vs split depth: cover 32/16 shards, reflect_refract 16 shards at RTC_SPLIT_MAX 2/3/4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
for envs in "RTC_SPLIT_MAX=2" "RTC_SPLIT_MAX=3" "RTC_SPLIT_MAX=4" "RTC_SPLIT_MAX=4 RTC_URGENT=0"; do
  for sc in "cover 3840 2160 8,32" "reflect_refract 1920 1080 4,16"; do
    set -- $sc
    echo "$envs"; env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' || exit 1
  done
done
