#!/bin/bash
# split-factor sweep (RTC_SPLIT) on full frames and 8-way shards, per-scene kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sp in 1.5 1.0 0.75 0.5; do
  for sc in cover table; do
    echo "RTC_SPLIT=$sp"; RTC_SPLIT=$sp SHARD_COUNTS=1,8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo "RTC_SPLIT=$sp"; RTC_SPLIT=$sp SHARD_COUNTS=1,4 timeout -k 10 120 python scripts/shard_times.py reflect_refract 1920 1080 2>&1 | grep -v amdgpu.ids || exit 1
done
