#!/bin/bash
# 8-part splits (RTC_SPLIT_MAX=3) on 8-way shards and whole frames; split exactness test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -k "split" -q -p no:cacheprovider 2>&1 | tail -3
for cfg in "RTC_SPLIT_MAX=2" "RTC_SPLIT_MAX=3" "RTC_SPLIT_MAX=3 RTC_SPLIT=0.75"; do
  for sc in cover table; do
    echo "$cfg"; env $cfg SHARD_COUNTS=1,8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo "$cfg"; env $cfg SHARD_COUNTS=1,4 timeout -k 10 120 python scripts/shard_times.py reflect_refract 1920 1080 2>&1 | grep -v amdgpu.ids || exit 1
done
