#!/bin/bash
# (1) shard time vs shard count (fixed cost a + b x work); (2) LDS pool size on shards; (3) per-scene headers dump
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/jit
export RTC_JIT_CACHE=0
for sc in "cover 3840 2160 1,2,4,8,16,32" "reflect_refract 1920 1080 1,2,4,8,16"; do
  set -- $sc
  SHARD_COUNTS=$4 timeout -k 10 180 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids || exit 1
done
for envs in "RTC_POOL_LDS_RAYS=768" "RTC_POOL_LDS_RAYS=1024" "RTC_POOL_LDS_RAYS=1792"; do
  for sc in "cover 3840 2160 1,8" "table 3840 2160 1,8" "reflect_refract 1920 1080 1,4"; do
    set -- $sc
    echo "$envs"; env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
RTC_JIT_DUMP=gpurun_out/jit timeout -k 10 60 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
RTC_JIT_DUMP=gpurun_out/jit timeout -k 10 60 python bench.py --scene reflect_refract --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
ls gpurun_out/jit
