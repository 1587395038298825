#!/bin/bash
# Driver-like short bench, then the urgency threshold (RTC_URGENT) re-swept on the specialised build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/driver_like.log 2>&1 || exit 1
grep '^{' gpurun_out/driver_like.log | cut -c1-400
for envs in "X=0" "RTC_URGENT=0.0625" "RTC_URGENT=0.25" "RTC_URGENT=0.5"; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8" "reflect_refract 1920 1080 4"; do
    set -- $sc
    echo "$envs :: $(env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/')"
  done
done
AB_STEPS=200 bash scripts/ab_env.sh "reflect_refract refraction cylinders cover:3840x2160 table:3840x2160" "X=0" "RTC_URGENT=0.0625" "RTC_URGENT=0.25"
