#!/bin/bash
# urgent-item wave priority (RTC_URGENT) sweep: 8-way shards at 4K and whole frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for u in 0 1.0 0.5 0.25; do
  for sc in cover table; do
    echo "RTC_URGENT=$u"; RTC_URGENT=$u SHARD_COUNTS=1,8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
  echo "RTC_URGENT=$u"; RTC_URGENT=$u SHARD_COUNTS=1,4 timeout -k 10 120 python scripts/shard_times.py reflect_refract 1920 1080 2>&1 | grep -v amdgpu.ids || exit 1
done
AB_STEPS=300 bash scripts/ab_env.sh "reflect_refract refraction cover:3840x2160 table:3840x2160" "RTC_URGENT=0" "RTC_URGENT=1.0" "RTC_URGENT=0.5" "RTC_URGENT=0.25"
