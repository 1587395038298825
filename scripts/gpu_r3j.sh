#!/bin/bash
# urgent-item wave priority: lower thresholds and graded levels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "RTC_URGENT=0" "RTC_URGENT=0.25" "RTC_URGENT=0.125" "RTC_URGENT=0.0625" "RTC_URGENT=0.125 RTC_URGENT_GRADED=1" "RTC_URGENT=0.0625 RTC_URGENT_GRADED=1"; do
  for sc in cover table; do
    echo "$e"; env $e SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
AB_STEPS=300 bash scripts/ab_env.sh "reflect_refract refraction metal cylinders cover:3840x2160 table:3840x2160" "RTC_URGENT=0" "RTC_URGENT=0.25" "RTC_URGENT=0.125" "RTC_URGENT=0.0625" "RTC_URGENT=0.125 RTC_URGENT_GRADED=1" "RTC_URGENT=0.0625 RTC_URGENT_GRADED=1"
