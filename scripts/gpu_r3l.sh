#!/bin/bash
# generation-count priority raise (RTC_PRIO_GEN) and split 0.75 with urgent priority on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "RTC_PRIO_GEN=0" "RTC_PRIO_GEN=8" "RTC_SPLIT=0.75" "RTC_SPLIT=0.75 RTC_PRIO_GEN=8"; do
  for sc in cover table; do
    echo "$e"; env $e SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
AB_STEPS=200 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "RTC_PRIO_GEN=0" "RTC_PRIO_GEN=4" "RTC_PRIO_GEN=8" "RTC_PRIO_GEN=16" "RTC_SPLIT=0.75" "RTC_SPLIT=0.75 RTC_PRIO_GEN=8"
