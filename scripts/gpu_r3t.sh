#!/bin/bash
# Cold-launch cost probe sweep (RTC_COLD_PROBE=wr,wt[,split]); cold_kernel_ms per scene, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
AB_STEPS=40 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "X=0" "RTC_COLD_PROBE=0" \
  "RTC_COLD_PROBE=8,24,1" "RTC_COLD_PROBE=8,64" "RTC_COLD_PROBE=8,64,1" "RTC_COLD_PROBE=16,128,1" "RTC_COLD_PROBE=4,32,1"
