#!/bin/bash
# cold-launch tile-cost probe (RTC_COLD_PROBE) sweep: cold_kernel_ms of pool scenes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=100 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "RTC_COLD_PROBE=0" "RTC_COLD_PROBE=8,24" "RTC_COLD_PROBE=4,12" "RTC_COLD_PROBE=16,48" "RTC_COLD_PROBE=8,24,1" "RTC_COLD_PROBE=2,32"
bash scripts/pmc_ablate.sh || exit 1
