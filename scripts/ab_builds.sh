#!/bin/bash
# A/B of build variants (built beforehand into rtc_amd/_lib_<name>/ with
# `make OUT=rtc_amd/_lib_<name> EXTRA=...`) selected per run via RTC_LIBRARY.
# Usage: ab_builds.sh "<variant> ..." "<scene> ..." ["<env assignments per run>" ...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
VARIANTS=${1:-default}
SCENES=${2:-three_sphere_scene}
shift 2 || true
ENVS=("${@:-X=0}")
B="python bench.py --steps ${AB_STEPS:-1000} --warmup 30 --no-cpu-baseline"
for sc in $SCENES; do
  for v in $VARIANTS; do
    lib=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib/librtc.so
    [ "$v" != default ] && lib=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib_$v/librtc.so
    for e in "${ENVS[@]}"; do
      run "$v [$e] $sc" env RTC_LIBRARY=$lib $e $B --scene $sc
    done
  done
done
