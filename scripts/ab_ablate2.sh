#!/bin/bash
# Time breakdown of the direct kernel by ablation flags (outputs are wrong
# with flags; timing only): 4 = camera ray only, 2 = closest hit only,
# 3 = closest hit without counters, 0 = full.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
B="python bench.py --steps 300 --warmup 20 --no-cpu-baseline"
for sc in ${SCENES:-three_sphere_scene shadow_puppets}; do
  for v in ${VARIANTS:-default}; do
    lib=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib/librtc.so
    [ "$v" != default ] && lib=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib_$v/librtc.so
    for f in 0 4 2 1; do
      run "$v flags=$f $sc" env RTC_LIBRARY=$lib $B --scene $sc --flags $f
    done
  done
done
