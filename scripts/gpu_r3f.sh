#!/bin/bash
# (1) A/B: static build without machine LICM (f64 kernels, generic f32 kernels)
# (2) PMC of reflect_refract after the AoS spill change
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source scripts/ab_lib.sh
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
for r in 1 2; do
  for v in _lib _lib_nolicm; do
    for sc in reflect_refract:1920:1080 cover:3840:2160 three_sphere_scene:1920:1080; do
      IFS=: read n w h <<< "$sc"
      run "$v f64 $n" env RTC_LIBRARY=$L/$v/librtc.so python bench.py --scene $n --width $w --height $h --precision f64 --steps 100 --warmup 10 --no-cpu-baseline || exit 1
      run "$v generic-f32 $n" env RTC_JIT=0 RTC_LIBRARY=$L/$v/librtc.so python bench.py --scene $n --width $w --height $h --steps 200 --warmup 10 --no-cpu-baseline || exit 1
    done
  done
done
PMC_NAME=r03_pmc_reflect_refract BENCH_ARGS="--scene reflect_refract" bash scripts/pmc.sh "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" || exit 1
