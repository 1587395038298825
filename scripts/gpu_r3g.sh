#!/bin/bash
# A/B: one-copy world staging (worktree) vs HEAD; LDS world / direct grid knobs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source scripts/ab_lib.sh
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
for r in 1 2; do
  for v in "_lib" "_lib_base" "_lib RTC_LDS_WORLD=0" "_lib_base RTC_LDS_WORLD=0"; do
    set -- $v; lib=$1; e=${2:-X=0}
    for sc in three_sphere_scene:1920:1080 shadow_puppets:1920:1080 three_sphere_scene:3840:2160 reflect_refract:1920:1080 cover:3840:2160; do
      IFS=: read n w h <<< "$sc"
      run "$v $n $w" env RTC_LIBRARY=$L/$lib/librtc.so $e python bench.py --scene $n --width $w --height $h --steps 400 --warmup 20 --no-cpu-baseline || exit 1
    done
  done
done
