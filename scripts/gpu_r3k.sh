#!/bin/bash
# with urgent priority on: pool waves/SIMD 7 / 6 / 5 and split knobs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source scripts/ab_lib.sh
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
for v in _lib _lib_w7 _lib_w5; do
  for sc in cover table; do
    echo "$v"; RTC_LIBRARY=$L/$v/librtc.so SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for e in "RTC_SPLIT=0.75" "RTC_SPLIT_MAX=3" "RTC_SPLIT=0.75 RTC_SPLIT_MAX=3"; do
  for sc in cover table; do
    echo "$e"; env $e SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for r in 1 2; do
  for v in _lib _lib_w7 _lib_w5; do
    for sc in reflect_refract:1920:1080 refraction:1920:1080 cylinders:1920:1080 cover:3840:2160 table:3840:2160; do
      IFS=: read n w h <<< "$sc"
      run "$v $n" env RTC_LIBRARY=$L/$v/librtc.so python bench.py --scene $n --width $w --height $h --steps 200 --warmup 10 --no-cpu-baseline || exit 1
    done
  done
done
