#!/bin/bash
# (1) split-threshold sweep of the 8-shard frames
# (2) A/B: AoS spill records (worktree, _lib) against HEAD (_lib_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source scripts/ab_lib.sh
for sp in 1.5 1.0 0.75; do
  for sc in cover table; do
    echo "RTC_SPLIT=$sp"; RTC_SPLIT=$sp SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
for r in 1 2; do
  for v in _lib _lib_base; do
    for sc in reflect_refract:1920:1080 refraction:1920:1080 cover:3840:2160 table:3840:2160; do
      IFS=: read n w h <<< "$sc"
      run "$v $n" env RTC_LIBRARY=$L/$v/librtc.so python bench.py --scene $n --width $w --height $h --steps 300 --warmup 20 --no-cpu-baseline || exit 1
    done
  done
done
