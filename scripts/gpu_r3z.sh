#!/bin/bash
# Direct kernel: grid-size sweep on the per-scene build (RTC_DIRECT_GRID) + stamps of the generic kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
for a in "--scene three_sphere_scene" "--scene three_sphere_scene --width 3840 --height 2160"; do
  STAMPS_DETAIL=1 timeout -k 10 60 python scripts/stamps.py $a 2>/dev/null | grep '^{' || exit 1
done
AB_STEPS=1000 bash scripts/ab_env.sh "three_sphere_scene shadow_puppets" "X=0" "RTC_DIRECT_GRID=2048" "RTC_DIRECT_GRID=4096" "RTC_DIRECT_GRID=6144" "RTC_DIRECT_GRID=8160" "RTC_SCHED_DIRECT=grid" || exit 1
