#!/bin/bash
# Item-level timeline of shards (RT_FLAG_STAMPS item log) + bench A/B of the build with the log compiled in
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
for a in "cover 3840 2160 8 0,4" "table 3840 2160 8 0" "reflect_refract 1920 1080 4 0" "cover 3840 2160 1 0"; do
  timeout -k 10 120 python scripts/shard_tail.py $a 2>&1 | grep -v amdgpu.ids || exit 1
done
AB_STEPS=300 bash scripts/ab_env.sh "three_sphere_scene reflect_refract cover:3840x2160" "X=0"
