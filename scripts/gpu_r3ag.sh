#!/bin/bash
# Direct per-scene kernel after the round-3 specialisations: fence spacing (RTC_JIT_FENCE_EVERY) and grid size
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
AB_STEPS=1000 bash scripts/ab_env.sh "three_sphere_scene shadow_puppets" "X=0" \
  "RTC_JIT_FLAGS=-URTC_JIT_FENCE_EVERY,-DRTC_JIT_FENCE_EVERY=1" "RTC_JIT_FLAGS=-URTC_JIT_FENCE_EVERY,-DRTC_JIT_FENCE_EVERY=2" \
  "RTC_JIT_FLAGS=-URTC_JIT_FENCE_EVERY,-DRTC_JIT_FENCE_EVERY=6" "RTC_JIT_FLAGS=-URTC_JIT_FENCE_EVERY,-DRTC_JIT_FENCE_EVERY=100" \
  "RTC_DIRECT_GRID=4096" "RTC_DIRECT_GRID=6144" "RTC_DIRECT_GRID=8160"
