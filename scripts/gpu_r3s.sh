#!/bin/bash
# Scheduler strategies for the per-scene builds (RTC_JIT_FLAGS), kernel ms, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
AB_STEPS=300 bash scripts/ab_env.sh "three_sphere_scene shadow_puppets reflect_refract cover:3840x2160" "X=0" \
  "RTC_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=max-ilp" "RTC_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=iterative-ilp" \
  "RTC_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=iterative-minreg" "RTC_JIT_FLAGS=-mllvm,-amdgpu-sched-strategy=max-memory-clause" \
  "RTC_JIT_FLAGS=-mllvm,-amdgpu-use-amdgpu-trackers=1"
