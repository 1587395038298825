#!/bin/bash
# World tables from global memory instead of LDS (per-scene kernels), direct and pool scenes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
AB_STEPS=1000 bash scripts/ab_env.sh "three_sphere_scene shadow_puppets three_sphere_scene:3840x2160" "X=0" "RTC_LDS_WORLD=0" || exit 1
AB_STEPS=200 bash scripts/ab_env.sh "reflect_refract metal" "X=0" "RTC_LDS_WORLD=0" || exit 1
