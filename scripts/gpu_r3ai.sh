#!/bin/bash
# Time attribution on the specialised build: without the containers walk / without shadow rays (diagnostic variants)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
AB_STEPS=200 bash scripts/ab_builds.sh "default nowalk noshadow" "reflect_refract refraction cover table cylinders" || exit 1
AB_STEPS=1000 bash scripts/ab_builds.sh "default noshadow" "three_sphere_scene" || exit 1
