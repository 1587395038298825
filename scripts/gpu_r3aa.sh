#!/bin/bash
# Per-scene builds render frames only (no color_at branch): JIT bit-identity tests, then A/B vs HEAD build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/jit_test.log 2>&1
rc=$?; echo "jit tests rc=$rc"; tail -2 gpurun_out/jit_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do AB_STEPS=1000 bash scripts/ab_builds.sh "base default" "three_sphere_scene shadow_puppets" || exit 1; done
for r in 1 2; do AB_STEPS=200 bash scripts/ab_builds.sh "base default" "reflect_refract refraction" || exit 1; done
