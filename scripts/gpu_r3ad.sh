#!/bin/bash
# Per-scene builds with only the world's pattern kinds and no refraction code without glass: tests, A/B vs HEAD (_lib_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_parity.py tests/test_gpu_identity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/jit_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/jit_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do AB_STEPS=200 bash scripts/ab_builds.sh "base default" "reflect_refract refraction metal cylinders" || exit 1; done
for r in 1 2; do AB_STEPS=100 bash scripts/ab_builds.sh "base default" "cover table" || exit 1; done
AB_STEPS=1000 bash scripts/ab_builds.sh "base default" "three_sphere_scene" || exit 1
