#!/bin/bash
# Walk cull gated on >= 4 bounded shapes: tests, A/B vs HEAD (_lib_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_identity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/walkcull_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/walkcull_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do AB_STEPS=200 bash scripts/ab_builds.sh "base default" "reflect_refract refraction cylinders cover" || exit 1; done
