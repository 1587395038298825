#!/bin/bash
# Per-scene kernels without diagnostics: direct (default build) and pool (_lib_pd), A/B vs HEAD (_lib_base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_kats.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/jit_test.log 2>&1
rc=$?; echo "jit+kat tests rc=$rc"; tail -2 gpurun_out/jit_test.log; [ $rc -eq 0 ] || exit $rc
RTC_LIBRARY=$PWD/ray-tracer-challenge-rs_amd/rtc_amd/_lib_pd/librtc.so timeout -k 10 200 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/jit_test_pd.log 2>&1
rc=$?; echo "pd jit tests rc=$rc"; tail -2 gpurun_out/jit_test_pd.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do AB_STEPS=1000 bash scripts/ab_builds.sh "base default" "three_sphere_scene shadow_puppets" || exit 1; done
for r in 1 2; do AB_STEPS=200 bash scripts/ab_builds.sh "base default pd" "reflect_refract refraction metal" || exit 1; done
