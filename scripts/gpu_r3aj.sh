#!/bin/bash
# Line cull in the per-scene refractive-index walk: bit-identity tests, A/B vs HEAD (_lib_base), 8-shard times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_identity.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/walkcull_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/walkcull_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do AB_STEPS=200 bash scripts/ab_builds.sh "base default" "reflect_refract refraction cylinders table" || exit 1; done
for r in 1 2; do AB_STEPS=100 bash scripts/ab_builds.sh "base default" "cover" || exit 1; done
for v in base default; do
  for sc in "cover 3840 2160 1,8" "table 3840 2160 1,8"; do
    set -- $sc
    echo "$v :: $(RTC_LIBRARY=$PWD/ray-tracer-challenge-rs_amd/rtc_amd/_lib$([ $v = base ] && echo _base)/librtc.so SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' | tr '\n' ' ')"
  done
done
