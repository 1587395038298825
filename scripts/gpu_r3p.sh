#!/bin/bash
# 16-part split (RTC_SPLIT_MAX=4): exactness test, then slowest-of-N shard sweep under wave priority
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RTC_JIT_CACHE=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/split16_test.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -3 gpurun_out/split16_test.log
[ $rc -eq 0 ] || exit $rc
for envs in "RTC_SPLIT_MAX=2" "RTC_SPLIT_MAX=3" "RTC_SPLIT_MAX=4" "RTC_SPLIT_MAX=4 RTC_SPLIT=0.5" "RTC_SPLIT_MAX=4 RTC_SPLIT=2"; do
  for sc in "cover 3840 2160 1,8" "table 3840 2160 1,8" "reflect_refract 1920 1080 1,4"; do
    set -- $sc
    echo "$envs"; env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
