#!/bin/bash
# (historical: RTC_AGE_PRIO was measured, rejected and removed from the tree)
# Age-based wave priority (RTC_AGE_PRIO=g1,g2,g3): warm and cold kernel ms, 2 rounds; 8-shard cover/table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered or moved_camera" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/age_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/age_test.log; [ $rc -eq 0 ] || exit $rc
RTC_AGE_PRIO=4,8,16 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/age_test2.log 2>&1
rc=$?; echo "tests(age) rc=$rc"; tail -2 gpurun_out/age_test2.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=100 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "X=0" \
  "RTC_AGE_PRIO=4,8,16" "RTC_AGE_PRIO=8,16,32" "RTC_AGE_PRIO=16,32,64" "RTC_AGE_PRIO=2,4,8" || exit 1
for envs in "X=0" "RTC_AGE_PRIO=4,8,16" "RTC_AGE_PRIO=8,16,32"; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8"; do
    set -- $sc
    echo "$envs"; env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' || exit 1
  done
done
