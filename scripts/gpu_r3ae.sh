#!/bin/bash
# (historical: RTC_SPLIT_STICKY was measured, rejected and removed from the tree)
# Sticky splits (RTC_SPLIT_STICKY) and order-build count on shards and whole frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 env RTC_SPLIT_STICKY=1 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered or moved_camera" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sticky_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sticky_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for envs in "X=0" "RTC_SPLIT_STICKY=1" "RTC_ORDER_BUILDS=4" "RTC_ORDER_BUILDS=16" "RTC_SPLIT_STICKY=1 RTC_ORDER_BUILDS=16"; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8" "reflect_refract 1920 1080 4"; do
    set -- $sc
    echo "$envs :: $(env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/')"
  done
done
done
AB_STEPS=200 bash scripts/ab_env.sh "reflect_refract cover:3840x2160 table:3840x2160" "X=0" "RTC_SPLIT_STICKY=1"
