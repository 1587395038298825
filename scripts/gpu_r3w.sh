#!/bin/bash
# (historical: RTC_PRIO_CAP was measured, rejected and removed from the tree)
# Priority cap by queue position (RTC_PRIO_CAP=f3,f2,f1): shards and whole frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 env RTC_PRIO_CAP=0.167,0.5,1 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cap_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/cap_test.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for envs in "X=0" "RTC_PRIO_CAP=0.167,0.5,1" "RTC_PRIO_CAP=0.167,0.333,0.667" "RTC_PRIO_CAP=0.083,0.25,0.5" "RTC_PRIO_CAP=0.333,0.667,1"; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8" "reflect_refract 1920 1080 4"; do
    set -- $sc
    echo "$envs"; env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' || exit 1
  done
done
done
AB_STEPS=100 bash scripts/ab_env.sh "reflect_refract refraction cylinders cover:3840x2160 table:3840x2160" "X=0" "RTC_PRIO_CAP=0.167,0.5,1" "RTC_PRIO_CAP=0.083,0.25,0.5"
