#!/bin/bash
# (historical: RTC_PRIO_CAP and RTC_OVERLAP was measured, rejected and removed from the tree)
# (1) priority cap by queue position (RTC_PRIO_CAP) on shards; (2) overlapped-items pool kernel (_lib_ov): tests, shards, frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
timeout -k 10 200 env RTC_PRIO_CAP=0.167,0.5,1 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cap_test.log 2>&1
rc=$?; echo "cap tests rc=$rc"; tail -2 gpurun_out/cap_test.log; [ $rc -eq 0 ] || exit $rc
for envs in "X=0" "RTC_PRIO_CAP=0.167,0.5,1" "RTC_PRIO_CAP=0.083,0.25,0.5" "RTC_PRIO_CAP=0.333,0.667,1"; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8" "reflect_refract 1920 1080 4"; do
    set -- $sc
    echo "$envs $(env $envs SHARD_COUNTS=$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/')" || exit 1
  done
done
RTC_LIBRARY=$L/_lib_ov/librtc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ov_tests.log 2>&1
rc=$?; echo "ov tests rc=$rc"; tail -3 gpurun_out/ov_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in _lib _lib_ov; do
  for sc in "cover 3840 2160 8" "table 3840 2160 8" "reflect_refract 1920 1080 4"; do
    set -- $sc
    echo "$v $(RTC_LIBRARY=$L/$v/librtc.so SHARD_COUNTS=1,$4 timeout -k 10 120 python scripts/shard_times.py $1 $2 $3 2>&1 | grep -v amdgpu.ids | sed 's/per-shard ms .*max/max/' | tr '\n' ' ')" || exit 1
  done
done
