#!/bin/bash
# (historical: RTC_COLD_PRIO was measured, rejected and removed from the tree)
# Cold launches: the first centre-out tiles at priority 2 (RTC_COLD_PRIO = fraction of the grid); new JIT tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export RTC_JIT_CACHE=0
timeout -k 10 200 python -u -m pytest tests/test_gpu_jit.py -k "all_kinds or complex" -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/jit_kinds.log 2>&1
rc=$?; echo "jit kinds tests rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/jit_kinds.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 env RTC_COLD_PRIO=0.5 python -u -m pytest tests/test_gpu_parity.py -k "split_tiles or cost_ordered or moved_camera or consecutive" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/coldprio_test.log 2>&1
rc=$?; echo "cold prio tests rc=$rc"; tail -1 gpurun_out/coldprio_test.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=40 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "X=0" "RTC_COLD_PRIO=0.25" "RTC_COLD_PRIO=0.5" "RTC_COLD_PRIO=1" "RTC_COLD_PRIO=2"
