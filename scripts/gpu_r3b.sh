#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -ne 0 ] && exit $rc
RTC_JIT_CACHE=0 timeout -k 5 60 python scripts/exit_probe.py inflight || exit $?
timeout -k 10 200 python scripts/shard_costs.py cover > gpurun_out/shard_costs.log 2>&1 || exit $?
timeout -k 10 200 python scripts/shard_costs.py table >> gpurun_out/shard_costs.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/shard_costs.log
