#!/bin/bash
# round 3: GPU tests + smoke + bench, then the 8-shard diagnostics of cover/table 4K
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS="-v --timeout 120 --timeout-method thread" bash scripts/gpu_check.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 > gpurun_out/shards_cover.log 2>&1 || exit $?
timeout -k 10 200 python scripts/shard_times.py table 3840 2160 > gpurun_out/shards_table.log 2>&1 || exit $?
for s in 0 3 7; do timeout -k 10 100 python scripts/stamps.py --scene cover --width 3840 --height 2160 --out u8 --shard $s/8 >> gpurun_out/stamps_cover.log 2>&1 || exit $?; done
cat gpurun_out/shards_cover.log gpurun_out/shards_table.log gpurun_out/stamps_cover.log | grep -v amdgpu.ids
