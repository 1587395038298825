#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/parity_report.py > gpurun_out/parity.log 2>&1; rc=$?
echo "parity rc=$rc"; tail -40 gpurun_out/parity.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
exit $rc
