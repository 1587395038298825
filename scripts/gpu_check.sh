#!/bin/bash
# One gpurun session: GPU parity tests, smoke, a short bench.  Each GPU step
# has its own time limit; a crash/timeout (rc not 0/1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"-q"}
timeout -k 10 ${PYTEST_TIMEOUT:-480} python -m pytest tests -m gpu $PYTEST_ARGS -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python bench.py --steps ${BENCH_STEPS:-100} --warmup 10 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 && timeout -k 10 120 python bench.py --precision f64 --no-cpu-baseline --steps 50 --warmup 5 >> gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
