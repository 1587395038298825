#!/bin/bash
# Round-end GPU check (one call): pytest -m gpu, __graft_entry__.smoke(), and the bench with
# the driver's own flags (--steps 20 --warmup 5); logs under gpurun_out/final_*.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/final_gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_driver_flags.log 2>&1 || exit 1
grep '^{' gpurun_out/final_bench_driver_flags.log | cut -c1-400
