set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v -rs --durations=5 --timeout 300 --timeout-method thread -p no:cacheprovider -k many_shapes > gpurun_out/r06_t33.log 2>&1; rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|SKIPPED|^E |slowest|s call" gpurun_out/r06_t33.log | head -30; tail -2 gpurun_out/r06_t33.log; exit $rc
