set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "accelerations" > gpurun_out/r06_t36.log 2>&1; rc=$?; echo "rc=$rc"; grep -c PASSED gpurun_out/r06_t36.log; grep -E "FAILED|^E " gpurun_out/r06_t36.log | head -20; tail -1 gpurun_out/r06_t36.log; exit $rc
