set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t28.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "^seed|PASSED|FAILED|assert" gpurun_out/r06_t28.log | head -80; exit $rc
