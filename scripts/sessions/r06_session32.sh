set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v -rs --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t32.log 2>&1; rc=$?; echo "rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t32.log; grep -E "FAILED|SKIPPED" gpurun_out/r06_t32.log | head -20; grep -E "^E " gpurun_out/r06_t32.log | head -10; tail -2 gpurun_out/r06_t32.log; exit $rc
