set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "per_scene or color_at" > gpurun_out/r06_t31.log 2>&1; rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|SKIPPED" gpurun_out/r06_t31.log | sed 's/.*:://' | head -20; grep -E "^E " gpurun_out/r06_t31.log | head -20; tail -2 gpurun_out/r06_t31.log; exit $rc
