set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -q -rs --timeout 120 --timeout-method thread -p no:cacheprovider -k per_scene > gpurun_out/r06_t45.log 2>&1; rc=$?; echo "rc=$rc"; tail -2 gpurun_out/r06_t45.log; exit $rc
