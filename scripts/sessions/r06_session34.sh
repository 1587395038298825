set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "parity" > gpurun_out/r06_t34.log 2>&1; rc=$?; echo "rc=$rc"; grep -c PASSED gpurun_out/r06_t34.log; grep -E "FAILED|^E " gpurun_out/r06_t34.log | head; grep -o "seed [0-9]* depth.*" gpurun_out/r06_t34.log | tail -8; exit $rc
