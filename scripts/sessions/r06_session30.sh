set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_worlds.py -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t30.log 2>&1; rc=$?; echo "random rc=$rc"; grep -c PASSED gpurun_out/r06_t30.log; grep -E "FAILED|assert" gpurun_out/r06_t30.log | head -20; grep -o "seed [0-9]* depth.*" gpurun_out/r06_t30.log | sort -t' ' -k11 | head -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t30b.log 2>&1; rc2=$?; echo "suite rc=$rc2"; tail -3 gpurun_out/r06_t30b.log; exit $((rc + rc2))
