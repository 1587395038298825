set -u
mkdir -p gpurun_out
export TMPDIR=/tmp ROUND=r06
timeout -k 10 400 python -u -m pytest tests/test_bench_contract.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t25.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t25.log; grep -E "FAILED" gpurun_out/r06_t25.log | head; [ $rc -le 1 ] || exit $rc
bash scripts/round_bench.sh > gpurun_out/r06_bench.log 2>&1 || { echo "bench lines failed"; tail -5 gpurun_out/r06_bench.log; exit 1; }
echo "bench lines ok"
