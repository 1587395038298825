set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bench_contract.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t48.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r06_t48.log; [ $rc -eq 0 ] || exit $rc
bash scripts/sessions/r06_session40.sh
