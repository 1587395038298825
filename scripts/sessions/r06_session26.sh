set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t26.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t26.log; grep -E "FAILED|Error" gpurun_out/r06_t26.log | head; tail -2 gpurun_out/r06_t26.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke26.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r06_smoke26.log; exit $rc
