set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bench_contract.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t39.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r06_t39.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3 4; do for b in bench_old.py bench.py; do
  timeout -k 10 120 python $b --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline > gpurun_out/r06_ab39.log 2>&1 || { tail -3 gpurun_out/r06_ab39.log; exit 1; }
  grep '^{' gpurun_out/r06_ab39.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b', $r, round(d['value']/1e3,1), round(d['ms_per_step']*1e3,2), round(d['frame_latency_ms']*1e3,2))"
done; done
