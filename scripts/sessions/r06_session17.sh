set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_bench_contract.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t17.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t17.log; grep -E "FAILED" gpurun_out/r06_t17.log | head; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for f in 1 2 3; do timeout -k 10 240 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline --inflight $f > gpurun_out/r06_if_$f.log 2>&1 || exit 1; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_if_$f.log') if l.startswith('{')][-1]; print('inflight $f', round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'])"; done; done
for f in 1 2; do timeout -k 10 240 python bench.py --steps 1000 --mode frames --ab --no-cpu-baseline --inflight $f > gpurun_out/r06_if1000_$f.log 2>&1 || exit 1; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_if1000_$f.log') if l.startswith('{')][-1]; print('1000 steps inflight $f', round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'])"; done
