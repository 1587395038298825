set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_bench_contract.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_t21.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -cE "PASSED" gpurun_out/r06_t21.log; grep -E "FAILED" gpurun_out/r06_t21.log | head; [ $rc -le 1 ] || exit $rc
for a in "--steps 1000" "--scene reflect_refract --steps 300" "--steps 20 --warmup 5"; do timeout -k 10 240 python bench.py $a --mode frames --ab --no-cpu-baseline > gpurun_out/r06_b21.log 2>&1 || exit 1; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_b21.log') if l.startswith('{')][-1]; print('$a', round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'])"; done
