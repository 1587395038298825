set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bench_contract.py tests/test_gpu_streams.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_bench_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error" gpurun_out/r06_bench_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_default.log 2>&1; echo "default rc=$?"
python - <<'PY'
import json
d=[json.loads(l) for l in open('gpurun_out/r06_bench_default.log') if l.startswith('{')][-1]
print(round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'], d['device_state']['before'].get('sclk_mhz'))
for k,v in d['tile_split'].items(): print(k, v['ms_per_step'], v['speedup_vs_1gpu'], v.get('shards_of_8_on_one_gpu',{}).get('slowest_ms'))
PY
for r in 1 2; do for f in 1 2 3; do timeout -k 10 240 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline --inflight $f > gpurun_out/r06_inflight_$f.log 2>&1 || exit 1; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_inflight_$f.log') if l.startswith('{')][-1]; print('inflight $f', round(d['value']/1e3,1), d['ms_per_step'], d['frame_latency_ms'])"; done; done
