set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do for v in smi nosmi; do
  if [ $v = nosmi ]; then export BENCH_NO_SMI=1; else unset BENCH_NO_SMI; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline > gpurun_out/r06_smi2_$v.log 2>&1 || exit 1
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_smi2_$v.log') if l.startswith('{')][-1]; print('$v', round(d['value']/1e3,1), d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done
unset BENCH_NO_SMI
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_default.log 2>&1; echo "default rc=$?"
python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_bench_default.log') if l.startswith('{')][-1]; print(round(d['value']/1e3,1), d['ms_per_step'], d['roofline']['kernel_ms'], d['device_state']['before'].get('sclk_mhz'), {k:(v['ms_per_step'],v['render_ms_per_shard']) for k,v in d['tile_split'].items()})"
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
RTC_DEBUG=refill=256 timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_refill.log 2>&1; rc=$?; echo "tests refill rc=$rc"; tail -15 gpurun_out/pytest_gpu_refill.log; [ $rc -le 1 ] || exit $rc
ROUNDS=2 bash scripts/ab_knobs.sh "base=" "r256=refill=256" "r128=refill=128" > gpurun_out/r06_ab_refill.jsonl 2>&1; echo "ab rc=$?"; cat gpurun_out/r06_ab_refill.jsonl
for e in "refill=0" "refill=256" "refill=128" "refill=256,split_max=4"; do echo "== $e"; RTC_DEBUG=$e SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 || exit 1; RTC_DEBUG=$e SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py table 3840 2160 || exit 1; done 2>&1 | grep -v amdgpu.ids
