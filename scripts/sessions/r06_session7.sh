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
