set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench40.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r06_bench40.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print(round(d['value']/1e3,1), round(d['ms_per_step']*1e3,2), round(d['frame_latency_ms']*1e3,2), round(d['roofline']['frac'],3), d['frames_in_flight'])
for k,v in d['tile_split'].items(): print(k, round(v['value']/1e3,1), round(v['ms_per_step'],4), round(v['render_ms_per_shard'],4), v['shards_of_8_on_one_gpu']['slowest_ms'], v['roofline'].get('wait_frac'))
print('cpu', d['cpu_baseline']['value'], 'one_shot', d['one_shot']['total_ms'])"; exit $rc
