set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3 4; do for v in "4 3" "8 3" "8 4" "8 6"; do
  set -- $v
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline --inflight $2 > gpurun_out/r06_if50.log 2>&1 || { tail -3 gpurun_out/r06_if50.log; exit 1; }
  grep '^{' gpurun_out/r06_if50.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('hwq', $1, 'inflight', $2, 'round', $r, round(d['value']/1e3,1), round(d['ms_per_step']*1e3,2))"
done; done
