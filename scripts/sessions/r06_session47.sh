set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do for f in 2 3; do
  timeout -k 10 120 python bench.py --steps 1000 --mode frames --ab --no-cpu-baseline --inflight $f > gpurun_out/r06_if47.log 2>&1 || { tail -3 gpurun_out/r06_if47.log; exit 1; }
  grep '^{' gpurun_out/r06_if47.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('frames1000 inflight', $f, 'round', $r, round(d['value']/1e3,1), round(d['ms_per_step']*1e3,2))"
  timeout -k 10 200 python bench.py --mode tiled --steps 20 --warmup 5 --no-cpu-baseline --ab --inflight $f > gpurun_out/r06_if47t.log 2>&1 || { tail -3 gpurun_out/r06_if47t.log; exit 1; }
  grep '^{' gpurun_out/r06_if47t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tiled20 inflight', $f, 'round', $r, round(d['value']/1e3,1), round(d['ms_per_step'],4))"
done; done
for f in 2 3; do SHARD_INFLIGHT=$f SHARD_COUNTS=8 timeout -k 10 180 python scripts/shard_times.py cover 3840 2160 2>/dev/null | grep inflight; done
