set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3 4 5 6 7 8; do for f in 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline --inflight $f > gpurun_out/r06_if46.log 2>&1 || { tail -3 gpurun_out/r06_if46.log; exit 1; }
  grep '^{' gpurun_out/r06_if46.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflight', $f, 'round', $r, round(d['value']/1e3,1), round(d['ms_per_step']*1e3,2), round(d['frame_latency_ms']*1e3,2))"
done; done
