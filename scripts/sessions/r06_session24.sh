set -u
mkdir -p gpurun_out
export TMPDIR=/tmp ROUND=r06
bash scripts/round_bench.sh > gpurun_out/r06_bench.log 2>&1 || { echo "bench lines failed"; tail -5 gpurun_out/r06_bench.log; exit 1; }
echo "bench lines ok"
{ SHARD_INFLIGHT=2 SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py cover 3840 2160 &&
  SHARD_INFLIGHT=2 SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py table 3840 2160; } > gpurun_out/r06_shard_times.txt 2>&1 || { echo "shard times failed"; exit 1; }
cat gpurun_out/r06_shard_times.txt
