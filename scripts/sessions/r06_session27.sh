set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --mode frames --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r06_n2_shared.log 2>&1; rc=$?; echo "n2 rc=$rc"; grep '^{' gpurun_out/r06_n2_shared.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r06_n2_shared.log; exit $rc; }
