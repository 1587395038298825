#!/bin/bash
# N = 2 rehearsal of the bench's frames line on one GPU (BENCH_SHARE_GPU=1; the tiled split needs one GPU per rank)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --mode frames --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/n2_frames.log 2>&1
rc=$?; echo "n2 rc=$rc"; grep '^{' gpurun_out/n2_frames.log | cut -c1-500; tail -3 gpurun_out/n2_frames.log
exit $rc
