cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 300 --cpu-seconds 3 2>/dev/null | grep '^{' || exit 1
timeout -k 10 200 python bench.py --scene cover --width 3840 --height 2160 --steps 50 --no-cpu-baseline 2>/dev/null | grep '^{' || exit 1
BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 200 --warmup 10 > gpurun_out/dist2.log 2>&1; rc=$?; grep '^{' gpurun_out/dist2.log; tail -5 gpurun_out/dist2.log; exit $rc
