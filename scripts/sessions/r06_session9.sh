set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
RTC_DEBUG=refill=256 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_refill.log 2>&1; rc=$?; echo "tests refill rc=$rc"; tail -8 gpurun_out/pytest_gpu_refill.log; [ $rc -le 1 ] || exit $rc
ROUNDS=2 bash scripts/ab_knobs.sh "base=" "r256=refill=256" "r128=refill=128" > gpurun_out/r06_ab_refill.jsonl 2>&1; echo "ab rc=$?"; cat gpurun_out/r06_ab_refill.jsonl
for e in "refill=0" "refill=256" "refill=128" "refill=256,split_max=4"; do echo "== $e"; RTC_DEBUG=$e SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 || exit 1; RTC_DEBUG=$e SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py table 3840 2160 || exit 1; done > gpurun_out/r06_refill_shards.txt 2>&1; echo "shards rc=$?"; grep -v amdgpu.ids gpurun_out/r06_refill_shards.txt
