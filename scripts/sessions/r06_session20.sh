set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_knobs.sh "hint=" "s10=split=1" > gpurun_out/r06_ab_split_whole.jsonl 2>&1; echo "rc=$?"; cat gpurun_out/r06_ab_split_whole.jsonl
SHARD_INFLIGHT=2 SHARD_COUNTS=8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 2>&1 | grep -v amdgpu.ids
SHARD_INFLIGHT=2 SHARD_COUNTS=8 timeout -k 10 200 python scripts/shard_times.py table 3840 2160 2>&1 | grep -v amdgpu.ids
