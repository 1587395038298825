set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in "-" "split=1.5" "split=2" "split=3" "split=4" "split=2,urgent=0" "split=2,split_max=2"; do echo "== $e"; for sc in cover table; do RTC_DEBUG=${e/#-/} SHARD_INFLIGHT=2 SHARD_COUNTS=8 timeout -k 10 200 python scripts/shard_times.py $sc 3840 2160 || exit 1; done; done 2>&1 | grep -v amdgpu.ids
