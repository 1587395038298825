set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do for v in smi nosmi; do
  if [ $v = nosmi ]; then export BENCH_NO_SMI=1; else unset BENCH_NO_SMI; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --mode frames --ab --no-cpu-baseline > gpurun_out/r06_smi_$v.log 2>&1 || exit 1
  python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r06_smi_$v.log') if l.startswith('{')][-1]; print('$v', round(d['value']/1e3,1), d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done
unset BENCH_NO_SMI
for e in "split_max=4" "split_max=5" "split=0.5" "split=2"; do echo "== $e"; RTC_DEBUG=$e SHARD_COUNTS=8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 || exit 1; RTC_DEBUG=$e SHARD_COUNTS=8 timeout -k 10 200 python scripts/shard_times.py table 3840 2160 || exit 1; done > gpurun_out/r06_shard_knobs2.txt 2>&1; echo "knobs rc=$?"; grep -v amdgpu.ids gpurun_out/r06_shard_knobs2.txt
SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 | grep -v amdgpu.ids; SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py table 3840 2160 | grep -v amdgpu.ids
