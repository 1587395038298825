set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/region_probe.py 15 > gpurun_out/r06_region_probe.jsonl 2> gpurun_out/r06_region_probe.err; echo "region rc=$?"; cat gpurun_out/r06_region_probe.jsonl
timeout -k 10 300 python scripts/shard_concurrency.py cover table > gpurun_out/r06_shard_conc.jsonl 2> gpurun_out/r06_shard_conc.err; echo "conc rc=$?"; cat gpurun_out/r06_shard_conc.jsonl
for e in "split=0" "urgent=0" "tile_order=0"; do echo "== $e"; RTC_DEBUG=$e SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 || exit 1; done > gpurun_out/r06_shard_knobs.txt 2>&1; echo "knobs rc=$?"; cat gpurun_out/r06_shard_knobs.txt
