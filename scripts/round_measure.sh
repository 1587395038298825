#!/bin/bash
# One GPU call for a round's measurements: the profile set
# (scripts/profile_round.sh) reduced on the box by scripts/collect_profiles.py
# into gpurun_out/$ROUND_collected/ (the raw traces exceed what gpurun copies
# back, so they are deleted there), the bench lines (scripts/round_bench.sh)
# and the 8-way shard times of cover and table at 4K (scripts/shard_times.py).
# Afterwards, here: cp gpurun_out/$ROUND_collected/* profiles/
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
export ROUND=${ROUND:-r05}
# (the profiled runs take one frame in flight: rocprof's per-kernel durations
# are then one launch's, as the lines' roofline.kernel_ms = frame_latency_ms)
bash scripts/profile_round.sh > gpurun_out/${ROUND}_profset.log 2>&1 || { echo "profile set failed"; tail -5 gpurun_out/${ROUND}_profset.log; exit 1; }
python scripts/collect_profiles.py $ROUND gpurun_out/${ROUND}_collected > gpurun_out/${ROUND}_collect.log 2>&1 || { echo "collect failed"; exit 1; }
rm -rf gpurun_out/${ROUND}_stats_* gpurun_out/${ROUND}_pmc_*
echo "profile set ok"
[ "${PROFILES_ONLY:-0}" = 1 ] && { du -sh gpurun_out; echo "all ok"; exit 0; }
bash scripts/round_bench.sh > gpurun_out/${ROUND}_bench.log 2>&1 || { echo "bench lines failed"; exit 1; }
echo "bench lines ok"
{ SHARD_INFLIGHT=2 SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py cover 3840 2160 &&
  SHARD_INFLIGHT=2 SHARD_COUNTS=1,8 timeout -k 10 180 python scripts/shard_times.py table 3840 2160; } > gpurun_out/${ROUND}_shard_times.txt 2>&1 || { echo "shard times failed"; exit 1; }
du -sh gpurun_out
echo "all ok"
