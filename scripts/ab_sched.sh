#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline"
for s in grid static dynamic; do
  run "direct=$s three_sphere f32" env RTC_SCHED_DIRECT=$s $B
  run "direct=$s three_sphere f32 nocount" env RTC_SCHED_DIRECT=$s $B --flags 1
  run "direct=$s three_sphere f32 notrace" env RTC_SCHED_DIRECT=$s $B --flags 5
done
for s in dynamic static grid; do
  run "pool=$s reflect_refract f32" env RTC_SCHED_POOL=$s $B --scene reflect_refract
  run "pool=$s cover f32" env RTC_SCHED_POOL=$s $B --scene cover
done
