#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
source scripts/ab_lib.sh
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline"
for sched in persistent grid; do
  for fl in 0 1 2 3 4 5; do
    run "$sched three_sphere flags=$fl" env RTC_DEBUG=sched_direct=$sched $B --flags $fl
  done
done
