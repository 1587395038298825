#!/bin/bash
# round-3 kernel-trace stats at steady clocks (the PMC passes of gpu_r3prof.sh stand)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
declare -A ARGS=([three_sphere]="" [reflect_refract]="--scene reflect_refract"
                 [cover]="--scene cover --width 3840 --height 2160" [table]="--scene table --width 3840 --height 2160")
for k in three_sphere reflect_refract cover table; do
  PROF_NAME=r03_stats_$k BENCH_ARGS="${ARGS[$k]}" bash scripts/gpu_prof.sh || exit $?
done
