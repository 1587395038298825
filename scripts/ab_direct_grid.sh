#!/bin/bash
# Direct-kernel grid: the default (2.5x resident) against the resident grid
# (RTC_DIRECT_GRID=2048 = 8 workgroups/CU x 256 CUs) at 1080p, 4K and f64.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
B="python bench.py --no-cpu-baseline --warmup 30"
for g in 0 2048; do
  run "grid=$g 1080p" env RTC_DIRECT_GRID=$g $B --steps 1000
  run "grid=$g 4K" env RTC_DIRECT_GRID=$g $B --steps 300 --width 3840 --height 2160
  run "grid=$g 1080p f64" env RTC_DIRECT_GRID=$g $B --steps 300 --precision f64
  run "grid=$g shadow_puppets" env RTC_DIRECT_GRID=$g $B --steps 1000 --scene shadow_puppets
done
