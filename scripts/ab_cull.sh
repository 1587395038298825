#!/bin/bash
# A/B: wave-cull coverage threshold (negative = off, huge = cull every bounded shape).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline"
for sc in three_sphere_scene reflect_refract cover table shadow_puppets cylinders metal refraction; do
  for c in -1 0.1 0.25 0.6 1e9; do
    run "cull<=$c $sc f32" env RTC_CULL_COVERAGE=$c $B --scene $sc
  done
done
