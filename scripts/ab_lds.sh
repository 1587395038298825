#!/bin/bash
# A/B: world tables staged in LDS (default) vs global gathers, across scenes.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out; rm -f gpurun_out/ab.log
source scripts/ab_lib.sh
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline"
for sc in three_sphere_scene reflect_refract cover table shadow_puppets cylinders metal refraction; do
  for l in 1 0; do
    run "lds=$l $sc f32" env RTC_DEBUG=lds_world=$l $B --scene $sc
  done
done
run "lds=1 three_sphere f64" $B --precision f64
