#!/bin/bash
# A/B matrix of short bench runs: each line = env + bench args; prints value/kernel_ms.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
run() {  # $1 = label, rest = command
  local label=$1; shift
  local line
  line=$(timeout -k 10 120 "$@" 2>/dev/null | grep '^{')
  local rc=$?
  echo "$label :: $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("value=%.0f Mray/s kernel_ms=%.4f frac=%.4f rays/frame=%d" % (d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], d["config"]["rays_per_frame"]))' 2>&1)" | tee -a gpurun_out/ab.log
}
B="python bench.py --steps 60 --warmup 10 --no-cpu-baseline"
for sched in persistent grid; do
  for scene in three_sphere_scene reflect_refract table cover; do
    run "$sched $scene f32" env RTC_SCHED_DIRECT=$sched RTC_SCHED_POOL=$sched $B --scene $scene
  done
  run "$sched three_sphere f64" env RTC_SCHED_DIRECT=$sched RTC_SCHED_POOL=$sched $B --precision f64
  run "$sched reflect_refract f64" env RTC_SCHED_DIRECT=$sched RTC_SCHED_POOL=$sched $B --precision f64 --scene reflect_refract
done
