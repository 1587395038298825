#!/bin/bash
# A/B of two source trees on one GPU box: this tree against an older build
# checked out (git worktree) and built under $OLD (default ab_old/), each
# running its own bench.py.  Alternates A, B per scene ROUNDS times; prints
# the kernel ms of every run.  Usage: ab_trees.sh "<scene[:WxH]> ..." [rounds]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OLD=${OLD:-$R/ab_old}
cd $R; mkdir -p gpurun_out
SCENES=${1:-three_sphere_scene}
ROUNDS=${2:-3}
STEPS=${AB_STEPS:-400}
for sc in $SCENES; do
  name=${sc%%:*}; size=${sc#*:}; [ "$size" = "$sc" ] && size=1920x1080
  w=${size%x*}; h=${size#*x}
  for r in $(seq $ROUNDS); do
    for tree in new old; do
      dir=$R; [ $tree = old ] && dir=$OLD
      out=$(cd $dir && timeout -k 10 120 python bench.py --scene $name --width $w --height $h --steps $STEPS --warmup 20 --no-cpu-baseline 2>/dev/null | grep '^{')
      rc=$?
      if [ $rc -ne 0 ]; then echo "$tree $name FAILED rc=$rc"; exit 1; fi
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tree', '$name', '$size', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'ms_per_step %.4f' % d['ms_per_step'], 'cold', d.get('cold_kernel_ms'))"
    done
  done
done
