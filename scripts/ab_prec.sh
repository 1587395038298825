#!/bin/bash
# A/B of this tree against $OLD (default ab_old/) at one precision:
# ab_prec.sh <f32|f64> "<scene[:WxH]> ..." [rounds]; prints kernel ms per run.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OLD=${OLD:-$R/ab_old}
PREC=$1; SCENES=$2; ROUNDS=${3:-2}
for sc in $SCENES; do
  name=${sc%%:*}; size=${sc#*:}; [ "$size" = "$sc" ] && size=1920x1080
  for r in $(seq $ROUNDS); do
    for tree in new old; do
      dir=$R; [ $tree = old ] && dir=$OLD
      out=$(cd $dir && timeout -k 10 120 python bench.py --scene $name --width ${size%x*} --height ${size#*x} --precision $PREC --steps ${AB_STEPS:-200} --warmup 20 --no-cpu-baseline 2>/dev/null | grep '^{') || { echo "$tree $name FAILED"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tree', '$name', '$size', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'])"
    done
  done
done
