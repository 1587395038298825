#!/bin/bash
# A/B of environment knobs on one build: ab_env.sh "<scene[:WxH]> ..." "<env assignments>" "<env assignments>" ...
# (use X=0 for the default); prints the kernel ms of each run, 2 rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
SCENES=$1; shift
for r in 1 2; do
  for sc in $SCENES; do
    name=${sc%%:*}; size=${sc#*:}; [ "$size" = "$sc" ] && size=1920x1080
    for e in "$@"; do
      out=$(env $e timeout -k 10 120 python bench.py --scene $name --width ${size%x*} --height ${size#*x} --steps ${AB_STEPS:-400} --warmup 20 --no-cpu-baseline --ab 2>/dev/null | grep '^{') || { echo "$e $name FAILED"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$e]', '$name', '$size', 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'cold', d.get('cold_kernel_ms'))"
    done
  done
done
