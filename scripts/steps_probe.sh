#!/bin/bash
# Bench value against steps/warmup on one box: the driver's short run
# (--steps 20 --warmup 5) next to long ones, to see the fixed costs of a
# short timed region (launch latency, final sync, clock ramp).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/steps_probe.jsonl; : > $OUT
b() { timeout -k 10 120 python bench.py --no-cpu-baseline "$@" 2>/dev/null | grep '^{' >> $OUT || exit 1
      python -c "import json,sys; d=json.loads(open('$OUT').readlines()[-1]); print('$*', round(d['value']), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))"; }
b --steps 20 --warmup 5 --warmup-ms 0
b --steps 20 --warmup 5
b --steps 20 --warmup 5
b --steps 1000 --warmup 50
b --steps 20 --warmup 5
b --scene reflect_refract --steps 20 --warmup 5
