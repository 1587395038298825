#!/bin/bash
# Pool-kernel check on one MI355X: the GPU suite, then short A/B bench lines
# (kernel ms) of the pool scenes.  Usage: scripts/pool_check.sh [tag] [pytest args]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
TAG=${1:-pool}; shift || true
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest.log
fi
OUT=gpurun_out/${TAG}_bench.jsonl; : > $OUT
b() { timeout -k 10 180 python bench.py --ab --no-cpu-baseline "$@" 2>gpurun_out/${TAG}_bench.err | grep '^{' >> $OUT || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('$OUT').read().splitlines()[-1]); print(d['config'].get('workload'), 'ms', round(d['ms_per_step'],4), 'kernel_ms', d['roofline'].get('kernel_ms'), 'frac', d['roofline'].get('frac'))"; }
b --scene reflect_refract --steps 200
b --scene cover --width 3840 --height 2160 --steps 100 --warmup 10
b --scene table --width 3840 --height 2160 --steps 100 --warmup 10
b --steps 200
