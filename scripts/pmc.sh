#!/bin/bash
# PMC counter passes (separate rocprofv3 runs; --pmc only with --kernel-trace/--stats).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PMC_NAME:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "${@}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --warmup-ms 0 --no-cpu-baseline --ab --mode frames --inflight 1 ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1 || exit $?
  echo "pass $i ($ctrs) ok"
done
