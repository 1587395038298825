#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no --pmc here), after
# the bench's own warm-up to steady clocks (its 200 ms default).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $R/bench.py --steps ${PROF_STEPS:-200} --warmup 10 --no-cpu-baseline --ab --mode frames --inflight 1 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -h '^{' $OUT/bench.log | cut -c1-600
cut -d, -f1-5 $OUT/run_kernel_stats.csv 2>/dev/null | head -6
exit $rc
