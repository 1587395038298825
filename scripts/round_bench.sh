#!/bin/bash
# Round bench lines (profiles/<round>_bench_lines.jsonl): the default bench
# line (BASELINE configs[1]), the other BASELINE scenes on one GPU, the f64
# parity path, and the N > 1 default (configs[3] tiled) with one rank.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R; mkdir -p gpurun_out
OUT=gpurun_out/${ROUND:-r02}_bench_lines.jsonl; : > $OUT
b() { timeout -k 10 240 python bench.py "$@" 2>/dev/null | grep '^{' >> $OUT || exit 1; tail -1 $OUT | cut -c1-300; }
b --cpu-seconds 12
b --scene reflect_refract --cpu-seconds 12
b --scene cover --width 3840 --height 2160 --steps 300 --warmup 10 --cpu-seconds 12
b --scene table --width 3840 --height 2160 --steps 300 --warmup 10 --cpu-seconds 12
b --precision f64 --steps 300 --no-cpu-baseline
b --mode tiled --steps 300 --warmup 10 --no-cpu-baseline
