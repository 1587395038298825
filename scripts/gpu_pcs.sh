#!/bin/bash
# PC sampling (host_trap, time) of the headline frame's per-scene direct kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pcs/avail.txt 2>&1 || true
grep -i -A3 "pc" gpurun_out/pcs/avail.txt | head -40
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs -o pcs --output-format csv -- python bench.py --steps 3000 --warmup 50 --no-cpu-baseline > gpurun_out/pcs/run.log 2>&1
rc=$?; echo "pcs rc=$rc"; tail -5 gpurun_out/pcs/run.log
find gpurun_out/pcs -name "*.csv" | head
