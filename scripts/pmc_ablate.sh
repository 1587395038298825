#!/bin/bash
# Instruction counts of the direct kernel per ablation (flags 4: camera ray
# only; 2: closest hit only; 0: full) — one PMC pass each.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for f in 4 2 0; do
  PMC_NAME=pmc_ablate_f$f BENCH_ARGS="--flags $f" bash $R/scripts/pmc.sh \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" || exit 1
  echo "flags=$f $(python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_ablate_f$f | tr -d '\n ')"
done
