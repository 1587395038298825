#!/bin/bash
# PMC breakdown of the pool kernel (one scene; --pmc passes with --kernel-trace only).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export PMC_NAME=${PMC_NAME:-pmc_pool}
export BENCH_ARGS=${BENCH_ARGS:-"--scene reflect_refract"}
bash $R/scripts/pmc.sh \
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES" \
 "SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
python3 $R/scripts/pmc_summary.py $R/gpurun_out/$PMC_NAME
