#!/bin/bash
# Round profile set: rocprofv3 kernel-trace stats of the default bench line
# and of a pool-kernel scene, then PMC passes (HBM bytes + SQ counters) for
# both.  --pmc runs use --kernel-trace only.  Output: gpurun_out/$ROUND_*;
# scripts/collect_profiles.py turns it into profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUND=${ROUND:-r01}
cd $R
PROF_NAME=${ROUND}_stats_three_sphere bash scripts/gpu_prof.sh || exit $?
PROF_NAME=${ROUND}_stats_reflect_refract BENCH_ARGS="--scene reflect_refract" bash scripts/gpu_prof.sh || exit $?
PMC_NAME=${ROUND}_pmc_three_sphere bash scripts/pmc.sh "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES" \
  "GRBM_GUI_ACTIVE SQ_LEVEL_WAVES SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM" || exit $?
PMC_NAME=${ROUND}_pmc_reflect_refract BENCH_ARGS="--scene reflect_refract" bash scripts/pmc.sh "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES" || exit $?
echo "profile set done"
