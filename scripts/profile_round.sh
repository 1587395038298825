#!/bin/bash
# Round profile set: rocprofv3 kernel-trace stats of the bench line of each
# BASELINE scene (three_sphere and reflect_refract at 1080p, cover and table
# at 4K on one GPU), then PMC passes (HBM bytes + SQ counters) for each:
# FETCH, WRITE, issue/wait, instruction mix, and two attribution passes
# (wait classes, memory-level occupancy: scripts/pmc_summary.py).
# --pmc runs use --kernel-trace only, one counter group per run.  Output:
# gpurun_out/$ROUND_*; scripts/collect_profiles.py turns it into profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUND=${ROUND:-r02}
cd $R
declare -A ARGS=([three_sphere]="" [reflect_refract]="--scene reflect_refract"
                 [cover]="--scene cover --width 3840 --height 2160" [table]="--scene table --width 3840 --height 2160")
for k in ${SCENES:-three_sphere reflect_refract cover table}; do
  PROF_NAME=${ROUND}_stats_$k BENCH_ARGS="${ARGS[$k]}" bash scripts/gpu_prof.sh || exit $?
  PMC_NAME=${ROUND}_pmc_$k BENCH_ARGS="${ARGS[$k]}" bash scripts/pmc.sh "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES" \
    "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
    "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT" || exit $?
done
echo "profile set done"
