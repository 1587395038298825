#!/bin/bash
# PMC passes over the whole 4K frame and its 8 shards on one GPU, for cover
# and table (scripts/shard_pmc_run.py, one rocprofv3 run per counter group,
# --kernel-trace only) -> gpurun_out/shard_pmc/<scene>_<n>.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/shard_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ROUNDS=${ROUNDS:-5}
for sc in ${SCENES:-cover table}; do
  for n in 1 8; do
    D=$OUT/${sc}_$n
    i=0
    for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES"; do
      i=$((i+1))
      timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d $D/p$i -o run --output-format csv -- \
        python3 $R/scripts/shard_pmc_run.py $sc $n 3840 2160 $ROUNDS > $D.p$i.log 2>&1 || { echo "pmc $sc $n pass $i failed"; tail -5 $D.p$i.log; exit 1; }
    done
    python3 $R/scripts/shard_pmc_summary.py $D $n $ROUNDS > $D.json && echo "$sc $n: $(cat $D.json | head -c 600)"

  done
done
