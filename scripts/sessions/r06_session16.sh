set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
WORKLOADS="--steps 1000" ROUNDS=2 bash scripts/ab_knobs.sh "o25=" "o10=direct_oversub=10" "o15=direct_oversub=15" "o40=direct_oversub=40" "o60=direct_oversub=60" > gpurun_out/r06_ab_oversub.jsonl 2>&1; echo "rc=$?"; cat gpurun_out/r06_ab_oversub.jsonl
