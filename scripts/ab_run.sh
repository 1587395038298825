#!/bin/bash
# One-off A/B session: GPU parity tests, then variants x scenes x knobs.
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
AB_STEPS=${AB_STEPS:-1000} bash scripts/ab_builds.sh "$AB_VARIANTS" "$AB_SCENES" 
