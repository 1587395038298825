#!/bin/bash
# Final round-3 check on HEAD: full pytest -m gpu, smoke, bench (default line + f64 line)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS="-v --timeout 120 --timeout-method thread" PYTEST_TIMEOUT=600 bash scripts/gpu_check.sh
