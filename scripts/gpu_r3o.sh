#!/bin/bash
# Shard-tail diagnostics: stamps + recorded tile costs per shard (scripts/shard_tail.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in "cover 3840 2160 8 0,3" "table 3840 2160 8 0,5" "cover 3840 2160 1 0" "reflect_refract 1920 1080 4 0" "reflect_refract 1920 1080 1 0"; do
  timeout -k 10 120 python scripts/shard_tail.py $a 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/shard_tail.log || exit 1
done
