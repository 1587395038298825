#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for kd in 0 1; do
 for st in 1 0; do
  for s in grid static; do
   for f in 0 5; do
    echo -n "kernarg_dev=$kd staged=$st "
    HIP_FORCE_DEV_KERNARG=$kd RTC_STAGED_STORE=$st RTC_SCHED_DIRECT=$s timeout -k 10 60 python scripts/stamps.py --flags $f 2>/dev/null | grep '^{'
   done
  done
 done
done
