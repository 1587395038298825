#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for s in grid static; do
  for f in 0 1 5; do
    RTC_SCHED_DIRECT=$s timeout -k 10 60 python scripts/stamps.py --flags $f 2>/dev/null | grep '^{'
  done
done
RTC_SCHED_POOL=dynamic timeout -k 10 60 python scripts/stamps.py --scene reflect_refract 2>/dev/null | grep '^{'
