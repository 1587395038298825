#!/bin/bash
# Per-workgroup timelines (RT_FLAG_STAMPS) of the direct kernel on the
# headline frame: full, camera-only (flags 4), camera-only with u8 output.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for args in "--flags 0" "--flags 4" "--flags 4 --out u8" "--flags 0 --out u8" "--flags 2"; do
  timeout -k 10 60 python scripts/stamps.py $args 2>/dev/null | grep '^{' || exit 1
done
for args in "--flags 0" "--flags 4"; do
  RTC_SCHED_DIRECT=grid timeout -k 10 60 python scripts/stamps.py $args 2>/dev/null | grep '^{' || exit 1
done
