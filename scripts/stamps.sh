#!/bin/bash
# Per-workgroup timelines (RT_FLAG_STAMPS) of the headline frame and a pool scene.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for args in "--flags 0" "--flags 4" "--flags 2" "--scene shadow_puppets" "--scene reflect_refract" "--scene cover"; do
  timeout -k 10 60 python scripts/stamps.py $args 2>/dev/null | grep '^{' || exit 1
done
