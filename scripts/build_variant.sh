#!/bin/bash
# Build the render library of git revision REV (default HEAD) with extra
# compiler flags into ray-tracer-challenge-rs_amd/rtc_amd/_lib_NAME/, for
# same-box A/B runs (scripts/ab_builds.sh).  CPU-only.
# REV "WORKTREE" builds the current working tree (uncommitted edits).
# Usage: build_variant.sh NAME [REV] [EXTRA_FLAGS]
set -eu
NAME=$1; REV=${2:-HEAD}; EXTRA=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rtc_variant_XXXX)
if [ "$REV" = WORKTREE ]; then
  mkdir -p $T/ray-tracer-challenge-rs_amd
  cp -r $R/include $T/ && cp -r $R/ray-tracer-challenge-rs_amd/csrc $R/ray-tracer-challenge-rs_amd/tools $R/ray-tracer-challenge-rs_amd/Makefile $T/ray-tracer-challenge-rs_amd/
else
  (cd $R && git archive "$REV" ray-tracer-challenge-rs_amd include) | tar -x -C $T
fi
make -s -C $T/ray-tracer-challenge-rs_amd OUT=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib_$NAME EXTRA="$EXTRA" -j8
rm -rf $T
echo "built $NAME from $REV -> rtc_amd/_lib_$NAME"
