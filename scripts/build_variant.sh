#!/bin/bash
# Build the render library of git revision REV (default HEAD) with extra
# compiler flags into ray-tracer-challenge-rs_amd/rtc_amd/_lib_NAME/, for
# same-box A/B runs (scripts/ab_builds.sh).  CPU-only.
# Usage: build_variant.sh NAME [REV] [EXTRA_FLAGS]
set -eu
NAME=$1; REV=${2:-HEAD}; EXTRA=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rtc_variant_XXXX)
(cd $R && git archive "$REV" ray-tracer-challenge-rs_amd include) | tar -x -C $T
make -s -C $T/ray-tracer-challenge-rs_amd OUT=$R/ray-tracer-challenge-rs_amd/rtc_amd/_lib_$NAME EXTRA="$EXTRA" -j8
rm -rf $T
echo "built $NAME from $REV -> rtc_amd/_lib_$NAME"
