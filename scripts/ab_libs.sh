#!/bin/bash
# Same-box A/B of library builds (kernel ms and cold first launch per scene,
# two alternating rounds): builds under ray-tracer-challenge-rs_amd/rtc_amd/,
# made with scripts/build_variant.sh NAME [REV], picked through RTC_LIBRARY.
#   VARIANTS="_lib_base _lib" SCENES="rr cover table" bash scripts/ab_libs.sh   (on a GPU box)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
b() { local tag=$1; shift; timeout -k 10 60 python bench.py --ab --mode frames --no-cpu-baseline "$@" 2>gpurun_out/ab.err | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['config']['workload'][:22], round(d['roofline']['kernel_ms'],4), 'cold', round(d.get('cold_kernel_ms') or 0,4))" || { tail -3 gpurun_out/ab.err; return 1; }; }
for r in 1 2; do
for v in ${VARIANTS:-_lib_base _lib}; do
  export RTC_LIBRARY=$GRAFT_REPO_ROOT/ray-tracer-challenge-rs_amd/rtc_amd/$v/librtc.so
  for sc in ${SCENES:-rr cover table}; do
    case $sc in
      rr) b "$v rr" --scene reflect_refract --steps 200 || exit 1;;
      refraction) b "$v refraction" --scene refraction --steps 200 || exit 1;;
      metal) b "$v metal" --scene metal --steps 200 || exit 1;;
      cylinders) b "$v cylinders" --scene cylinders --steps 200 || exit 1;;
      cover) b "$v cover" --scene cover --width 3840 --height 2160 --steps 60 --warmup 10 || exit 1;;
      table) b "$v table" --scene table --width 3840 --height 2160 --steps 60 --warmup 10 || exit 1;;
      three) b "$v three" --steps 300 || exit 1;;
    esac
  done
done
done
