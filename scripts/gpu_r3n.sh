#!/bin/bash
# (historical: RTC_OVERLAP was measured, rejected and removed from the tree)
# (1) overlapped-items pool kernel (RTC_OVERLAP build _lib_ov): smoke frame, parity/exactness tests, A/B
# (2) cold-launch probe sweep; (3) direct-kernel PMC ablation
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
source scripts/ab_lib.sh
L=$PWD/ray-tracer-challenge-rs_amd/rtc_amd
export RTC_JIT_CACHE=0
RTC_LIBRARY=$L/_lib_ov/librtc.so timeout -k 10 60 python bench.py --scene reflect_refract --width 320 --height 200 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ov_smoke.log 2>&1 || { echo "ov smoke failed rc=$?"; tail -20 gpurun_out/ov_smoke.log; exit 1; }
echo "ov smoke ok"
RTC_LIBRARY=$L/_lib_ov/librtc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ov_tests.log 2>&1
rc=$?; echo "ov tests rc=$rc"; tail -5 gpurun_out/ov_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in _lib _lib_ov; do
  for sc in cover table; do
    echo "$v"; RTC_LIBRARY=$L/$v/librtc.so SHARD_COUNTS=8 timeout -k 10 120 python scripts/shard_times.py $sc 3840 2160 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for r in 1 2; do
  for v in _lib _lib_ov; do
    for sc in reflect_refract:1920:1080 refraction:1920:1080 cylinders:1920:1080 metal:1920:1080 cover:3840:2160 table:3840:2160; do
      IFS=: read n w h <<< "$sc"
      run "$v $n" env RTC_LIBRARY=$L/$v/librtc.so python bench.py --scene $n --width $w --height $h --steps 200 --warmup 10 --no-cpu-baseline || exit 1
    done
  done
done
AB_STEPS=100 bash scripts/ab_env.sh "reflect_refract refraction cylinders metal cover:3840x2160 table:3840x2160" "RTC_COLD_PROBE=0" "RTC_COLD_PROBE=8,24" "RTC_COLD_PROBE=4,12" "RTC_COLD_PROBE=16,48" "RTC_COLD_PROBE=8,24,1" || exit 1
bash scripts/pmc_ablate.sh || exit 1
