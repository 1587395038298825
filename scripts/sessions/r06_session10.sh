set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="_lib_pre _lib" SCENES="rr cover table" bash scripts/ab_libs.sh > gpurun_out/r06_ab_pre.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/r06_ab_pre.txt
for v in _lib_pre _lib; do echo "== $v"; RTC_LIBRARY=$PWD/ray-tracer-challenge-rs_amd/rtc_amd/$v/librtc.so SHARD_COUNTS=1,8 timeout -k 10 200 python scripts/shard_times.py cover 3840 2160 || exit 1; done 2>&1 | grep -v amdgpu.ids
