set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/random_world_bisect.py 5 > gpurun_out/r06_bisect5.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r06_bisect5.log | head -4; [ $rc -eq 0 ] || exit $rc
RTC_DEBUG=cull=0 timeout -k 10 300 python -u scripts/random_world_bisect.py 5 > gpurun_out/r06_bisect5b.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r06_bisect5b.log; exit $rc
