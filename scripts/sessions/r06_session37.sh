set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/random_world_sweep.py > gpurun_out/r06_sweep37.jsonl 2> gpurun_out/r06_sweep37.err; rc=$?; echo "rc=$rc"; grep -v '"ok": true' gpurun_out/r06_sweep37.jsonl | head -20; grep -c '"jit_used": true' gpurun_out/r06_sweep37.jsonl; tail -3 gpurun_out/r06_sweep37.err | grep -v amdgpu.ids; exit $rc
