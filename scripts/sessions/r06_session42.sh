set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/region_inflight_probe.py 5 > gpurun_out/r06_region_inflight2.jsonl 2> gpurun_out/r06_region_inflight2.err || { tail -5 gpurun_out/r06_region_inflight2.err; exit 1; }
cat gpurun_out/r06_region_inflight2.jsonl
