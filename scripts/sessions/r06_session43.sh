set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 200 python -u scripts/region_inflight_probe.py 15 >> gpurun_out/r06_region_inflight3.jsonl 2> gpurun_out/r06_region_inflight3.err || { tail -5 gpurun_out/r06_region_inflight3.err; exit 1; }; done
cat gpurun_out/r06_region_inflight3.jsonl
